// Implicit-GEMM conv variants of tile group 3 (tiles 12-15); see conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group3(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 12: return launch_cfg<64, 32, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 13: return launch_cfg<128, 32, 128, 4, 1>(a, is1x1, a_f32, pro, epi, st);
    case 14: return launch_cfg<64, 64, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 15: return launch_cfg<64, 128, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
