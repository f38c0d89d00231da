// Implicit-GEMM conv variants of tile group 2 (tiles 8-11); see conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group2(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 8: return launch_cfg<64, 64, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 9: return launch_cfg<64, 32, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 10: return launch_cfg<256, 32, 64, 4, 1>(a, is1x1, a_f32, pro, epi, st);
    case 11: return launch_cfg<64, 128, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
