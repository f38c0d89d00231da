// Implicit-GEMM conv variants of tile group 4 (tiles 16-18); see conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group4(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 16: return launch_cfg<128, 64, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 17: return launch_cfg<64, 32, 256, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 18: return launch_cfg<64, 64, 256, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
