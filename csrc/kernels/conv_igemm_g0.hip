// Implicit-GEMM conv variants of tile group 0 (tiles 0-3); see conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group0(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 0: return launch_cfg<128, 128, 32, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 1: return launch_cfg<128, 64, 32, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 2: return launch_cfg<256, 32, 32, 4, 1>(a, is1x1, a_f32, pro, epi, st);
    case 3: return launch_cfg<64, 64, 32, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
