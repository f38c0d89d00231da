// Implicit-GEMM conv variants of tile group 1 (tiles 4-7); see conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group1(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 4: return launch_cfg<64, 32, 32, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 5: return launch_cfg<128, 128, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 6: return launch_cfg<128, 64, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 7: return launch_cfg<128, 32, 64, 4, 1>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
