// Implicit-GEMM conv variants of tile group 5 (tiles 19-22): 32-row tiles.  The small-M layers
// (DenseNet stages 3-4, VGG block 5) are bound by what one CU can pull per K-step (~10 B/clk at
// one 4-wave workgroup per CU): halving the rows of a tile halves each workgroup's bytes and
// doubles the workgroups, so 2x more CUs share the layer's operand traffic.  See conv_igemm_impl.h.
#include "conv_igemm_impl.h"

namespace idc {

hipError_t conv_igemm_group5(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st) {
  switch (tile) {
    case 19: return launch_cfg<32, 32, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 20: return launch_cfg<32, 32, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 21: return launch_cfg<32, 64, 64, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    case 22: return launch_cfg<32, 64, 128, 2, 2>(a, is1x1, a_f32, pro, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
