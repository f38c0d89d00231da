#pragma once
#include "common.h"

namespace idc {

// One MobileNetV2 inverted-residual block in INFERENCE mode (every BatchNorm a constant affine from
// its moving statistics): expand 1x1 -> BN -> ReLU6 -> depthwise 3x3 -> BN -> ReLU6 -> project 1x1
// -> BN (+ identity shortcut), as ONE launch (mb_infer.hip).  All activations NHWC bf16.
struct MbInferArgs {
  const bf16_t* x; int ldx;     // block input [N, H, W, Cin], raw
  int ldres;
  BnArgs xbn;                   // x's pending BatchNorm + activation (mode 0 + act 0: identity)
  const bf16_t* res;            // nullable: added after xbn (the previous block's shortcut)
  const bf16_t* we;             // expand kernel bf16 [Cexp][Cin]; null: no expand (Cexp == Cin)
  BnArgs ebn;                   // expand BN + ReLU6
  const float* wd;              // depthwise kernel, fp32 Keras layout (3, 3, Cexp, 1)
  BnArgs dbn;                   // depthwise BN + ReLU6
  const bf16_t* wp;             // project kernel bf16 [Cout][Cexp]
  BnArgs pbn;                   // project BN (linear)
  bf16_t* y; int ldy;           // output [N, Ho, Wo, Cout] = pbn(project) (+ x_eff)
  int N, H, W, Cin, Cexp, Cout, Ho, Wo, S, PT, PL;
  int residual;                 // 1: y += act(xbn(x)) + res (stride 1, Cin == Cout)
  int ipg;                      // whole images per workgroup
  int cs;                       // expanded channels per workgroup (multiple of MBI_CC); the
                                // ceil(Cexp / cs) workgroups of an image group reduce their
                                // project partials through `slab` (last arriver: `tickets`)
  float* slab;                  // >= mb_infer_slab_floats() fp32 (cs < Cexp only)
  unsigned* tickets;            // one counter per image group, any start value (counts modulo)
};

constexpr int MBI_CC = 32;        // expanded channels per chunk (one MFMA K step of the project)
constexpr int MBI_NT = 512;       // threads per workgroup (8 waves, 2 per SIMD)
constexpr int MBI_MAX_ACC = 10;   // project accumulator tiles per wave (16 x 16 fp32 each)
constexpr int MBI_MAX_KX = 192;   // padded input channels (expand K)

// Dynamic LDS bytes of a launch, or -1 when the shape is outside the kernel's limits.
long long mb_infer_smem(const MbInferArgs& a);
long long mb_infer_slab_floats(const MbInferArgs& a);
hipError_t mb_infer(const MbInferArgs& a, hipStream_t st);

}  // namespace idc
