#pragma once
#include "common.h"

namespace idc {

// Flatten -> Dropout(p0) -> Dense(D0->D1, relu) -> Dropout(p1) -> Dense(D1->U) -> BCE / softmax-CE:
// the tiny-CNN head of secure_fed_model.py:90-95, fused (one workgroup per sample).  Dropout masks
// are counter-based Philox4x32-10 keyed by (seed, step[0]) and counted by (sample, layer, index),
// so forward and backward of a step regenerate the same masks without storing them, and every
// replay of a captured graph draws fresh ones once `step` is advanced (op kind MLP_STEP).
struct Mlp2Args {
  const bf16_t* x;        // [N][D0] (NHWC flatten of the pooled conv output)
  int N, D0, D1, U;
  const float* w1;        // [D0][D1] Keras Dense kernel (fp32 master)
  const float* b1;        // [D1]
  const float* w2;        // [D1][U]
  const float* b2;        // [U]
  float p0, p1;           // dropout rates (training only)
  unsigned long long seed;
  const unsigned int* step;  // device counter (dropout stream)
  const float* labels;    // [N] or [N][U]
  float* logits;          // [N][U]
  float* h1;              // [N][D1] post-relu, pre-dropout activations (saved for backward)
  float* loss;            // += mean loss
  float* dlogits;         // [N][U]
  float loss_scale;
  int training;
  // backward
  float* dw1; float* db1; float* dw2; float* db2;
  float* dx;              // [N][D0] fp32 gradient of the flattened input (may be null)
  float dl_scale;         // dlogits factor (loss_scale x the rank's uneven-batch weight)
};

__device__ __forceinline__ void gshift(Mlp2Args& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); a.w1 = gsh(a.w1, o); a.b1 = gsh(a.b1, o); a.w2 = gsh(a.w2, o); a.b2 = gsh(a.b2, o);
  a.step = gsh(a.step, o); a.labels = gsh(a.labels, o); a.logits = gsh(a.logits, o); a.h1 = gsh(a.h1, o);
  a.loss = gsh(a.loss, o); a.dlogits = gsh(a.dlogits, o); a.dw1 = gsh(a.dw1, o); a.db1 = gsh(a.db1, o);
  a.dw2 = gsh(a.dw2, o); a.db2 = gsh(a.db2, o); a.dx = gsh(a.dx, o);
}

hipError_t mlp2_fwd(const Mlp2Args& a, hipStream_t st);
hipError_t mlp2_bwd(const Mlp2Args& a, hipStream_t st);
hipError_t mlp2_step(unsigned int* step, hipStream_t st);

}  // namespace idc
