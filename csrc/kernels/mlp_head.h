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
};

hipError_t mlp2_fwd(const Mlp2Args& a, hipStream_t st);
hipError_t mlp2_bwd(const Mlp2Args& a, hipStream_t st);
hipError_t mlp2_step(unsigned int* step, hipStream_t st);

}  // namespace idc
