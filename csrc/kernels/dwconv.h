#pragma once
#include "common.h"

namespace idc {

// Depthwise KxK conv (depth multiplier 1), NHWC bf16, Keras kernel layout (KH,KW,C,1) fp32.
struct DwArgs {
  const bf16_t* x; int ldx;     // forward input (raw; pending BN+act via `pro`)
  int N, H, W, C;
  BnArgs pro;
  const float* w;               // (KH,KW,C) fp32 master
  int KH, KW, S, PT, PL, Ho, Wo;
  // fwd: y raw output + stats
  bf16_t* y; int ldy;
  float* stats; int stats_ld;
  // bwd data: dy -> dx (dZ through the pending BN+act; sums into gsum/gsumx)
  const bf16_t* dy; int lddy;
  bf16_t* dx; int lddx;
  float* gsum; float* gsumx;
  // wgrad: dw += sum over pixels; with a workspace (ws, >= dwconv_wgrad_ws_floats() floats)
  // the reduction is two-stage (per-block partials + column sums) instead of global atomics
  float* dw;
  float* ws;
  int stats_slots, gsum_slots, gsum_ld;  // statistics slots (common.h)
  // bwd data / wgrad (3x3 only): dy is staged through the pending backward of the BatchNorm that
  // follows this depthwise conv (common.h BwdAff; x = the raw depthwise output at dy's positions)
  BwdAff dyaff;
  // fwd statistics shift per channel (nullable, common.h "Shifted statistics")
  const float* stats_shift;
};

__device__ __forceinline__ void gshift(DwArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); gshift(a.pro, o); a.w = gsh(a.w, o); a.y = gsh(a.y, o); a.stats = gsh(a.stats, o);
  a.dy = gsh(a.dy, o); a.dx = gsh(a.dx, o); a.gsum = gsh(a.gsum, o); a.gsumx = gsh(a.gsumx, o);
  a.dw = gsh(a.dw, o); a.ws = gsh(a.ws, o); gshift(a.dyaff, o); a.stats_shift = gsh(a.stats_shift, o);
}

long long dwconv_wgrad_ws_floats(long long M, int C, int taps);

hipError_t dwconv_fwd(const DwArgs& a, hipStream_t st);
hipError_t dwconv_bwd_data(const DwArgs& a, hipStream_t st);
hipError_t dwconv_wgrad(const DwArgs& a, hipStream_t st);
// stride-1 3x3: data + weight gradients in one pass (dx, gsum/gsumx as dwconv_bwd_data; the weight
// gradient's per-block partials into ws), then dwconv_wgrad_sum folds ws into dw
bool dwconv_bwd_fused_ok(const DwArgs& a);
hipError_t dwconv_bwd_fused(const DwArgs& a, hipStream_t st);
hipError_t dwconv_wgrad_sum(const DwArgs& a, hipStream_t st);

}  // namespace idc
