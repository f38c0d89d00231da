#pragma once
#include "common.h"

namespace idc {

struct WgradArgs {
  const bf16_t* x;  // forward input (raw; BN+act re-applied via `pro`), channel slice, ld = ldx
  int N, H, W, Cin, ldx;
  const void* g;    // dY [M, ldg] (bf16 or fp32), channel slice
  int ldg;
  int Ho, Wo, Cout;
  int KH, KW, SH, SW, PT, PL;
  BnArgs pro;
  float* dw;        // [K][Cout] fp32 (Keras HWIO), accumulated atomically
  float scale;      // multiplies the contribution (1.0 normally)
  int cin_real;     // Keras Cin when the staged input is channel-padded (0: == Cin)
  int pix_per_split;
  // backward pending affine on G (common.h BwdAff; gpro.mode != 0 selects it): the staged
  // gradient is A*g + B*x + C, x read from gpro.x at the same pixel and output channel
  BwdAff gpro;
  // deterministic mode: with `part` set, pixel-slice z stores its partial dW (fp32, dW layout)
  // to part[z * numel(dW) + i] instead of adding atomically; wgrad_reduce then sums the slices
  // in a fixed order (csrc/kernels/conv_wgrad.hip)
  float* part;
  long long part_floats;  // capacity, checked at launch
};

__device__ __forceinline__ void gshift(WgradArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); a.g = gsh(a.g, o); gshift(a.pro, o); a.dw = gsh(a.dw, o); gshift(a.gpro, o);
  a.part = gsh(a.part, o);
}

// variant 0: the general kernel; 1..wgrad_num_variants()-1: the large-tile DMA kernel
// (wgrad_big.hip) where wgrad_big_ok holds, else the general kernel
hipError_t conv_wgrad(WgradArgs a, int splits, bool g_f32, hipStream_t st, int variant = 0);
hipError_t wgrad_big(WgradArgs a, int splits, bool g_f32, int variant, hipStream_t st);
bool wgrad_big_ok(const WgradArgs& a, bool g_f32, int variant);
int wgrad_big_pick_splits(int M, int K, int Cout, int variant);
int wgrad_num_variants();
int wgrad_variant_bp(int variant);
// dw[i] += sum_{z < splits} part[z * n + i], in slice order
hipError_t wgrad_reduce(const float* part, float* dw, long long n, int splits, hipStream_t st);
int wgrad_effective_splits(const WgradArgs& a, int splits, int variant = 0);
// the image-resident stem weight gradient (wgrad_stem.hip): 8-channel staged images, KxK stride
// 1/2, <= 64 outputs; with IDC_WGRAD_STEM=1 conv_wgrad takes it whenever it applies (opt-in)
bool wgrad_stem_ok(const WgradArgs& a, bool g_f32);
hipError_t wgrad_stem(const WgradArgs& a, hipStream_t st);
int wgrad_stem_slices(const WgradArgs& a);
int wgrad_pick_splits(int M, int K, int Cout);

// ---- batched weight gradients -----------------------------------------------------------------
// Many independent weight gradients with the same kernel shape in ONE launch (DenseNet's
// late-stage dense layers: dozens of small wgrads whose operands are final once the stage's
// data-gradient chain has run).  Workgroup b of the 1-D grid runs tile (b - begin[m]) of member
// m = #{begin <= b} - 1, found with one ballot over the <= 64 member begins.
constexpr int WG_BATCH_MAX = 64;
struct WgBatchEntry {
  WgradArgs a;       // pix_per_split resolved
  int gx, gy, gz;    // the member's own grid (general: k tiles, cout tiles, pixel slices;
                     // halo: image groups, 64-channel blocks, 1)
  int ipw;           // halo kernel: images per workgroup
};
// batch signature of one member (members of one launch must share it), -1: not batchable
int wgrad_batch_sig(const WgradArgs& a, bool g_f32, int variant);
// fill entry `e` for a member launched with `splits`; returns its workgroup count, `smem` = its
// LDS bytes
int wgrad_batch_entry(const WgradArgs& a, int splits, WgBatchEntry& e, long long& smem);
// dev_entries / dev_begins: device copies (begins padded with INT_MAX to WG_BATCH_MAX)
hipError_t wgrad_batch(const WgBatchEntry* dev_entries, const int* dev_begins, int n, int total, int sig,
                       long long smem, hipStream_t st);

}  // namespace idc
