// Large-tile weight gradient for the wide, plain layers (VGG16 blocks 2-5), gfx950.
//
//   dW[k, co] = sum_m A[m, k] * G[m, co]     k = (r, s, c) Keras HWIO rows, m = output pixel
//
// The general wgrad kernel (conv_wgrad.hip) stages both operands through VGPRs (it re-applies a
// pending BN to A) in 64x128 tiles of 32-pixel steps: on VGG16's layers (K up to 4608, Cout up to
// 512, no BN) it ran at ~9 % of the MFMA peak, each 32-pixel step one global-load round trip for
// 8 MFMAs per wave.  Here, in the manner of conv_big.hip:
//
//   * 256 (k) x BC (co) tiles, BC = 128 / 256, 8 waves as 4 (k) x 2 (co): each wave a 64 x BC/2
//     sub-tile of v_mfma_f32_32x32x16_bf16 accumulators (2 x BC/64 of them);
//   * both operands go global -> LDS with global_load_lds_dwordx4 (no VGPR staging), BP pixels
//     per step, NBUF buffers, one barrier per step (NBUF - 1 steps in flight, counted vmcnt);
//     A rows are one im2col row each: lane-chunk c of a row is 8 input channels of ONE tap
//     (Cin % 64 == 0), fixed per lane for the whole pixel loop; pixels outside the image, past
//     the slice or past K load a 16-B zero block;
//   * the pixel index is the MFMA k dimension but both operands arrive pixel-major, so they are
//     read transposed out of LDS with ds_read_b64_tr_b16; the chunk XOR swizzle (c ^ 4*(row&3))
//     makes those reads conflict-free (each 32-lane half reads 4 rows x 64 B), and is applied to
//     the DMA SOURCE address (the LDS side of global_load_lds is lane-linear);
//   * 32x32x16 rather than 16x16x32: the accumulator register r of a 32x32 tile is two 128-B row
//     segments, the shape the memory-side float atomics take at full rate (MI355X_MICROARCH.md
//     "Global float atomics"), so the split-K partial tiles are added straight from the
//     accumulators into dW — no LDS staging pass (the 16x16 layout would give 4 x 64 B);
//   * deterministic mode (`part`): plain stores of the slice's partial instead of atomics.
// Reference hot loop: the Conv2D weight gradients of dist_model_tf_vgg.py:119-138 (VGG16 DP).
#include "common.h"
#include "conv_wgrad.h"

namespace idc {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_wgz[8];  // zero source for padding / tails

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4bf lds_v4bf;

template <int BC_, int BP_, int NBUF_>
struct WbCfg {
  static_assert(NBUF_ >= 2 && NBUF_ <= 3, "the vmcnt ladder covers one step ahead of the waited one");
  static constexpr int BKR = 256, BC = BC_, BP = BP_, NBUF = NBUF_;
  static constexpr int WM = 4, WN = 2, NW = 8, NT = 512;
  static constexpr int WTM = BKR / WM, WTN = BC / WN;   // 64 x (64 | 128)
  static constexpr int TM = WTM / 32, TN = WTN / 32;    // 32x32 accumulators per wave
  static constexpr int AROWB = BKR * 2, GROWB = BC * 2; // bytes per LDS row (one pixel)
  static constexpr int A_BYTES = BP * AROWB, G_BYTES = BP * GROWB;
  static constexpr int BUF = A_BYTES + G_BYTES;
  static constexpr int LDS_BYTES = NBUF * BUF;
  static constexpr int ARPI = 1024 / AROWB, GRPI = 1024 / GROWB;  // rows per DMA wave-instruction
  static constexpr int NGA = BP / (ARPI * NW);  // DMA instructions per thread per step (A)
  static constexpr int NGG = BP / (GRPI * NW);  // (G)
  static_assert(NGA >= 1 && NGG >= 1, "pixel step too small for 8 waves");
};

// 256-B+ rows: each 32-lane half of a transposed fragment read touches 4 consecutive rows x 64 B
// (4 chunks) -> XOR the chunk with 4*(row & 3); 128-B rows (two per 256-B bank window) -> rows
// r and r+2 share a window, XOR with 4*((row >> 1) & 1)
template <int ROWB>
__device__ __forceinline__ int wb_swz(int row, int chunk) {
  if constexpr (ROWB >= 256) return chunk ^ ((row & 3) << 2);
  else return chunk ^ (((row >> 1) & 1) << 2);
}

// 32x32x16 MFMA operand (rows col_base..+31 of the dW / co axis, pixels r0..r0+15) read
// transposed from a [pixel][column] LDS image of ROWB bytes per row
template <int ROWB>
__device__ __forceinline__ v8bf wb_frag(const char* tile, int col_base, int lane, int r0) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  v8bf out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int row = r0 + 8 * (g >> 1) + 4 * t + q;
    const int col = col_base + 16 * (g & 1) + 4 * p;
    const int ch = col >> 3, sub = col & 7;
    const char* ptr = tile + row * ROWB + wb_swz<ROWB>(row, ch) * 16 + sub * 2;
    const v4bf v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(ptr));
    out[4 * t + 0] = v[0];
    out[4 * t + 1] = v[1];
    out[4 * t + 2] = v[2];
    out[4 * t + 3] = v[3];
  }
  return out;
}

// exact n / d for n * d < 2^41 (pixel indices < 2^21, divisors < 2^20)
struct FDiv {
  unsigned long long mul;
  int d;
  __device__ void init(int dd) {
    d = dd;
    mul = (1ull << 41) / (unsigned long long)dd + 1ull;
  }
  __device__ __forceinline__ int div(int n) const { return (int)(((unsigned long long)n * mul) >> 41); }
};

}  // namespace

template <int BC, int BP, int NBUF>
__global__ __launch_bounds__(512) void wgrad_big_kernel(WgradArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(WgradArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  using C = WbCfg<BC, BP, NBUF>;
  constexpr int NW = C::NW, TM = C::TM, TN = C::TN, NGA = C::NGA, NGG = C::NGG;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int wr = wid / C::WN, wc = wid % C::WN;
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.KH * a.KW * a.Cin;
  // 1-D grid, pixel-slice-major logical order remapped so that the workgroups of one slice
  // (every k tile and column tile: they read the same pixels of x and dY) share an XCD's L2
  const int gx = (K + C::BKR - 1) / C::BKR, gxy = gx * (a.Cout / BC);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int zslice = bid / gxy, rem = bid - zslice * gxy;
  const int k0 = (rem % gx) * C::BKR;
  const int c0 = (rem / gx) * BC;
  const int pbeg = zslice * a.pix_per_split;
  const int pend = min(M, pbeg + a.pix_per_split);
  if (pbeg >= pend) return;
  const int nsteps = (pend - pbeg + BP - 1) / BP;

  // ---- per-lane DMA sources (fixed for the pixel loop) --------------------------------------
  // A: instruction j of wave w covers rows ARPI*(j*NW + w) + lane / 32 (ARPI = 2), LDS chunk
  // lane % 32; row & 3 does not depend on j, so neither does the logical chunk
  constexpr int ACH = C::AROWB / 16, GCH = C::GROWB / 16;
  const int a_sub = lane / ACH, a_pos = lane % ACH;
  const int a_row0 = C::ARPI * wid + a_sub;  // + ARPI * NW * j
  const int a_c = wb_swz<C::AROWB>(a_row0, a_pos);
  const int kk = k0 + a_c * 8;
  const bool k_ok = kk < K;
  const int rs = k_ok ? kk / a.Cin : 0, cc = k_ok ? kk - rs * a.Cin : 0;
  const int kr = rs / a.KW, ks = rs - kr * a.KW;
  const int g_sub = lane / GCH, g_pos = lane % GCH;
  const int g_row0 = C::GRPI * wid + g_sub;
  const int g_c = wb_swz<C::GROWB>(g_row0, g_pos);
  FDiv dwo, dho;
  dwo.init(a.Wo);
  dho.init(a.Ho);
  const bf16_t* __restrict__ X = a.x;
  const bf16_t* __restrict__ G = reinterpret_cast<const bf16_t*>(a.g);
  const void* zsrc = g_wgz;

  auto issue = [&](int kt, int buf) {
    char* As = smem + buf * C::BUF;
    char* Gs = As + C::A_BYTES;
    const int mb = pbeg + kt * BP;
#pragma unroll
    for (int j = 0; j < NGA; ++j) {
      const int m = mb + a_row0 + C::ARPI * NW * j;
      const int t = dwo.div(m), wo = m - t * a.Wo;
      const int img = dho.div(t), ho = t - img * a.Ho;
      const int h = ho * a.SH - a.PT + kr, w = wo * a.SW - a.PL + ks;
      const bool ok = k_ok && m < pend && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const void* src = ok ? (const void*)(X + ((size_t)(img * a.H + h) * a.W + w) * a.ldx + cc) : zsrc;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(As + (j * NW + wid) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NGG; ++j) {
      const int m = mb + g_row0 + C::GRPI * NW * j;
      const void* src = m < pend ? (const void*)(G + (size_t)m * a.ldg + c0 + g_c * 8) : zsrc;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(Gs + (j * NW + wid) * 1024), 16, 0, 0);
    }
  };

  v16f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one barrier per step: at the top of step kt every wave has (a) waited for its own step-kt
  // DMA and (b) finished step kt-1, whose buffer then takes step kt+NBUF-1 (NBUF-1 steps ahead)
  constexpr int NG = NGA + NGG;
#pragma unroll
  for (int b = 0; b < NBUF - 1; ++b)
    if (b < nsteps) issue(b, b);
  for (int kt = 0; kt < nsteps; ++kt) {
    const int after = min(NBUF - 2, nsteps - 1 - kt);  // steps after kt already issued
    if (after >= 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NG) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NBUF - 1 < nsteps) issue(kt + NBUF - 1, (kt + NBUF - 1) % NBUF);
    const char* As = smem + (kt % NBUF) * C::BUF;
    const char* Gs = As + C::A_BYTES;
#pragma unroll
    for (int ps = 0; ps < BP / 16; ++ps) {
      v8bf af[TM], gf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = wb_frag<C::AROWB>(As, wr * C::WTM + i * 32, lane, ps * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j) gf[j] = wb_frag<C::GROWB>(Gs, wc * C::WTN + j * 32, lane, ps * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], gf[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: accumulator register r = rows 8*(r/4) + 4*(lane/32) + r%4, column lane%32:
  // two 128-B row segments per wave-instruction, added (or stored) straight into dW[k][co]
  const long long n_dw = (long long)K * a.Cout;
  const int col = lane & 31, rhalf = (lane >> 5) * 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = c0 + wc * C::WTN + j * 32 + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = k0 + wr * C::WTM + i * 32 + 8 * (r >> 2) + rhalf + (r & 3);
        if (k >= K) continue;
        const float v = acc[i][j][r] * a.scale;
        const size_t o = (size_t)k * a.Cout + co;
        if (a.part) a.part[(size_t)zslice * n_dw + o] = v;
        else atomicAdd(&a.dw[o], v);
      }
    }
}

namespace {
struct WbVariant {
  int bc, bp, nbuf;
};
// autotune candidates (OP_WGRAD i[2] = variant; 0 = the general kernel)
constexpr WbVariant kWb[] = {{0, 0, 0},     {128, 32, 3}, {128, 64, 2}, {128, 64, 3}, {256, 32, 3},
                             {256, 64, 2}, {128, 32, 2}, {64, 64, 2},  {64, 64, 3}};
constexpr int kWbN = sizeof(kWb) / sizeof(kWb[0]);
}  // namespace

int wgrad_num_variants() { return kWbN; }
int wgrad_variant_bc(int v) { return (v > 0 && v < kWbN) ? kWb[v].bc : 0; }
int wgrad_variant_bp(int v) { return (v > 0 && v < kWbN) ? kWb[v].bp : 32; }

bool wgrad_big_ok(const WgradArgs& a, bool g_f32, int variant) {
  if (variant <= 0 || variant >= kWbN) return false;
  const int bc = kWb[variant].bc;
  return !g_f32 && a.pro.mode == 0 && a.pro.act == ACT_NONE && a.gpro.mode == 0 && a.Cin % 64 == 0 &&
         a.Cout % bc == 0 && a.ldx % 8 == 0 && a.ldg % 8 == 0 && (a.cin_real == 0 || a.cin_real == a.Cin) &&
         (long long)a.N * a.Ho * a.Wo < (1 << 21) && a.Wo < (1 << 20) && a.Ho < (1 << 20);
}

int wgrad_big_pick_splits(int M, int K, int Cout, int variant) {
  if (variant <= 0 || variant >= kWbN) return 1;
  const WbVariant v = kWb[variant];
  const int tiles = ((K + 255) / 256) * ((Cout + v.bc - 1) / v.bc);
  const int per_cu = (160 * 1024) / (v.nbuf * v.bp * (256 + v.bc) * 2);
  const int target = 256 * (per_cu < 1 ? 1 : per_cu);
  int s = (target + tiles - 1) / tiles;
  const int maxs = (M + 4 * v.bp - 1) / (4 * v.bp);  // at least 4 steps per slice
  if (s > maxs) s = maxs;
  return s < 1 ? 1 : s;
}

template <int BC, int BP, int NBUF>
static hipError_t wb_launch(const WgradArgs& a, int splits, hipStream_t st) {
  using C = WbCfg<BC, BP, NBUF>;
  const int K = a.KH * a.KW * a.Cin;
  const int grid = ((K + C::BKR - 1) / C::BKR) * (a.Cout / BC) * splits;
  hipLaunchKernelGGL((wgrad_big_kernel<BC, BP, NBUF>), ggrid(grid), dim3(C::NT), C::LDS_BYTES, st, a, garg());
  return hipGetLastError();
}

hipError_t wgrad_big(WgradArgs a, int splits, bool g_f32, int variant, hipStream_t st) {
  if (!wgrad_big_ok(a, g_f32, variant)) return hipErrorInvalidValue;
  const WbVariant v = kWb[variant];
  const int M = a.N * a.Ho * a.Wo;
  if (splits < 1) splits = 1;
  int per = (M + splits - 1) / splits;
  per = (per + v.bp - 1) / v.bp * v.bp;
  splits = (M + per - 1) / per;
  a.pix_per_split = per;
  if (a.part && (long long)splits * a.KH * a.KW * a.Cin * a.Cout > a.part_floats) return hipErrorInvalidValue;
  if (M == 0) return hipSuccess;
  switch (variant) {
    case 1: return wb_launch<128, 32, 3>(a, splits, st);
    case 2: return wb_launch<128, 64, 2>(a, splits, st);
    case 3: return wb_launch<128, 64, 3>(a, splits, st);
    case 4: return wb_launch<256, 32, 3>(a, splits, st);
    case 5: return wb_launch<256, 64, 2>(a, splits, st);
    case 6: return wb_launch<128, 32, 2>(a, splits, st);
    case 7: return wb_launch<64, 64, 2>(a, splits, st);
    case 8: return wb_launch<64, 64, 3>(a, splits, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace idc
