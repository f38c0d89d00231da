// Weight gradient of an NHWC convolution on MFMA (v_mfma_f32_16x16x32_bf16), gfx950.
//
//   dW[k, co] = sum_m A[m, k] * G[m, co]      (Keras HWIO layout: k = (r, s, c), row stride Cout)
//   A = im2col(act(bn(x)))  — the forward operand, RECOMPUTED from the saved raw input + BN
//                             statistics (no saved activation), exactly as the forward staged it
//   G = dY                  — bf16 or fp32 (DenseNet's fp32 concat-gradient buffer)
//
// The reduction dimension is the pixel count M = N*Ho*Wo (up to 640k) while the output is tiny,
// so the pixel range is split over gridDim.z slices (split-K) and partial tiles are combined with
// fp32 atomics shaped as whole 128/256-byte rows (staged through LDS; guide Guideline 12).
// Both MFMA operands need the PIXEL index as their k dimension but arrive pixel-major from HBM,
// so tiles are staged [pixel][column] in LDS and read transposed with ds_read_b64_tr_b16
// (guide §5.5 T10); the XOR swizzles below were brute-force checked conflict-free for those
// reads and for the ds_write_b128 staging stores.
#include <cstdlib>

#include "common.h"
#include "conv_wgrad.h"

namespace idc {

typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4bf lds_v4bf;

// swizzled 16-B chunk index for a row of ROWB bytes
template <int ROWB>
__device__ __forceinline__ int wswz(int row, int chunk) {
  if constexpr (ROWB == 64) return chunk ^ (((row >> 3) & 1) << 1);
  else if constexpr (ROWB == 128) return chunk ^ ((((row >> 3) & 1) << 1) ^ ((row & 3) << 1));
  else return chunk ^ (((row & 3) << 2) | ((row >> 2) & 3));
}

template <int BKR, int BC, int BP_>
struct WgCfg {
  static constexpr int NT = 256;
  static constexpr int BP = BP_;  // pixels per k-step (a multiple of the MFMA k = 32)
  static constexpr int A_ELEMS = BP * BKR, G_ELEMS = BP * BC;
  static constexpr int STAGE = 2 * (A_ELEMS + G_ELEMS) * 2;
  static constexpr int CS_LD = BC + 4;
  static constexpr int EPI = BKR * CS_LD * 4;
  static constexpr int MAIN = STAGE > EPI ? STAGE : EPI;
  static int smem_bytes(int cpro) { return MAIN + 2 * ((cpro + 3) / 4 * 4) * 4 + 3 * BC * 4; }
};

// 8 bf16 from two transposed 4-element reads (pixels r0+8g..+3 and r0+8g+4..+7)
template <int ROWB>
__device__ __forceinline__ v8bf tr_frag(const bf16_t* tile, int col_base, int lane, int r0) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  v8bf out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    int row = r0 + 8 * g + 4 * t + q;
    int col = col_base + 4 * p;
    int ch = col >> 3, sub = col & 7;
    const bf16_t* ptr = tile + row * (ROWB / 2) + wswz<ROWB>(row, ch) * 8 + sub;
    v4bf v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(ptr));
    out[4 * t + 0] = v[0];
    out[4 * t + 1] = v[1];
    out[4 * t + 2] = v[2];
    out[4 * t + 3] = v[3];
  }
  return out;
}

// One (k tile bkx, cout tile bky, pixel slice zslice) workgroup of the pixel-split GEMM; shared by
// the per-layer kernel below and the batched launch (conv_wgrad_batch_kernel).
template <int BKR, int BC, int BP_, int WM, int WN, bool IS1X1, typename TG, int PRO, int GPRO>
__device__ __forceinline__ void wgrad_tile(const WgradArgs& a, const int bkx, const int bky, const int zslice) {
  using C = WgCfg<BKR, BC, BP_>;
  constexpr int NT = C::NT, BP = C::BP;
  constexpr int WTM = BKR / WM, WTN = BC / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int ACH = BKR / 8, GCH = BC / 8;           // 16-B chunks per LDS row
  constexpr int NA = (BP * ACH + NT - 1) / NT;
  constexpr int NG = (BP * GCH + NT - 1) / NT;
  constexpr int AROWB = BKR * 2, GROWB = BC * 2;
  static_assert(NT % ACH == 0, "A chunk mapping");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Gs = As + 2 * C::A_ELEMS;
  float* Cs = reinterpret_cast<float*>(smem);
  const int cpro = PRO ? (a.Cin + 3) / 4 * 4 : 0;
  float* s_scale = reinterpret_cast<float*>(smem + C::MAIN);
  float* s_shift = s_scale + cpro;
  float* s_ga = s_shift + cpro;  // GPRO: backward-affine coefficients of the G columns
  float* s_gb = s_ga + BC;
  float* s_gc = s_gb + BC;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int wr = wid / WN, wc = wid % WN;
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.KH * a.KW * a.Cin;
  const int k0 = bkx * BKR;
  const int c0 = bky * BC;
  const int per = a.pix_per_split;
  const int pbeg = zslice * per;
  const int pend = min(M, pbeg + per);
  if (pbeg >= pend) return;

  // ---- A (im2col) staging: thread owns k-chunk `ach` (fixed) for pixel rows arow + 32/..*i ----
  const int ach = tid % ACH;
  const int arow0 = tid / ACH;            // first pixel row (0..BP) this thread stages
  constexpr int AROW_STEP = NT / ACH;     // rows between a thread's successive chunks
  const int kk = k0 + ach * 8;
  const bool k_ok = kk < K;
  int kr = 0, ks = 0, kc = kk;
  if constexpr (!IS1X1) {
    int rs = kk / a.Cin;
    kc = kk - rs * a.Cin;
    kr = rs / a.KW;
    ks = rs - kr * a.KW;
  }

  const bf16_t* __restrict__ X = a.x;
  const TG* __restrict__ G = reinterpret_cast<const TG*>(a.g);
  uint4 ra[NA];
  bool rv[NA];
  uint4 rg[NG];
  uint4 rgx[GPRO ? NG : 1];
  bool gv[NG];
  float rgf[sizeof(TG) == 4 ? NG : 1][8];

  auto load = [&](int mbase) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int row = arow0 + i * AROW_STEP;
      int m = mbase + row;
      bool ok = (row < BP) && (m < pend) && k_ok;
      size_t off = 0;
      if constexpr (IS1X1) {
        off = (size_t)m * a.ldx + kc;
      } else {
        // direct decode (a few integer divisions per row per step; an incremental walk costs
        // BP/Wo iterations per row on the small late-stage maps)
        const int mm = ok ? m : 0;
        const int wo = mm % a.Wo, t = mm / a.Wo;
        const int ho = t % a.Ho, img = t / a.Ho;
        int h = ho * a.SH - a.PT + kr, w = wo * a.SW - a.PL + ks;
        ok = ok && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        off = ((size_t)(img * a.H + h) * a.W + w) * a.ldx + kc;
      }
      rv[i] = ok;
      ra[i] = *reinterpret_cast<const uint4*>(X + (ok ? off : 0));  // unconditional (no drain)
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      int idx = tid + i * NT;
      int row = idx / GCH, ch = idx % GCH;
      int m = mbase + row;
      int co = c0 + ch * 8;
      bool ok = (idx < BP * GCH) && (m < pend) && (co < a.Cout);
      const size_t gm = ok ? (size_t)m : 0;
      const size_t goff = ok ? gm * a.ldg + co : 0;
      gv[i] = ok;
      if constexpr (GPRO) rgx[i] = *reinterpret_cast<const uint4*>(a.gpro.x + gm * a.gpro.ldx + (ok ? co : 0));
      if constexpr (sizeof(TG) == 2) {
        rg[i] = *reinterpret_cast<const uint4*>(G + goff);
      } else {
        float4 u = *reinterpret_cast<const float4*>(G + goff);
        float4 v = *reinterpret_cast<const float4*>(G + goff + 4);
        rgf[i][0] = u.x; rgf[i][1] = u.y; rgf[i][2] = u.z; rgf[i][3] = u.w;
        rgf[i][4] = v.x; rgf[i][5] = v.y; rgf[i][6] = v.z; rgf[i][7] = v.w;
      }
    }
  };

  auto store = [&](int buf) {
    bf16_t* as = As + buf * C::A_ELEMS;
    bf16_t* gs = Gs + buf * C::G_ELEMS;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int row = arow0 + i * AROW_STEP;
      if (row >= BP) break;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (rv[i]) {
        if constexpr (PRO) {
          float f[8];
          unpack8(ra[i], f);
          affine_act8(f, s_scale + kc, s_shift + kc, act_lo(a.pro.act), act_hi(a.pro.act));
          v = pack8(f);
        } else {
          v = ra[i];
        }
      }
      *reinterpret_cast<uint4*>(as + row * BKR + wswz<AROWB>(row, ach) * 8) = v;
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      int idx = tid + i * NT;
      if (idx >= BP * GCH) break;
      int row = idx / GCH, ch = idx % GCH;
      uint4 v;
      if constexpr (GPRO) {
        float f[8], xf[8];
        if constexpr (sizeof(TG) == 2) {
          unpack8(rg[i], f);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = rgf[i][j];
        }
        unpack8(rgx[i], xf);
        bwd_aff8(f, xf, s_ga + ch * 8, s_gb + ch * 8, s_gc + ch * 8);
        v = pack8(f);
      } else if constexpr (sizeof(TG) == 2) {
        v = rg[i];
      } else {
        v = pack8(rgf[i]);
      }
      if (!gv[i]) v = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(gs + row * BC + wswz<GROWB>(row, ch) * 8) = v;
    }
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int nsteps = (pend - pbeg + BP - 1) / BP;
  load(pbeg);  // first tile in flight while the BN table is built (its loads overlap)
  if constexpr (PRO) bn_coeff_table<NT>(a.pro, a.Cin, s_scale, s_shift);
  if constexpr (GPRO) bwd_aff_table<NT>(a.gpro, c0, BC, a.Cout, s_ga, s_gb, s_gc);
  __syncthreads();
  store(0);
  __syncthreads();
  for (int it = 0; it < nsteps; ++it) {
    const int cur = it & 1;
    // unconditional prefetch (rows past `pend` are masked): no back-edge vmcnt(0) drain
    load(pbeg + (it + 1) * BP);
    const bf16_t* as = As + cur * C::A_ELEMS;
    const bf16_t* gs = Gs + cur * C::G_ELEMS;
#pragma unroll
    for (int kq = 0; kq < BP / 32; ++kq) {
      v8bf af[TM], gf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag<AROWB>(as, wr * WTM + i * 16, lane, kq * 32);
#pragma unroll
      for (int j = 0; j < TN; ++j) gf[j] = tr_frag<GROWB>(gs, wc * WTN + j * 16, lane, kq * 32);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], gf[j], acc[i][j], 0, 0, 0);
    }
    store(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: tile -> LDS -> row-contiguous fp32 atomics into dW[k][co] ----------------
  constexpr int CS_LD = C::CS_LD;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = wc * WTN + j * 16 + (lane & 15);
      int rbase = wr * WTM + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(rbase + r) * CS_LD + col] = acc[i][j][r];
    }
  __syncthreads();
  for (int idx = tid; idx < BKR * BC; idx += NT) {
    int row = idx / BC, col = idx % BC;
    int k = k0 + row, co = c0 + col;
    if (k >= K || co >= a.Cout) continue;
    int kdst = k;
    if (a.cin_real && a.cin_real != a.Cin) {
      int rs = k / a.Cin, c = k - rs * a.Cin;
      if (c >= a.cin_real) continue;
      kdst = rs * a.cin_real + c;
    }
    const float v = Cs[row * CS_LD + col] * a.scale;
    if (a.part) a.part[(size_t)zslice * ((size_t)a.KH * a.KW * (a.cin_real ? a.cin_real : a.Cin) * a.Cout) +
                       (size_t)kdst * a.Cout + co] = v;
    else atomicAdd(&a.dw[(size_t)kdst * a.Cout + co], v);
  }
}

template <int BKR, int BC, int BP_, int WM, int WN, bool IS1X1, typename TG, int PRO, int GPRO>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(WgradArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  // this workgroup's pixel slice (z = copy * splits + slice)
  wgrad_tile<BKR, BC, BP_, WM, WN, IS1X1, TG, PRO, GPRO>(a, blockIdx.x, blockIdx.y, gz(ga));
}

// ----------------------------------------------------------------------------------------------
// Direct 3x3 weight gradient for SMALL images (DenseNet growth convs: 3x3 / s1 / 'same',
// Cout = 32, on 13x13, 6x6 and 3x3 maps).  As a pixel-split GEMM (conv_wgrad_kernel) these take
// 20-50 us on the side lane: 32-pixel K steps of 4 MFMAs per wave, each behind a global load
// round trip, plus ~100 fp32 atomics per dW element from the pixel slices.  Here a workgroup owns
// a run of whole images and 64 input channels and keeps the full 9 x 64 x 32 dW partial in
// registers (wave w: channels 16w..16w+15, all 9 taps, both 16-column halves of Cout):
//
//   * a pass stages P images as one stacked halo tile X[(img, h+1, w+1)][c] (BN + act applied,
//     zero padding AFTER the activation, Keras semantics) and G[(img, h, w)][co] in the SAME
//     padded (H+2)x(W+2) row space, so for tap (r, s) the im2col operand of output position q is
//     simply row q + r*(W+2) + s of X: every tap is a shifted window, no gather, no im2col;
//   * dW[tap][c][co] += sum_q X[q + off(tap)][c] * G[q][co] over q = pixel rows of the pass, in
//     32-row chunks with v_mfma_f32_16x16x32_bf16; both operands are read transposed from their
//     [row][column] LDS images with ds_read_b64_tr_b16 (tr_frag above), the G fragments once per
//     chunk for all 9 taps;
//   * positions outside an image (the W+2 padding columns, the rows between stacked images) have
//     G = 0, so they add nothing; the next pass's loads are in flight during the MFMAs;
//   * at the end, one fp32 atomic per dW element per workgroup (or a plain store into the
//     deterministic mode's per-group partial slab).
// Reference hot loop: the Conv2D gradient of dist_model_tf_dense.py:131-150 (DenseNet-121).
namespace {
constexpr int WH_CB = 64;        // input channels per workgroup
constexpr int WH_MAXPIX = 256;   // valid pixels staged per pass (<= 8 X / 4 G chunks per thread)
constexpr int WH_XROWB = WH_CB * 2;  // 128 B per X row
constexpr int WH_GROWB = 32 * 2;     // 64 B per G row

struct WhGeom {
  int Hp, Wp, RI, P, q_max, qpad, xrows, grows;
  size_t x_bytes, g_bytes;
};

__host__ __device__ inline WhGeom wh_geom(int H, int W, int ipw) {
  WhGeom g;
  g.Hp = H + 2;
  g.Wp = W + 2;
  g.RI = g.Hp * g.Wp;
  int p = WH_MAXPIX / (H * W);
  const int p_lds = (56 * 1024) / (g.RI * WH_XROWB);  // X tile budget
  if (p > p_lds) p = p_lds;
  if (p > ipw) p = ipw;
  g.P = p < 1 ? 1 : p;
  g.q_max = (g.P - 1) * g.RI + (H - 1) * g.Wp + W;  // one past the last valid output row
  g.qpad = (g.q_max + 31) / 32 * 32;
  const int need_x = g.qpad + 2 * g.Wp + 2;          // rows the shifted windows touch
  g.xrows = need_x > g.P * g.RI ? need_x : g.P * g.RI;
  g.grows = g.qpad;
  g.x_bytes = (size_t)g.xrows * WH_XROWB;
  g.g_bytes = (size_t)g.grows * WH_GROWB;
  return g;
}
}  // namespace

__device__ __forceinline__ void wgrad3x3_img_tile(const WgradArgs& a, const int ipw, const int bx, const int by) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, W = a.W;
  const WhGeom geo = wh_geom(H, W, ipw);
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Gs = reinterpret_cast<bf16_t*>(smem + geo.x_bytes);
  float* s_scale = reinterpret_cast<float*>(smem + geo.x_bytes + geo.g_bytes);
  float* s_shift = s_scale + a.Cin;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int c0 = by * WH_CB;
  const int img_beg = bx * ipw;
  const int img_end = min(a.N, img_beg + ipw);
  const int HW = H * W, Wp = geo.Wp, RI = geo.RI, P = geo.P;

  // zero both tiles once: padding rows / columns are never written afterwards
  {
    uint4* z = reinterpret_cast<uint4*>(smem);
    const int n16 = (int)((geo.x_bytes + geo.g_bytes) / 16);
    for (int i = tid; i < n16; i += 256) z[i] = make_uint4(0, 0, 0, 0);
  }
  bn_coeff_table<256>(a.pro, a.Cin, s_scale, s_shift);
  const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);

  const bf16_t* __restrict__ X = a.x;
  const bf16_t* __restrict__ G = reinterpret_cast<const bf16_t*>(a.g);
  uint4 rx[8], rg[4];

  // chunk i of a pass: X chunk e = tid + 256*i -> (pixel e/8, channel chunk e%8);
  //                    G chunk e = tid + 256*i -> (pixel e/4, column chunk e%4)
  auto load = [&](int ib) {
    const int np = min(P, img_end - ib) * HW;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, px = e >> 3, ch = e & 7;
      const bool ok = px < np;
      const size_t pix = (size_t)ib * HW + (ok ? px : 0);
      rx[i] = *reinterpret_cast<const uint4*>(X + pix * a.ldx + c0 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, px = e >> 2, ch = e & 3;
      const bool ok = px < np;
      const size_t pix = (size_t)ib * HW + (ok ? px : 0);
      rg[i] = *reinterpret_cast<const uint4*>(G + pix * a.ldg + ch * 8);
    }
  };
  auto store = [&](int ib) {
    const int nimg = min(P, img_end - ib);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, px = e >> 3, ch = e & 7;
      if (px >= nimg * HW) continue;  // rows of absent images keep stale finite values (G = 0 there)
      const int im = px / HW, r = px - im * HW, h = r / W, w = r - h * W;
      const int row = im * RI + (h + 1) * Wp + (w + 1);
      float f[8];
      unpack8(rx[i], f);
      affine_act8(f, s_scale + c0 + ch * 8, s_shift + c0 + ch * 8, lo, hi);
      *reinterpret_cast<uint4*>(Xs + row * WH_CB + wswz<WH_XROWB>(row, ch) * 8) = pack8(f);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, px = e >> 2, ch = e & 3;
      if (px >= P * HW) continue;
      const int im = px / HW, r = px - im * HW, h = r / W, w = r - h * W;
      const int row = im * RI + h * Wp + w;
      const uint4 v = px < nimg * HW ? rg[i] : make_uint4(0, 0, 0, 0);  // absent images: G = 0
      *reinterpret_cast<uint4*>(Gs + row * 32 + wswz<WH_GROWB>(row, ch) * 8) = v;
    }
  };

  v4f acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = (v4f){0.f, 0.f, 0.f, 0.f};

  if (img_beg < img_end) load(img_beg);
  __syncthreads();  // zero fill + coefficient table
  for (int ib = img_beg; ib < img_end; ib += P) {
    store(ib);
    __syncthreads();
    if (ib + P < img_end) load(ib + P);  // next pass in flight under the MFMAs
    const int nq = geo.qpad / 32;
    for (int qc = 0; qc < nq; ++qc) {
      const int q0 = qc * 32;
      const v8bf g0 = tr_frag<WH_GROWB>(Gs, 0, lane, q0);
      const v8bf g1 = tr_frag<WH_GROWB>(Gs, 16, lane, q0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = (t / 3) * Wp + (t % 3);
        const v8bf xf = tr_frag<WH_XROWB>(Xs, wid * 16, lane, q0 + off);
        acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, g0, acc[t][0], 0, 0, 0);
        acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, g1, acc[t][1], 0, 0, 0);
      }
    }
    __syncthreads();  // LDS reads done before the next pass overwrites the tiles
  }

  // epilogue: C[row = channel, col = co]; row = (lane>>4)*4 + r, col = lane&15 (+16 for half 1)
  const long long n_dw = 9LL * a.Cin * 32;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + wid * 16 + (lane >> 4) * 4 + r;
        const int co = j * 16 + (lane & 15);
        const size_t k = (size_t)t * a.Cin + c;
        const float v = acc[t][j][r] * a.scale;
        if (a.part) a.part[(size_t)bx * n_dw + k * 32 + co] = v;
        else atomicAdd(&a.dw[k * 32 + co], v);
      }
}

__global__ __launch_bounds__(256) void wgrad3x3_img_kernel(WgradArgs a, int ipw, GroupArg ga) {
  gshift(a, goff(ga));
  prefetch_kernargs<sizeof(WgradArgs)>();
  wgrad3x3_img_tile(a, ipw, blockIdx.x, blockIdx.y);
}

// the direct small-image path applies (and then `splits` counts image groups): 3x3 / s1 / pad 1,
// Cout 32, bf16 G without a pending affine, Cin a multiple of 64, maps of at most 16x16
static bool wgrad_halo_ok(const WgradArgs& a, bool g_f32) {
  static const bool on = [] {
    const char* e = std::getenv("IDC_WG_HALO");
    return !(e && e[0] == '0');
  }();
  return on && !g_f32 && a.KH == 3 && a.KW == 3 && a.SH == 1 && a.SW == 1 && a.PT == 1 && a.PL == 1 &&
         a.Ho == a.H && a.Wo == a.W && a.Cout == 32 && a.Cin % WH_CB == 0 && a.gpro.mode == 0 &&
         (a.cin_real == 0 || a.cin_real == a.Cin) && a.H <= 16 && a.W <= 16 && a.H * a.W >= 4 &&
         a.ldx % 8 == 0 && a.ldg % 8 == 0;
}

static int wgrad_halo_groups(const WgradArgs& a, int splits) {
  int g = splits < 1 ? 1 : (splits > a.N ? a.N : splits);
  const int ipw = (a.N + g - 1) / g;
  return (a.N + ipw - 1) / ipw;
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                           long long n, int splits, GroupArg ga) {
  const long long go = goff(ga);
  part = gsh(part, go);
  dw = gsh(dw, go);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += part[(size_t)z * n + i];
    dw[i] += s;
  }
}

hipError_t wgrad_reduce(const float* part, float* dw, long long n, int splits, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (part == nullptr || dw == nullptr || splits < 1) return hipErrorInvalidValue;
  long long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  hipLaunchKernelGGL(wgrad_reduce_kernel, ggrid((int)b), dim3(256), 0, st, part, dw, n, splits, garg());
  return hipGetLastError();
}

template <int BKR, int BC, int BP, int WM, int WN>
static hipError_t launch_wg(const WgradArgs& a, bool is1x1, bool g_f32, int pro, int splits,
                            hipStream_t st) {
  const int K = a.KH * a.KW * a.Cin;
  dim3 grid((K + BKR - 1) / BKR, (a.Cout + BC - 1) / BC, splits);
  const size_t shm = WgCfg<BKR, BC, BP>::smem_bytes(pro ? a.Cin : 0);
  const bool gpro = a.gpro.mode != 0;
#define IDC_W(IS1, TG, P, GP) \
  hipLaunchKernelGGL((conv_wgrad_kernel<BKR, BC, BP, WM, WN, IS1, TG, P, GP>), ggrid(grid), dim3(256), shm, st, a, \
                     garg(splits))
#define IDC_WG(IS1, TG, P) if (gpro) IDC_W(IS1, TG, P, 1); else IDC_W(IS1, TG, P, 0);
#define IDC_WP(IS1, TG) if (pro) { IDC_WG(IS1, TG, 1) } else { IDC_WG(IS1, TG, 0) }
  if (g_f32) {
    if (is1x1) { IDC_WP(true, float) } else { IDC_WP(false, float) }
  } else {
    if (is1x1) { IDC_WP(true, bf16_t) } else { IDC_WP(false, bf16_t) }
  }
#undef IDC_WP
#undef IDC_WG
#undef IDC_W
  return hipGetLastError();
}

// pixels per k-step of the tile chosen for Cout (launch_wg below)
// (32: the deeper 64/128-pixel steps measured slower — their 58-83 KB LDS footprint cuts the
// workgroups per CU, and these kernels are latency-bound, not MFMA-bound)
static int wgrad_bp(int) { return 32; }

// 128x128 tiles (64x64 per wave: 16 MFMAs per 32-pixel step against 8 transposed fragment
// reads, vs 8 against 6 for 32x64) for wide layers over few pixels (K >= 512, Cout >= 128,
// M <= 16384).  Opt-in (IDC_WG_BIG=1): measured slower on VGG16 (3.12 vs 3.02 ms/step, blocks
// 4-5) and neutral on DenseNet-121 (4.34-4.44 both ways) — these loops are load-latency bound,
// and the bigger tile halves the workgroups that hide it.
static bool wgrad_big_on() {
  static const bool on = [] {
    const char* e = std::getenv("IDC_WG_BIG");
    return e && e[0] == '1';
  }();
  return on;
}
static bool wgrad_big_tile(const WgradArgs& a) {
  return wgrad_big_on() && a.Cout >= 128 && a.KH * a.KW * a.Cin >= 512 && a.N * a.Ho * a.Wo <= 16384;
}

hipError_t conv_wgrad(WgradArgs a, int splits, bool g_f32, hipStream_t st, int variant) {
  if (wgrad_stem_ok(a, g_f32)) return wgrad_stem(a, st);
  if (variant > 0 && wgrad_big_ok(a, g_f32, variant)) return wgrad_big(a, splits, g_f32, variant, st);
  if (wgrad_halo_ok(a, g_f32)) {
    const int groups = wgrad_halo_groups(a, splits);
    const int ipw = (a.N + groups - 1) / groups;
    if (a.part && (long long)groups * 9 * a.Cin * 32 > a.part_floats) return hipErrorInvalidValue;
    const WhGeom geo = wh_geom(a.H, a.W, ipw);
    const size_t shm = geo.x_bytes + geo.g_bytes + 2 * (size_t)a.Cin * 4;
    hipLaunchKernelGGL(wgrad3x3_img_kernel, ggrid(dim3(groups, a.Cin / WH_CB)), dim3(256), shm, st, a, ipw, garg());
    return hipGetLastError();
  }
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0;
  const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  const int M = a.N * a.Ho * a.Wo;
  if (splits < 1) splits = 1;
  const int bp = wgrad_bp(a.Cout);
  int per = (M + splits - 1) / splits;
  per = (per + bp - 1) / bp * bp;
  splits = (M + per - 1) / per;
  a.pix_per_split = per;
  if (a.part) {  // the partial slab must hold every slice
    const long long n = (long long)a.KH * a.KW * (a.cin_real ? a.cin_real : a.Cin) * a.Cout;
    if ((long long)splits * n > a.part_floats) return hipErrorInvalidValue;
  }
  if (a.Cout <= 32) return launch_wg<128, 32, 32, 4, 1>(a, is1x1, g_f32, pro, splits, st);
  if (a.Cout <= 64) return launch_wg<128, 64, 32, 2, 2>(a, is1x1, g_f32, pro, splits, st);
  if (wgrad_big_tile(a)) return launch_wg<128, 128, 32, 2, 2>(a, is1x1, g_f32, pro, splits, st);
  return launch_wg<64, 128, 32, 2, 2>(a, is1x1, g_f32, pro, splits, st);
}

int wgrad_effective_splits(const WgradArgs& a, int splits, int variant) {
  if (wgrad_stem_ok(a, false)) return wgrad_stem_slices(a);
  const bool big = variant > 0 && wgrad_big_ok(a, false, variant);
  if (!big && wgrad_halo_ok(a, false)) return wgrad_halo_groups(a, splits);
  const int M = a.N * a.Ho * a.Wo;
  if (splits < 1) splits = 1;
  const int bp = big ? wgrad_variant_bp(variant) : wgrad_bp(a.Cout);
  int per = (M + splits - 1) / splits;
  per = (per + bp - 1) / bp * bp;
  return (M + per - 1) / per;
}

// ---- batched weight gradients (conv_wgrad.h) -------------------------------------------------
__device__ __forceinline__ int wg_batch_member(const int* __restrict__ begins, int lin) {
  const int lane = threadIdx.x & 63;
  const int v = begins[lane];  // padded with INT_MAX to WG_BATCH_MAX entries
  return __popcll(__ballot(v <= lin)) - 1;
}

template <int BKR, int BC, int BP, int WM, int WN, bool IS1X1, int PRO>
__global__ __launch_bounds__(256) void conv_wgrad_batch_kernel(const WgBatchEntry* __restrict__ list,
                                                               const int* __restrict__ begins, GroupArg ga) {
  const int lin = blockIdx.x;
  const int m = wg_batch_member(begins, lin);
  WgradArgs a = list[m].a;
  gshift(a, goff(ga));
  const int gx = list[m].gx, gxy = gx * list[m].gy;
  const int r = lin - begins[m];
  const int z = r / gxy, rem = r - z * gxy;
  wgrad_tile<BKR, BC, BP, WM, WN, IS1X1, bf16_t, PRO, 0>(a, rem % gx, rem / gx, z);
}

__global__ __launch_bounds__(256) void wgrad3x3_img_batch_kernel(const WgBatchEntry* __restrict__ list,
                                                                 const int* __restrict__ begins, GroupArg ga) {
  const int lin = blockIdx.x;
  const int m = wg_batch_member(begins, lin);
  WgradArgs a = list[m].a;
  gshift(a, goff(ga));
  const int gx = list[m].gx;
  const int r = lin - begins[m];
  wgrad3x3_img_tile(a, list[m].ipw, r % gx, r / gx);
}

// general-kernel tile of a member: 0 <128,32>, 1 <128,64>, 2 <128,128>, 3 <64,128>
static int wg_tile_sel(const WgradArgs& a) {
  if (a.Cout <= 32) return 0;
  if (a.Cout <= 64) return 1;
  if (wgrad_big_tile(a)) return 2;
  return 3;
}

int wgrad_batch_sig(const WgradArgs& a, bool g_f32, int variant) {
  if (a.part || g_f32 || a.gpro.mode != 0) return -1;
  if (variant > 0 && wgrad_big_ok(a, g_f32, variant)) return -1;
  if (wgrad_halo_ok(a, g_f32)) return 1;
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0;
  const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  return 16 + wg_tile_sel(a) * 4 + (is1x1 ? 2 : 0) + pro;
}

int wgrad_batch_entry(const WgradArgs& a0, int splits, WgBatchEntry& e, long long& smem) {
  WgradArgs a = a0;
  e.ipw = 0;
  if (wgrad_halo_ok(a, false)) {
    const int groups = wgrad_halo_groups(a, splits);
    e.ipw = (a.N + groups - 1) / groups;
    const WhGeom geo = wh_geom(a.H, a.W, e.ipw);
    smem = (long long)(geo.x_bytes + geo.g_bytes + 2 * (size_t)a.Cin * 4);
    e.a = a;
    e.gx = groups;
    e.gy = a.Cin / WH_CB;
    e.gz = 1;
    return e.gx * e.gy;
  }
  const int M = a.N * a.Ho * a.Wo;
  if (splits < 1) splits = 1;
  const int bp = wgrad_bp(a.Cout);
  int per = (M + splits - 1) / splits;
  per = (per + bp - 1) / bp * bp;
  splits = (M + per - 1) / per;
  a.pix_per_split = per;
  const int K = a.KH * a.KW * a.Cin;
  const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  int bkr = 64, bc = 128;
  switch (wg_tile_sel(a)) {
    case 0: bkr = 128; bc = 32; smem = WgCfg<128, 32, 32>::smem_bytes(pro ? a.Cin : 0); break;
    case 1: bkr = 128; bc = 64; smem = WgCfg<128, 64, 32>::smem_bytes(pro ? a.Cin : 0); break;
    case 2: bkr = 128; bc = 128; smem = WgCfg<128, 128, 32>::smem_bytes(pro ? a.Cin : 0); break;
    default: smem = WgCfg<64, 128, 32>::smem_bytes(pro ? a.Cin : 0); break;
  }
  e.a = a;
  e.gx = (K + bkr - 1) / bkr;
  e.gy = (a.Cout + bc - 1) / bc;
  e.gz = splits;
  return e.gx * e.gy * e.gz;
}

hipError_t wgrad_batch(const WgBatchEntry* list, const int* begins, int n, int total, int sig, long long smem,
                       hipStream_t st) {
  if (n <= 0 || total <= 0) return hipSuccess;
  if (n > WG_BATCH_MAX || list == nullptr || begins == nullptr || smem > 160 * 1024) return hipErrorInvalidValue;
  const size_t shm = (size_t)smem;
  if (sig == 1) {
    hipLaunchKernelGGL(wgrad3x3_img_batch_kernel, ggrid(total), dim3(256), shm, st, list, begins, garg());
    return hipGetLastError();
  }
  if (sig < 16 || sig >= 32) return hipErrorInvalidValue;
  const int tile = (sig - 16) / 4, is1x1 = (sig >> 1) & 1, pro = sig & 1;
#define IDC_WB(BKR, BC, WM, WN)                                                                              \
  {                                                                                                          \
    if (is1x1) {                                                                                             \
      if (pro) hipLaunchKernelGGL((conv_wgrad_batch_kernel<BKR, BC, 32, WM, WN, true, 1>), ggrid(total),     \
                                  dim3(256), shm, st, list, begins, garg());                                 \
      else hipLaunchKernelGGL((conv_wgrad_batch_kernel<BKR, BC, 32, WM, WN, true, 0>), ggrid(total),         \
                              dim3(256), shm, st, list, begins, garg());                                     \
    } else {                                                                                                 \
      if (pro) hipLaunchKernelGGL((conv_wgrad_batch_kernel<BKR, BC, 32, WM, WN, false, 1>), ggrid(total),    \
                                  dim3(256), shm, st, list, begins, garg());                                 \
      else hipLaunchKernelGGL((conv_wgrad_batch_kernel<BKR, BC, 32, WM, WN, false, 0>), ggrid(total),        \
                              dim3(256), shm, st, list, begins, garg());                                     \
    }                                                                                                        \
  }
  switch (tile) {
    case 0: IDC_WB(128, 32, 4, 1) break;
    case 1: IDC_WB(128, 64, 2, 2) break;
    case 2: IDC_WB(128, 128, 2, 2) break;
    default: IDC_WB(64, 128, 2, 2) break;
  }
#undef IDC_WB
  return hipGetLastError();
}

int wgrad_pick_splits(int M, int K, int Cout) {
  int tiles;
  if (Cout <= 32) tiles = ((K + 127) / 128) * ((Cout + 31) / 32);
  else if (Cout <= 64) tiles = ((K + 127) / 128) * ((Cout + 63) / 64);
  else if (wgrad_big_on() && Cout >= 128 && K >= 512 && M <= 16384) tiles = ((K + 127) / 128) * ((Cout + 127) / 128);
  else tiles = ((K + 63) / 64) * ((Cout + 127) / 128);
  int target = 512;  // ~2 blocks per CU
  int s = (target + tiles - 1) / tiles;
  const int bp = wgrad_bp(Cout);
  int maxs = (M + 8 * bp - 1) / (8 * bp);  // at least 8 k-steps per slice
  if (s > maxs) s = maxs;
  return s < 1 ? 1 : s;
}

}  // namespace idc
