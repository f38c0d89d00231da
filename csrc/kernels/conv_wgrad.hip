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

template <int BKR, int BC, int BP_, int WM, int WN, bool IS1X1, typename TG, int PRO, int GPRO>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  prefetch_kernargs<sizeof(WgradArgs)>();
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

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.KH * a.KW * a.Cin;
  const int k0 = blockIdx.x * BKR;
  const int c0 = blockIdx.y * BC;
  const int per = a.pix_per_split;
  const int pbeg = blockIdx.z * per;
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
    if (a.part) a.part[(size_t)blockIdx.z * ((size_t)a.KH * a.KW * (a.cin_real ? a.cin_real : a.Cin) * a.Cout) +
                       (size_t)kdst * a.Cout + co] = v;
    else atomicAdd(&a.dw[(size_t)kdst * a.Cout + co], v);
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                           long long n, int splits) {
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
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((int)b), dim3(256), 0, st, part, dw, n, splits);
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
  hipLaunchKernelGGL((conv_wgrad_kernel<BKR, BC, BP, WM, WN, IS1, TG, P, GP>), grid, dim3(256), shm, st, a)
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

hipError_t conv_wgrad(WgradArgs a, int splits, bool g_f32, hipStream_t st) {
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
  return launch_wg<64, 128, 32, 2, 2>(a, is1x1, g_f32, pro, splits, st);
}

int wgrad_effective_splits(const WgradArgs& a, int splits) {
  const int M = a.N * a.Ho * a.Wo;
  if (splits < 1) splits = 1;
  const int bp = wgrad_bp(a.Cout);
  int per = (M + splits - 1) / splits;
  per = (per + bp - 1) / bp * bp;
  return (M + per - 1) / per;
}

int wgrad_pick_splits(int M, int K, int Cout) {
  int tiles;
  if (Cout <= 32) tiles = ((K + 127) / 128) * ((Cout + 31) / 32);
  else if (Cout <= 64) tiles = ((K + 127) / 128) * ((Cout + 63) / 64);
  else tiles = ((K + 63) / 64) * ((Cout + 127) / 128);
  int target = 512;  // ~2 blocks per CU
  int s = (target + tiles - 1) / tiles;
  const int bp = wgrad_bp(Cout);
  int maxs = (M + 8 * bp - 1) / (8 * bp);  // at least 8 k-steps per slice
  if (s > maxs) s = maxs;
  return s < 1 ? 1 : s;
}

}  // namespace idc
