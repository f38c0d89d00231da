// Deep-ring small-tile implicit-GEMM convolution (forward, pending-BN prologue), gfx950.
//
// Phase stamps of the general kernel (conv_igemm_impl.h, tools/micro/conv_phases.hip) on the
// DenseNet tail layers show the K loop of a 64x32 tile at ~1,240 cycles per 64-deep step against
// ~100 cycles of MFMA work: each step waits for loads issued one step earlier (two VGPR staging
// sets), i.e. a CU pulls ~10 B/clk.  Deeper VGPR staging costs registers the small tiles cannot
// spare.  Here the operands go global -> LDS by DMA (global_load_lds_dwordx4, no VGPRs), into a
// ring of NS stages, so NS-1 K steps are in flight while one is computed:
//
//   * a K step is 64 channels of one tap (3x3 layers: Cin % 64 == 0) or, for 1x1 convolutions, 64
//     consecutive channels with the K tail (Cin % 64 != 0, DenseNet's 64 + 32k) read as zeros;
//     rows past M and padding taps load a 16-B zero block;
//   * the pending BatchNorm + activation of the operand (the PRODUCER's batch statistics; SURVEY
//     §7.3 item 2) is applied to each A fragment after its ds_read, before the MFMA (DMA lands raw
//     data), with padding taps forced to zero AFTER the activation (Keras pads the activated
//     tensor);
//   * one s_barrier per K step: a wave reaches the barrier of step k only after computing step
//     k-1, so the buffer of step k-1 is refilled (with step k+NS-1) right after it;
//   * LDS image lane-linear per DMA instruction (8 rows x 128 B) with the chunk XOR swizzle applied
//     to the per-lane SOURCE address (conv_big.hip, guide §5.4 rule 21);
//   * epilogue: the fp32 tile through LDS -> bias + activation -> 16-B bf16 stores, and the output
//     channels' shifted [sum | sumsq] for the next BatchNorm (wave DPP/shuffle reduction, one LDS
//     atomic per channel per wave, one global atomic per channel per workgroup).
// Used by the autotuner as tiles TILE_RING_* next to the general kernel's.
#include "common.h"
#include "conv_igemm.h"

namespace idc {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_ring_zero[8];  // zero-initialised padding source

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ int rswz(int row, int chunk) { return chunk ^ (row & 6); }

template <int BM_, int BN_, int NS_>
struct RingCfg {
  static constexpr int BM = BM_, BN = BN_, NS = NS_, BK = 64, NT = 256, NW = 4, WM = 2, WN = 2;
  static constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  static constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK, BUF = A_ELEMS + B_ELEMS;
  static constexpr int NGA = BM / 32, NGB = BN / 32;  // DMA instructions per wave per stage
  static constexpr int NG = NGA + NGB;
  static constexpr int RING_BYTES = NS * BUF * 2;
  static constexpr int CS_LD = BN + 4;
  static constexpr int STAGE_BYTES = BM * CS_LD * 4;
  static constexpr int MAIN = RING_BYTES > STAGE_BYTES ? RING_BYTES : STAGE_BYTES;
  static size_t smem_bytes(int ctab) { return MAIN + (size_t)(2 * ctab + 2 * BN) * 4; }
  static_assert(TM >= 1 && TN >= 1, "wave tile");
};

}  // namespace

template <int BM, int BN, int NS, bool IS1X1, int PRO>
__global__ __launch_bounds__(256) void conv_ring_kernel(ConvArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  using C = RingCfg<BM, BN, NS>;
  constexpr int BK = C::BK, NW = C::NW, TM = C::TM, TN = C::TN, WTM = C::WTM, WTN = C::WTN;
  constexpr int NGA = C::NGA, NGB = C::NGB, NG = C::NG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  const int Cin = a.Cin;
  const int K = a.KH * a.KW * Cin;
  const int nk = (K + BK - 1) / BK;
  const int ctab = PRO ? nk * BK : 0;  // tables cover the padded K tail (zeros there)
  float* s_scale = reinterpret_cast<float*>(smem + C::MAIN);
  float* s_shift = s_scale + ctab;
  float* s_sum = s_shift + ctab;
  float* s_sq = s_sum + BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / C::WN, wc = wid % C::WN;
  const int M = a.N * a.Ho * a.Wo;
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int mtiles = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  // ---- DMA source rows of this lane (fixed for the whole K loop) ---------------------------
  const int lrow = lane >> 3, pch = lane & 7;
  const int sch = pch ^ (lrow & 6);
  int a_pix[NGA], a_h0[NGA], a_w0[NGA];
  bool a_ok[NGA];
#pragma unroll
  for (int j = 0; j < NGA; ++j) {
    const int m = m0 + (j * NW + wid) * 8 + lrow;
    a_ok[j] = m < M;
    const int mm = a_ok[j] ? m : 0;
    if constexpr (IS1X1) {
      a_pix[j] = mm;
      a_h0[j] = a_w0[j] = 0;
    } else {
      const int wo = mm % a.Wo, t = mm / a.Wo, ho = t % a.Ho;
      a_pix[j] = (t / a.Ho) * a.H * a.W;  // image base pixel
      a_h0[j] = ho * a.SH - a.PT;
      a_w0[j] = wo * a.SW - a.PL;
    }
  }
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ Wt = a.w;
  const void* zsrc = g_ring_zero;

  auto issue = [&](int kt) {
    const int k0 = kt * BK;
    bf16_t* As = ring + (kt % NS) * C::BUF;
    bf16_t* Bs = As + C::A_ELEMS;
    int c0, kr = 0, ks = 0;
    if constexpr (IS1X1) {
      c0 = k0;
    } else {
      const int rs = k0 / Cin;
      c0 = k0 - rs * Cin;
      kr = rs / a.KW;
      ks = rs - kr * a.KW;
    }
    const int c = c0 + sch * 8;
#pragma unroll
    for (int j = 0; j < NGA; ++j) {
      const void* src;
      if constexpr (IS1X1) {
        src = (a_ok[j] && c < Cin) ? (const void*)(X + (size_t)a_pix[j] * a.ldx + c) : zsrc;
      } else {
        const int h = a_h0[j] + kr, w = a_w0[j] + ks;
        const bool ok = a_ok[j] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        src = ok ? (const void*)(X + ((size_t)a_pix[j] + h * a.W + w) * a.ldx + c) : zsrc;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(As + (j * NW + wid) * 8 * BK), 16, 0, 0);
    }
    const int kk = k0 + sch * 8;
#pragma unroll
    for (int j = 0; j < NGB; ++j) {
      const int n = n0 + (j * NW + wid) * 8 + lrow;
      const void* src = (n < a.Cout && kk < K) ? (const void*)(Wt + (size_t)n * K + kk) : zsrc;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(Bs + (j * NW + wid) * 8 * BK), 16, 0, 0);
    }
  };

  // the first NS-1 stages go out before the prologue tables are built: their latency hides the
  // tables' own loads
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);

  if constexpr (PRO) {
    bn_coeff_table<256>(a.pro, min(Cin, ctab), s_scale, s_shift);
    for (int c = Cin + tid; c < ctab; c += 256) {  // K tail: finite zeros (B is zero there too)
      s_scale[c] = 0.f;
      s_shift[c] = 0.f;
    }
  }
  for (int c = tid; c < BN; c += 256) {
    s_sum[c] = 0.f;
    s_sq[c] = 0.f;
  }

  // per-lane fragment rows: (h0, w0, image ok) of the output pixel each A fragment row is
  const int frow = lane & 15, fk = lane >> 4;
  int f_h0[TM], f_w0[TM];
  bool f_ok[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wr * WTM + i * 16 + frow;
    f_ok[i] = m < M;
    if constexpr (!IS1X1) {
      const int mm = f_ok[i] ? m : 0;
      const int wo = mm % a.Wo, ho = (mm / a.Wo) % a.Ho;
      f_h0[i] = ho * a.SH - a.PT;
      f_w0[i] = wo * a.SW - a.PL;
    } else {
      f_h0[i] = f_w0[i] = 0;
    }
  }
  const float plo = act_lo(a.pro.act), phi = act_hi(a.pro.act);
  const bool pro_bn = PRO && a.pro.mode != 0;

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // tables visible (no DMA waited here: a __syncthreads drains nothing we need)

  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once only the stages issued after it are outstanding
    const int after = min(NS - 2, nk - 1 - kt);
    if (after >= 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * NG) : "memory");
    else if (after == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * NG) : "memory");
    else if (after == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NG) : "memory");
    else if (after == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NG) : "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NG) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's stage-kt DMA landed; stage kt-1 fully consumed
    if (kt + NS - 1 < nk) issue(kt + NS - 1);  // into the buffer of stage kt-1
    const bf16_t* As = ring + (kt % NS) * C::BUF;
    const bf16_t* Bs = As + C::A_ELEMS;
    int cbase = kt * BK, kr = 0, ks = 0;
    if constexpr (!IS1X1) {
      const int rs = cbase / Cin;
      cbase -= rs * Cin;
      kr = rs / a.KW;
      ks = rs - kr * a.KW;
    }
    bool ok[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (IS1X1) {
        ok[i] = true;
      } else {
        const int h = f_h0[i] + kr, w = f_w0[i] + ks;
        ok[i] = f_ok[i] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      }
    }
#pragma unroll
    for (int q = 0; q < BK / 32; ++q) {
      v8bf af[TM], bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wc * WTN + j * 16 + frow;
        bfr[j] = *reinterpret_cast<const v8bf*>(Bs + row * BK + rswz(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wr * WTM + i * 16 + frow;
        const uint4 raw = *reinterpret_cast<const uint4*>(As + row * BK + rswz(row, q * 4 + fk) * 8);
        uint4 v = raw;
        if constexpr (PRO) {
          float f[8];
          unpack8(raw, f);
          const int c = (IS1X1 ? kt * BK : cbase) + q * 32 + fk * 8;
          if (pro_bn) {
            affine_act8(f, s_scale + c, s_shift + c, plo, phi);
          } else {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) f[jj] = clampf(f[jj], plo, phi);
          }
          v = pack8(f);
          if (!ok[i]) v = make_uint4(0u, 0u, 0u, 0u);  // padding AFTER the activation
        }
        af[i] = *reinterpret_cast<const v8bf*>(&v);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue --------------------------------------------------------------------------
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // ring dead: the fp32 tile is staged over it
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int CS_LD = C::CS_LD;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wc * WTN + j * 16 + frow;
      const int rb = wr * WTM + i * 16 + fk * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(rb + r) * CS_LD + col] = acc[i][j][r];
    }
  __syncthreads();
  constexpr int CPB = BN / 8, ITEMS = (BM * CPB + 255) / 256;
  const int my_c8 = tid % CPB;  // 256 % CPB == 0: a thread's channel chunk is fixed
  const float elo = act_lo(a.epi_act), ehi = act_hi(a.epi_act);
  const bool want_stats = a.stats_out != nullptr;
  float t_bias[8], t_k[8], ps[8], pq[8];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int n = n0 + my_c8 * 8 + jj;
    t_bias[jj] = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
    t_k[jj] = (a.stats_shift && n < a.Cout) ? a.stats_shift[n] : 0.f;
    ps[jj] = pq[jj] = 0.f;
  }
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) {
    const int idx = tid + it * 256;
    const int rr = idx / CPB;
    const int m = m0 + rr, n = n0 + my_c8 * 8;
    if (rr < BM && m < M && n < a.Cout) {
      float v[8];
      const float4 lo = *reinterpret_cast<const float4*>(Cs + rr * CS_LD + my_c8 * 8);
      const float4 hi = *reinterpret_cast<const float4*>(Cs + rr * CS_LD + my_c8 * 8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = clampf(v[jj] + t_bias[jj], elo, ehi);
      const uint4 p = pack8(v);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (size_t)m * a.ldy + n) = p;
      if (want_stats) {
        float r8[8];
        unpack8(p, r8);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float d = r8[jj] - t_k[jj];
          ps[jj] += d;
          pq[jj] += d * d;
        }
      }
    }
  }
  if (want_stats) {
    wave_reduce_chunks<CPB>(ps);
    wave_reduce_chunks<CPB>(pq);
    if (lane < CPB) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        atomicAdd(&s_sum[lane * 8 + jj], ps[jj]);
        atomicAdd(&s_sq[lane * 8 + jj], pq[jj]);
      }
    }
    __syncthreads();
    const size_t so = (size_t)(mt % stat_slots(a.stats_slots)) * 2 * a.stats_ld;
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c < a.Cout) {
        atomicAdd(&a.stats_out[so + a.stats_off + n0 + c], s_sum[c]);
        atomicAdd(&a.stats_out[so + a.stats_ld + a.stats_off + n0 + c], s_sq[c]);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
static bool ring_is1x1(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0;
}

bool conv_ring_ok(const ConvArgs& a, bool a_f32) {
  if (a_f32 || a.bpro.mode != 0 || a.epi_mode != 0 || a.out_mode != OUT_BF16) return false;
  if ((a.Cin % 8) || (a.ldx % 8) || (a.ldy % 8) || (a.Cout % 8)) return false;
  if (!ring_is1x1(a) && (a.Cin % 64)) return false;  // a K step is one tap
  const int K = a.KH * a.KW * a.Cin;
  if (a.pro.mode != 0 && ((K + 63) / 64) * 64 > 4096) return false;  // LDS tables
  if (a.stats_out != nullptr && a.stats_ld <= 0) return false;
  return true;
}

template <int BM, int BN, int NS>
static hipError_t ring_launch(const ConvArgs& a, hipStream_t st) {
  using C = RingCfg<BM, BN, NS>;
  const int M = a.N * a.Ho * a.Wo;
  const int grid = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (grid == 0) return hipSuccess;
  const int K = a.KH * a.KW * a.Cin;
  const bool pro = a.pro.mode != 0 || a.pro.act != ACT_NONE;
  const size_t shm = C::smem_bytes(pro ? ((K + 63) / 64) * 64 : 0);
  if (shm > 160 * 1024) return hipErrorInvalidValue;
  const bool is1 = ring_is1x1(a);
#define IDC_R(IS1, P) \
  hipLaunchKernelGGL((conv_ring_kernel<BM, BN, NS, IS1, P>), ggrid(grid), dim3(256), shm, st, a, garg())
  if (is1) {
    if (pro) IDC_R(true, 1); else IDC_R(true, 0);
  } else {
    if (pro) IDC_R(false, 1); else IDC_R(false, 0);
  }
#undef IDC_R
  return hipGetLastError();
}

hipError_t conv_ring(const ConvArgs& a, int variant, bool a_f32, hipStream_t st) {
  if (!conv_ring_ok(a, a_f32)) return hipErrorInvalidValue;
  switch (variant) {
    case 0: return ring_launch<64, 32, 6>(a, st);
    case 1: return ring_launch<64, 64, 6>(a, st);
    case 2: return ring_launch<32, 32, 8>(a, st);
    case 3: return ring_launch<32, 64, 8>(a, st);
    case 4: return ring_launch<64, 128, 4>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace idc
