// (conv_igemm_impl.h: kernel template + launcher, instantiated per tile group by
// conv_igemm_g*.hip so the variants compile in parallel; dispatch lives in conv_igemm.hip)
//
// Implicit-GEMM convolution on MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, gfx950.
//
// out[m, n] = sum_k A[m, k] * Wt[n, k]
//   m = (img, ho, wo)  in [0, M = N*Ho*Wo)
//   n = output channel in [0, Cout)
//   k = (r, s, c)      in [0, K = KH*KW*Cin)   (Cin % 8 == 0: one 16-B chunk never straddles (r,s))
//   A[m, k] = act(bn(x[img, ho*SH-PT+r, wo*SW-PL+s, c]))   (0 outside the image: padding is
//             applied AFTER the activation, as Keras' ZeroPadding/'same' conv does)
//
// Used for: every forward conv (3x3 s1 'same', 1x1, 7x7 s2 stem, 3x3 s2), and every stride-1
// dgrad (a conv of dY with the spatially flipped, in/out-transposed kernel prepared by the
// optimizer's cast kernel).
//
// Prologue (PRO=1): "pending BN" — the operand is the RAW output of a producer conv plus that
// producer's batch statistics; the BN affine + ReLU/ReLU6 is applied while staging the tile in
// LDS, so pre-activation DenseNet / post-activation MobileNetV2 need no
// standalone BN or activation kernels.
// Epilogue EPI=0: bias + activation, bf16/fp32 store into a channel slice of a wider buffer,
//   optional per-channel [sum|sumsq] of the stored values (the NEXT BN's batch statistics,
//   accumulated with one atomic per channel per block).
// Epilogue EPI=1 (backward through a BN+act that fed this conv's forward input): the GEMM value
//   is dA; dZ = dA * act'(z) with z recomputed from the saved forward input x; stores dZ (bf16)
//   and accumulates sum(dZ) (= dbeta, or the previous conv's dbias) and sum(dZ*xhat) (= dgamma).
//
// Tiling: BM x BN x BK block tile, 4 waves in a WM x WN grid, each wave (BM/WM) x (BN/WN) of 16x16
// MFMA fragments.  Global -> registers -> (prologue) -> LDS double buffer, one barrier per K-step;
// LDS chunk XOR swizzle verified conflict-free for ds_read_b128 fragment reads and ds_write_b128.
// The epilogue stages the fp32 tile through LDS so global stores (and the epilogue loads of x)
// are 16-byte coalesced.  Block ids are remapped XCD-aware (guide §5 T1).
#pragma once
#include "common.h"
#include "conv_igemm.h"

// phase timestamps for tools/micro/conv_phases.hip (compiled out everywhere else)
#ifndef IDC_PHASE_STAMP
#define IDC_PHASE_STAMP(i)
#endif

namespace idc {

template <int BK>
__device__ __forceinline__ int swz_chunk(int row, int chunk) {
  if constexpr (BK == 32) return chunk ^ (((row >> 2) & 1) << 1);
  else if constexpr (BK == 64) return chunk ^ (row & 6);
  else return chunk ^ (row & 15);  // BK 128 / 256: XOR within 16-chunk groups (brute-force checked)
}

template <int BM, int BN, int BK, int WM, int WN>
struct IgemmCfg {
  static constexpr int NT = 256;
  static constexpr int CPR = BK / 8;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  static constexpr int STAGE_BYTES = 2 * (A_ELEMS + B_ELEMS) * 2;
  static constexpr int CS_LD = BN + 4;
  // epilogue staging: the whole fp32 tile in one pass when it fits the staging buffers (or 20 KB),
  // else one wave-row of the tile per pass
  static constexpr int FULL_BYTES = BM * CS_LD * 4;
  static constexpr int NPASS = FULL_BYTES <= (STAGE_BYTES > 20480 ? STAGE_BYTES : 20480) ? 1 : WM;
  static constexpr int PROWS = BM / NPASS;
  static constexpr int EPI_BYTES = PROWS * CS_LD * 4;
  // statistics: every thread's 16 partials, transposed reduction (row stride 20 floats)
  static constexpr int RED_LD = 20;
  static constexpr int RED_BYTES = NT * RED_LD * 4;
  static constexpr int MAIN0 = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  static constexpr int MAIN = MAIN0 > RED_BYTES ? MAIN0 : RED_BYTES;
  static int smem_bytes(int cpro) {
    int t = (cpro + 3) / 4 * 4;
    return MAIN + 3 * t * 4 + 10 * BN * 4;
  }
};

template <int BM, int BN, int BK, int WM, int WN, bool IS1X1, typename TA, int PRO, int EPI>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a, GroupArg ga) {
  IDC_PHASE_STAMP(0);
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  using C = IgemmCfg<BM, BN, BK, WM, WN>;
  constexpr int NT = C::NT, CPR = C::CPR, WTM = C::WTM, WTN = C::WTN;
  constexpr int NA = (BM * CPR + NT - 1) / NT;  // A chunks per thread
  constexpr int NB = (BN * CPR + NT - 1) / NT;  // B chunks per thread
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_ELEMS = C::A_ELEMS, B_ELEMS = C::B_ELEMS, CS_LD = C::CS_LD;
  static_assert(TM >= 1 && TN >= 1, "bad wave tile");
  static_assert(NT / (2 * BN) <= 4 && NT % (2 * BN) == 0, "statistics reducer layout");
  static_assert(NT % CPR == 0, "chunk mapping");
  static_assert(BN <= NT, "one epilogue channel per thread in the table builders");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + 2 * A_ELEMS;
  float* Cs = reinterpret_cast<float*>(smem);
  const int cpro = PRO ? (a.Cin + 3) / 4 * 4 : 0;
  const bf16_t* __restrict__ XB = a.bpro.x;  // PRO 2: the BatchNorm's forward input
  float* s_scale = reinterpret_cast<float*>(smem + C::MAIN);
  float* s_shift = s_scale + cpro;
  float* s_third = s_shift + cpro;  // PRO 2: the C coefficients (s_scale = A, s_shift = B)
  float* s_sum = s_third + cpro;
  float* s_sq = s_sum + BN;
  float* s_e0 = s_sq + BN;
  float* s_e1 = s_e0 + BN;
  float* s_e2 = s_e1 + BN;
  float* s_e3 = s_e2 + BN;
  float* s_pa = s_e3 + BN;  // EPI 2: pending coefficients of the previous BatchNorm
  float* s_pb = s_pa + BN;
  float* s_pc = s_pb + BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int wr = wid / WN, wc = wid % WN;

  const int M = a.N * a.Ho * a.Wo;
  const int K = a.KH * a.KW * a.Cin;
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int mtiles = (M + BM - 1) / BM;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  // the slices of one output tile are consecutive logical ids -> same XCD under the remap, so the
  // reducer reads same-XCD partials (a speed choice only: the hand-off is placement independent)
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles * nsplit);
  const int tile = bid / nsplit, slice = bid - tile * nsplit;
  const int mt = tile / ntiles, nt = tile % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk_all = (K + BK - 1) / BK;
  const int per_slice = (nk_all + nsplit - 1) / nsplit;
  const int kt_begin = slice * per_slice;
  const int nk = max(0, min(nk_all, kt_begin + per_slice) - kt_begin);
  const bool aout_on = PRO == 2 && a.aout != nullptr && nt == 0;

  // ---- per-thread A row decode (fixed for the whole K loop) -------------------------------
  const int my_chunk = tid % CPR;  // the k-chunk this thread stages (same for all its rows)
  int a_img[NA], a_h0[NA], a_w0[NA];
  bool a_ok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    int idx = tid + i * NT;
    int row = idx / CPR;
    int m = m0 + row;
    a_ok[i] = (idx < BM * CPR) && (m < M);
    int mm = a_ok[i] ? m : 0;
    if constexpr (IS1X1) {
      a_img[i] = mm; a_h0[i] = 0; a_w0[i] = 0;
    } else {
      int wo = mm % a.Wo;
      int t = mm / a.Wo;
      int ho = t % a.Ho;
      a_img[i] = t / a.Ho;
      a_h0[i] = ho * a.SH - a.PT;
      a_w0[i] = wo * a.SW - a.PL;
    }
  }
  int kglob = kt_begin * BK + my_chunk * 8;  // global k of this thread's chunk in the current tile
  int kc = kglob, kr = 0, ks = 0;
  if constexpr (!IS1X1) {
    while (kc >= a.Cin) { kc -= a.Cin; if (++ks == a.KW) { ks = 0; ++kr; } }
  }

  const TA* __restrict__ X = reinterpret_cast<const TA*>(a.x);
  const bf16_t* __restrict__ Wt = a.w;
  const float pro_lo = act_lo(a.pro.act), pro_hi = act_hi(a.pro.act);
  const float epi_lo = act_lo(a.epi_act), epi_hi = act_hi(a.epi_act);
  const float msk_lo = act_lo(a.mbn.act), msk_hi = act_hi(a.mbn.act);

  // NS staging register sets, tile t in set t % NS: tile t+NS is issued while tile t is computed
  // from LDS and tile t+1 waits in registers to be written, so each global load has NS-1 compute
  // phases to land.  The small tiles (the DenseNet layers: a few MFMAs per K-step against a
  // ~2k-cycle load latency) take 4 sets, the big ones 2 (register budget).
  struct Stage {
    uint4 ra[NA];
    uint4 rx[PRO == 2 ? NA : 1];
    int rp[PRO == 2 ? NA : 1];  // pixel of each A chunk (operand side output)
    bool rvalid[NA];
    float rpre[sizeof(TA) == 4 ? NA : 1][8];
    uint4 rb[NB];
    bool bvalid[NB];
    int kc, kr, ks;
  };
  constexpr int STAGE_VGPR = NA * (sizeof(TA) == 4 ? 9 : 5) + (PRO == 2 ? NA * 5 : 0) + NB * 5;
  constexpr int NS = 2;  // 4 sets measured slower: the small-tile K loop is issue-bound, not load-latency-bound
  (void)STAGE_VGPR;
  Stage st[NS];

  auto load_tile = [&](Stage& S) {
    uint4* ra = S.ra;
    bool* rvalid = S.rvalid;
    auto& rpre = S.rpre;
    uint4* rb = S.rb;
    S.kc = kc;
    S.kr = kr;
    S.ks = ks;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      bool ok = a_ok[i] && (kglob < K);
      size_t pix = 0;
      if constexpr (IS1X1) {
        pix = (size_t)a_img[i];
      } else {
        int h = a_h0[i] + kr, w = a_w0[i] + ks;
        ok = ok && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        pix = (size_t)(a_img[i] * a.H + h) * a.W + w;
      }
      // unconditional loads from a clamped address: a guarded "ok ? load : 0" makes hipcc branch
      // around each load and drain vmcnt(0), which destroys the two-deep prefetch
      rvalid[i] = ok;
      pix = ok ? pix : 0;
      const size_t off = pix * a.ldx + kc;
      if constexpr (PRO == 2) {
        S.rx[i] = *reinterpret_cast<const uint4*>(XB + pix * a.bpro.ldx + kc);
        S.rp[i] = (int)pix;
      }
      if constexpr (sizeof(TA) == 2) {
        ra[i] = *reinterpret_cast<const uint4*>(X + off);
      } else {
        float4 u = *reinterpret_cast<const float4*>(X + off);
        float4 v = *reinterpret_cast<const float4*>(X + off + 4);
        rpre[i][0] = u.x; rpre[i][1] = u.y; rpre[i][2] = u.z; rpre[i][3] = u.w;
        rpre[i][4] = v.x; rpre[i][5] = v.y; rpre[i][6] = v.z; rpre[i][7] = v.w;
      }
    }
    const int k0 = kglob - my_chunk * 8;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int idx = tid + i * NT;
      int row = idx / CPR, ch = idx % CPR;
      int n = n0 + row;
      int k = k0 + ch * 8;
      bool ok = (idx < BN * CPR) && (n < a.Cout) && (k < K);
      S.bvalid[i] = ok;
      rb[i] = *reinterpret_cast<const uint4*>(Wt + (ok ? (size_t)n * K + k : 0));
    }
  };

  auto store_tile = [&](Stage& S, int buf) {
    bf16_t* as = As + buf * A_ELEMS;
    bf16_t* bs = Bs + buf * B_ELEMS;
    const uint4* ra = S.ra;
    const bool* rvalid = S.rvalid;
    const auto& rpre = S.rpre;
    const uint4* rb = S.rb;
    const int kc = S.kc;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int idx = tid + i * NT;
      if (idx >= BM * CPR) break;
      int row = idx / CPR, ch = idx % CPR;
      // branch-free: transform unconditionally, then select zero for padding / tails (an
      // exec-masked branch per chunk costs a scalar branch + waitcnt split per chunk)
      uint4 v;
      if constexpr (PRO == 2) {
        float f[8], xf[8];
        if constexpr (sizeof(TA) == 2) {
          unpack8(ra[i], f);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = rpre[i][j];
        }
        unpack8(S.rx[i], xf);
        bwd_aff8(f, xf, s_scale + kc, s_shift + kc, s_third + kc);
        v = pack8(f);
        if (aout_on && rvalid[i] && (IS1X1 || (S.kr == a.PT && S.ks == a.PL)))
          *reinterpret_cast<uint4*>(a.aout + (size_t)S.rp[i] * a.ldaout + kc) = v;
      } else if constexpr (sizeof(TA) == 2) {
        if constexpr (PRO) {
          float f[8];
          unpack8(ra[i], f);
          affine_act8(f, s_scale + kc, s_shift + kc, pro_lo, pro_hi);
          v = pack8(f);
        } else {
          v = ra[i];
        }
      } else {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = rpre[i][j];
        if constexpr (PRO) affine_act8(f, s_scale + kc, s_shift + kc, pro_lo, pro_hi);
        v = pack8(f);
      }
      const bool ok = rvalid[i];
      v.x = ok ? v.x : 0u;
      v.y = ok ? v.y : 0u;
      v.z = ok ? v.z : 0u;
      v.w = ok ? v.w : 0u;
      *reinterpret_cast<uint4*>(as + row * BK + swz_chunk<BK>(row, ch) * 8) = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int idx = tid + i * NT;
      if (idx >= BN * CPR) break;
      int row = idx / CPR, ch = idx % CPR;
      const bool ok = S.bvalid[i];
      uint4 v = rb[i];
      v.x = ok ? v.x : 0u;
      v.y = ok ? v.y : 0u;
      v.z = ok ? v.z : 0u;
      v.w = ok ? v.w : 0u;
      *reinterpret_cast<uint4*>(bs + row * BK + swz_chunk<BK>(row, ch) * 8) = v;
    }
  };

  auto advance_k = [&]() {
    kglob += BK;
    kc += BK;
    if constexpr (!IS1X1) {
      while (kc >= a.Cin) { kc -= a.Cin; if (++ks == a.KW) { ks = 0; ++kr; } }
    }
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  // the first two tiles are issued BEFORE the prologue tables are built: the tables' own global
  // loads (BN statistics, gamma, beta) then overlap the tile loads instead of adding a second
  // full memory latency in front of the K loop
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s) advance_k();
    load_tile(st[s]);
  }
  IDC_PHASE_STAMP(1);
  // ---- prologue tables ----
  if constexpr (PRO == 1) bn_coeff_table<NT>(a.pro, a.Cin, s_scale, s_shift);
  // backward tables (pending-affine prologue, epilogue BatchNorm, epilogue pending affine): one
  // batched round trip when every statistic has <= 4 slot copies (common.h "Batched table inputs")
  // (compiled into the small-accumulator tiles only: they are the ones small layers pick, and the
  // extra live registers made the big tiles spill)
  bool batched = false;
  if constexpr ((PRO == 2 || EPI >= 1) && TM * TN <= 8) {
    batched = (PRO != 2 || (a.Cin <= NT && (!a.bpro.mode || (a.bpro.bn.mode == 1 && bwd_aff_slots4(a.bpro))))) &&
              (EPI != 2 || !a.bepi.mode || (a.bepi.bn.mode == 1 && bwd_aff_slots4(a.bepi))) &&
              (EPI < 1 || bn_slots4(a.mbn));
  }
  if (batched) {
    const int cp = tid < a.Cin ? tid : 0;           // PRO 2 channel of this thread
    const int ce = n0 + tid < a.Cout ? n0 + tid : 0;  // epilogue channel (BN <= NT)
    BwdAffRaw rp, re2;
    Raw4 rm;
    float mg = 1.f, mb = 0.f, mk = 0.f;
    if constexpr (PRO == 2) {
      if (a.bpro.mode) bwd_aff_load(a.bpro, cp, rp);
    }
    if constexpr (EPI == 2) {
      if (a.bepi.mode) bwd_aff_load(a.bepi, ce, re2);
    }
    if constexpr (EPI >= 1) {
      if (a.mbn.mode == 1) {
        load4(a.mbn.stats, a.mbn.stats + a.mbn.C, stat_slots(a.mbn.slots), 2 * (size_t)a.mbn.C, ce, rm);
        mk = bn_shift(a.mbn, ce);
      }
      else if (a.mbn.mode == 2) { rm.a0[0] = a.mbn.mmean[ce]; rm.a1[0] = a.mbn.mvar[ce]; }
      if (a.mbn.mode) {
        mg = a.mbn.gamma ? a.mbn.gamma[ce] : 1.f;
        mb = a.mbn.beta ? a.mbn.beta[ce] : 0.f;
      }
    }
    if constexpr (PRO == 2) {
      if (tid < a.Cin) {
        float A = 1.f, B = 0.f, Cc = 0.f;
        if (a.bpro.mode) bwd_aff_finish(a.bpro, rp, A, B, Cc);
        s_scale[tid] = A; s_shift[tid] = B; s_third[tid] = Cc;
      }
    }
    if (tid < BN) {
      if constexpr (EPI == 2) {
        float A = 1.f, B = 0.f, Cc = 0.f;
        if (a.bepi.mode && n0 + tid < a.Cout) bwd_aff_finish(a.bepi, re2, A, B, Cc);
        s_pa[tid] = A; s_pb[tid] = B; s_pc[tid] = Cc;
      }
      if constexpr (EPI >= 1) {
        float sc = 1.f, sh = 0.f, mean = 0.f, rstd = 1.f;
        if (n0 + tid < a.Cout && a.mbn.mode) {
          float v0, v1 = rm.a1[0];
          if (a.mbn.mode == 1) {
            sum4(rm, stat_slots(a.mbn.slots), v0, v1);
            shifted_mean_var(mk, v0, v1, a.mbn.inv_count, mean, v1);
          } else {
            mean = rm.a0[0];
          }
          rstd = rsqrtf(v1 + a.mbn.eps);
          sc = mg * rstd;
          sh = mb - mean * sc;
        }
        s_e0[tid] = sc; s_e1[tid] = sh; s_e2[tid] = mean; s_e3[tid] = rstd;
      }
    }
  } else {
    if constexpr (PRO == 2) bwd_aff_table<NT>(a.bpro, 0, a.Cin, a.Cin, s_scale, s_shift, s_third);
    IDC_PHASE_STAMP(2);
    if constexpr (EPI == 2) bwd_aff_table<NT>(a.bepi, n0, BN, a.Cout, s_pa, s_pb, s_pc);
    IDC_PHASE_STAMP(3);
    if constexpr (EPI >= 1) {
      for (int j = tid; j < BN; j += NT) {
        int c = n0 + j;
        float sc = 1.f, sh = 0.f, mean = 0.f, rstd = 1.f;
        if (c < a.Cout && a.mbn.mode) {
          bn_mean_rstd(a.mbn, c, mean, rstd);
          const float g = a.mbn.gamma ? a.mbn.gamma[c] : 1.f;
          const float be = a.mbn.beta ? a.mbn.beta[c] : 0.f;
          sc = g * rstd;
          sh = be - mean * sc;
        }
        s_e0[j] = sc; s_e1[j] = sh; s_e2[j] = mean; s_e3[j] = rstd;
      }
    }
  }
  if constexpr (PRO == 2) bwd_aff_fold<NT>(a.bpro);
  IDC_PHASE_STAMP(4);

  // Epilogue operands (the forward input x for the activation mask / x-hat, and the old fp32
  // accumulator of epilogue 2) do not depend on the GEMM: issue them now, youngest of all, so
  // their memory latency hides under the K loop instead of adding a dependent round trip after
  // it (the small late-stage GEMMs are latency chains).  Up to 4 chunks per thread.
  constexpr int CPB = BN / 8;
  constexpr int NPASS = C::NPASS, PROWS = C::PROWS;
  constexpr int EPI_IT = (PROWS * CPB + NT - 1) / NT;
  constexpr bool EPF = (EPI >= 1) && (NPASS * EPI_IT <= 4);
  constexpr int NEP = EPF ? NPASS * EPI_IT : 1;
  uint4 ep_x[NEP];
  float4 ep_o0[EPI == 2 ? NEP : 1], ep_o1[EPI == 2 ? NEP : 1];
  if constexpr (EPF) {
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass)
#pragma unroll
      for (int it = 0; it < EPI_IT; ++it) {
        const int idx = tid + it * NT;
        const int lrow = idx / CPB, c8 = idx % CPB;
        const int m = m0 + pass * PROWS + lrow, n = n0 + c8 * 8;
        const bool ok = idx < PROWS * CPB && m < M && n < a.Cout;
        const size_t mm = ok ? (size_t)m : 0, nn = ok ? (size_t)n : 0;
        ep_x[pass * EPI_IT + it] = *reinterpret_cast<const uint4*>(a.mx + mm * a.ldmx + nn);
        if constexpr (EPI == 2) {
          const float* yp = reinterpret_cast<const float*>(a.y) + mm * a.ldy + nn;
          ep_o0[pass * EPI_IT + it] = *reinterpret_cast<const float4*>(yp);
          ep_o1[pass * EPI_IT + it] = *reinterpret_cast<const float4*>(yp + 4);
        }
      }
  }

  IDC_PHASE_STAMP(5);
  __syncthreads();  // prologue tables visible
  store_tile(st[0], 0);
  __syncthreads();
  IDC_PHASE_STAMP(6);

  const int frow = lane & 15;
  const int fk = lane >> 4;

  auto compute = [&](int buf) {
    const bf16_t* as = As + buf * A_ELEMS;
    const bf16_t* bs = Bs + buf * B_ELEMS;
#pragma unroll
    for (int q = 0; q < BK / 32; ++q) {
      v8bf af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int row = wr * WTM + i * 16 + frow;
        af[i] = *reinterpret_cast<const v8bf*>(as + row * BK + swz_chunk<BK>(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int row = wc * WTN + j * 16 + frow;
        bfr[j] = *reinterpret_cast<const v8bf*>(bs + row * BK + swz_chunk<BK>(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // step kt: LDS[kt&1] holds tile kt and sets (kt+1..kt+NS-1) % NS hold the next tiles; set
  // kt % NS is free (tile kt was stored last step) and receives tile kt+NS.  Loads are
  // unconditional (tiles past the end are clamped and zero-filled, never stored): conditional
  // load/store pairs made the waitcnt pass drain vmcnt(0) at the back-edge.  Stores past the end
  // are skipped, so no step waits for a load it does not use.  Every step ends with a barrier
  // (the epilogue's fp32 staging tile aliases the LDS buffers).
  for (int kb = 0; kb < nk; kb += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int kt = kb + u;
      if (kt >= nk) break;
      advance_k();
      load_tile(st[u]);
      compute(u & 1);
      if (kt + 1 < nk) store_tile(st[(u + 1) % NS], (u + 1) & 1);
      __syncthreads();
    }
  }
  IDC_PHASE_STAMP(7);

  // ---- split-K: publish this slice's partial tile; the last arriver of the tile reduces ------
  // (guide §5 "In-launch split-K reduction": plain stores -> every wave vmcnt(0) -> barrier ->
  //  lane 0 agent release -> asm vmcnt(0) -> relaxed agent ticket; reducer: agent acquire ->
  //  asm vmcnt(0) -> barrier -> plain loads)
  if (nsplit > 1) {
    constexpr int NF = TM * TN;
    float4* slab = reinterpret_cast<float4*>(a.slab) + (size_t)tile * nsplit * NF * NT;
    {
      float4* mine = slab + (size_t)slice * NF * NT;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          mine[(i * TN + j) * NT + tid] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* s_flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev =
          __hip_atomic_fetch_add(&a.tickets[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (prev % (unsigned)nsplit) == (unsigned)(nsplit - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_flag[0] = last;
    }
    __syncthreads();
    const int last = s_flag[0];
    __syncthreads();  // the epilogue reuses this LDS
    if (!last) return;
    // sum the other slices, four at a time with every load issued before the adds
    for (int s0 = 0; s0 < nsplit; s0 += 4) {
      float4 v[4][NF];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int sl = s0 + u;
        const bool use = sl < nsplit && sl != slice;
        const float4* o = slab + (size_t)(use ? sl : slice) * NF * NT;
#pragma unroll
        for (int f = 0; f < NF; ++f) v[u][f] = use ? o[f * NT + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const float4 q = v[u][i * TN + j];
            acc[i][j][0] += q.x;
            acc[i][j][1] += q.y;
            acc[i][j][2] += q.z;
            acc[i][j][3] += q.w;
          }
    }
  }

  // ---- epilogue: NPASS passes, each stages PROWS x BN fp32 results in LDS -------------------
  const bool want_stats = (EPI >= 1) || (a.stats_out != nullptr);
  float psum[8], psq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { psum[j] = 0.f; psq[j] = 0.f; }
  // a thread's 8-channel chunk is the same in every pass (NT % CPB == 0): on the small tiles its
  // per-channel epilogue coefficients (and bias) are read once into registers; the big tiles
  // keep their accumulators live across passes and read them from LDS per element instead
  constexpr bool HOIST = TM * TN <= 8;
  const int my_c8 = tid % CPB;
  float t_e0[8], t_e1[8], t_e2[8], t_e3[8], t_pb[8], t_pc[8], t_bias[8], t_k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = n0 + my_c8 * 8 + j;
    t_k[j] = (EPI == 0 && a.stats_shift && c < a.Cout) ? a.stats_shift[c] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8 && HOIST; ++j) {
    const int cj = my_c8 * 8 + j;
    if constexpr (EPI >= 1) {
      t_e0[j] = s_e0[cj]; t_e1[j] = s_e1[cj]; t_e2[j] = s_e2[cj]; t_e3[j] = s_e3[cj];
    }
    if constexpr (EPI == 2) {
      t_pb[j] = s_pb[cj]; t_pc[j] = s_pc[cj];
    }
    if constexpr (EPI == 0) t_bias[j] = (a.bias && n0 + cj < a.Cout) ? a.bias[n0 + cj] : 0.f;
  }

#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass) __syncthreads();
    if (pass == 0) IDC_PHASE_STAMP(11);
    if ((wr * WTM) / PROWS == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          int col = wc * WTN + j * 16 + (lane & 15);
          int rbase = (wr * WTM) % PROWS + i * 16 + (lane >> 4) * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) Cs[(rbase + r) * CS_LD + col] = acc[i][j][r];
        }
    }
    __syncthreads();
    if (pass == 0) IDC_PHASE_STAMP(12);
#pragma unroll
    for (int it = 0; it < EPI_IT; ++it) {
      const int idx = tid + it * NT;
      if (idx >= PROWS * CPB) break;
      int lrow = idx / CPB, c8 = idx % CPB;
      int m = m0 + pass * PROWS + lrow, n = n0 + c8 * 8;
      if (m >= M || n >= a.Cout) continue;
      float v[8];
      const float4 lo = *reinterpret_cast<const float4*>(&Cs[lrow * CS_LD + c8 * 8]);
      const float4 hi = *reinterpret_cast<const float4*>(&Cs[lrow * CS_LD + c8 * 8 + 4]);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      if constexpr (EPI == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = v[j] + (HOIST ? t_bias[j] : (a.bias ? a.bias[n + j] : 0.f));
          v[j] = clampf(t, epi_lo, epi_hi);
        }
        if (a.out_mode == OUT_BF16) {
          uint4 p = pack8(v);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (size_t)m * a.ldy + n) = p;
          if (want_stats) {
            float r[8];
            unpack8(p, r);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float dj = r[j] - t_k[j];
              psum[j] += dj;
              psq[j] += dj * dj;
            }
          }
        } else {
          float* yp = reinterpret_cast<float*>(a.y) + (size_t)m * a.ldy + n;
          if (a.out_mode == OUT_F32_ACC) {
            const float4 o0 = *reinterpret_cast<const float4*>(yp);
            const float4 o1 = *reinterpret_cast<const float4*>(yp + 4);
            v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w;
            v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
          }
          *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
          if (want_stats) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float dj = v[j] - t_k[j];
              psum[j] += dj;
              psq[j] += dj * dj;
            }
          }
        }
      } else if constexpr (EPI == 2) {
        // dZ = dA * act'(z) in fp32; the concat gradient takes gamma*rstd*dZ plus the previous
        // BatchNorm's pending B'*x + C' (both on the same raw x)
        float* yp = reinterpret_cast<float*>(a.y) + (size_t)m * a.ldy + n;
        uint4 xv;
        float4 o0, o1;
        if constexpr (EPF) {
          xv = ep_x[pass * EPI_IT + it];
          o0 = ep_o0[pass * EPI_IT + it];
          o1 = ep_o1[pass * EPI_IT + it];
        } else {
          xv = *reinterpret_cast<const uint4*>(a.mx + (size_t)m * a.ldmx + n);
          o0 = *reinterpret_cast<const float4*>(yp);
          o1 = *reinterpret_cast<const float4*>(yp + 4);
        }
        const float old[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
        float xf[8], o[8];
        unpack8(xv, xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cj = c8 * 8 + j;
          const float e0 = HOIST ? t_e0[j] : s_e0[cj], e1 = HOIST ? t_e1[j] : s_e1[cj];
          const float e2 = HOIST ? t_e2[j] : s_e2[cj], e3 = HOIST ? t_e3[j] : s_e3[cj];
          const float pb = HOIST ? t_pb[j] : s_pb[cj], pc = HOIST ? t_pc[j] : s_pc[cj];
          const float z = xf[j] * e0 + e1;
          const float d = (z > msk_lo && z < msk_hi) ? v[j] : 0.f;
          psum[j] += d;
          psq[j] += d * (xf[j] - e2) * e3;
          o[j] = old[j] + fmaf(e0, d, fmaf(pb, xf[j], pc));
        }
        *reinterpret_cast<float4*>(yp) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(yp + 4) = make_float4(o[4], o[5], o[6], o[7]);
      } else if (a.out_mode != OUT_BF16) {
        // fp32 gradient of a BatchNorm OUTPUT that also feeds a residual (MobileNetV2 block
        // outputs): store (or accumulate into) dL/dy in fp32 and reduce that final value against
        // the BN input mx -- the BN's backward reductions without a separate reduce pass
        uint4 xv;
        if constexpr (EPF) xv = ep_x[pass * EPI_IT + it];
        else xv = *reinterpret_cast<const uint4*>(a.mx + (size_t)m * a.ldmx + n);
        float* yp = reinterpret_cast<float*>(a.y) + (size_t)m * a.ldy + n;
        if (a.out_mode == OUT_F32_ACC) {
          const float4 o0 = *reinterpret_cast<const float4*>(yp);
          const float4 o1 = *reinterpret_cast<const float4*>(yp + 4);
          v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w;
          v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
        }
        float xf[8];
        unpack8(xv, xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cj = c8 * 8 + j;
          const float z = xf[j] * (HOIST ? t_e0[j] : s_e0[cj]) + (HOIST ? t_e1[j] : s_e1[cj]);
          v[j] = (z > msk_lo && z < msk_hi) ? v[j] : 0.f;
          psum[j] += v[j];
          psq[j] += v[j] * (xf[j] - (HOIST ? t_e2[j] : s_e2[cj])) * (HOIST ? t_e3[j] : s_e3[cj]);
        }
        *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        uint4 xv;
        if constexpr (EPF) xv = ep_x[pass * EPI_IT + it];
        else xv = *reinterpret_cast<const uint4*>(a.mx + (size_t)m * a.ldmx + n);
        float xf[8], d[8];
        unpack8(xv, xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cj = c8 * 8 + j;
          float z = xf[j] * (HOIST ? t_e0[j] : s_e0[cj]) + (HOIST ? t_e1[j] : s_e1[cj]);
          d[j] = (z > msk_lo && z < msk_hi) ? v[j] : 0.f;
        }
        uint4 p = pack8(d);
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (size_t)m * a.ldy + n) = p;
        float r[8];
        unpack8(p, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cj = c8 * 8 + j;
          psum[j] += r[j];
          psq[j] += r[j] * (xf[j] - (HOIST ? t_e2[j] : s_e2[cj])) * (HOIST ? t_e3[j] : s_e3[cj]);
        }
      }
    }
  }
  IDC_PHASE_STAMP(8);
  if (want_stats) {
    // transposed reduction: every thread's 16 partials (its chunk's 8 column sums and sums of
    // squares) to LDS, then Q = NT/(2*BN) threads per output sum 16 contributions each in a fixed
    // order and combine over their quad with DPP; deterministic, two barriers, no shuffles
    __syncthreads();  // the staging tile is dead
    IDC_PHASE_STAMP(13);
    float* s_red = reinterpret_cast<float*>(smem);
    {
      float4* d = reinterpret_cast<float4*>(s_red + tid * C::RED_LD);
      d[0] = make_float4(psum[0], psum[1], psum[2], psum[3]);
      d[1] = make_float4(psum[4], psum[5], psum[6], psum[7]);
      d[2] = make_float4(psq[0], psq[1], psq[2], psq[3]);
      d[3] = make_float4(psq[4], psq[5], psq[6], psq[7]);
    }
    __syncthreads();
    IDC_PHASE_STAMP(14);
    constexpr int Q = NT / (2 * BN);
    const int o = tid / Q, q = tid % Q;
    const int kind = o / BN, col = o % BN;
    const int base = (col >> 3) * C::RED_LD + kind * 8 + (col & 7);
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) v += s_red[base + (i * Q + q) * CPB * C::RED_LD];
    if constexpr (Q >= 2) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
    if constexpr (Q >= 4) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    IDC_PHASE_STAMP(9);
    const int c = n0 + col;
    if (q == 0 && c < a.Cout) {
      if constexpr (EPI == 0) {
        const size_t so = (size_t)(mt % stat_slots(a.stats_slots)) * 2 * a.stats_ld;
        atomicAdd(&a.stats_out[so + (kind ? a.stats_ld : 0) + a.stats_off + c], v);
      } else {
        const size_t so = (size_t)(mt % stat_slots(a.gsum_slots)) * a.gsum_ld;
        float* g = kind ? a.gsumx : a.gsum;
        if (g) atomicAdd(&g[so + c], v);
      }
    }
  }
  IDC_PHASE_STAMP(10);
}

// ----------------------------------------------------------------------------------------------
// host-side dispatch
// ----------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
static inline hipError_t launch_cfg(const ConvArgs& a, bool is1x1, bool a_f32, int pro, int epi,
                             hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  const int tiles = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (a.ksplit > 1) {
    // the partial slabs and tickets of every tile must fit the workspace the caller provided
    if ((long long)tiles * a.ksplit * BM * BN > a.slab_floats || tiles > a.tickets_n) return hipErrorInvalidValue;
  }
  const int grid = tiles * (a.ksplit > 1 ? a.ksplit : 1);
  if (grid == 0) return hipSuccess;
  const size_t shm = IgemmCfg<BM, BN, BK, WM, WN>::smem_bytes(pro ? a.Cin : 0);
#define IDC_L(IS1, TA, P, E)                                                                   \
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, WM, WN, IS1, TA, P, E>), ggrid(grid),     \
                     dim3(256), shm, st, a, garg())
#define IDC_E(IS1, TA, P)      \
  if (epi == 0) IDC_L(IS1, TA, P, 0); \
  else IDC_L(IS1, TA, P, 1);
#define IDC_E3(IS1, TA, P)                  \
  if (epi == 0) IDC_L(IS1, TA, P, 0);      \
  else if (epi == 1) IDC_L(IS1, TA, P, 1); \
  else IDC_L(IS1, TA, P, 2);
  // epi 2 (concat-gradient accumulate) only follows a backward-affine prologue
  if (epi == 2 && pro != 2) return hipErrorInvalidValue;
  if (pro == 2) {
    if (a_f32) {
      if (is1x1) { IDC_E3(true, float, 2) } else { IDC_E3(false, float, 2) }
    } else {
      if (is1x1) { IDC_E3(true, bf16_t, 2) } else { IDC_E3(false, bf16_t, 2) }
    }
    return hipGetLastError();
  }
  // fp32 operands (gradient buffers) never carry a forward pending-BN prologue
  if (a_f32) {
    if (pro) return hipErrorInvalidValue;
    if (is1x1) { IDC_E(true, float, 0) } else { IDC_E(false, float, 0) }
  } else if (pro) {
    if (is1x1) { IDC_E(true, bf16_t, 1) } else { IDC_E(false, bf16_t, 1) }
  } else {
    if (is1x1) { IDC_E(true, bf16_t, 0) } else { IDC_E(false, bf16_t, 0) }
  }
#undef IDC_E3
#undef IDC_E
#undef IDC_L
  return hipGetLastError();
}

}  // namespace idc
