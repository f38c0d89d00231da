// Image-resident 3x3 'same' convolution on MFMA (v_mfma_f32_16x16x32_bf16), gfx950.
//
// DenseNet's dense layers run their 3x3 convolutions on small maps (13x13, 6x6, 3x3 at 50x50
// input; 8x8 / 4x4 / 2x2 at 32x32) with fixed channel counts: forward 128 -> 32 (the bottleneck
// through BN + ReLU into the new slice), data gradient 32 -> 128 (the new slice's gradient back
// into the bottleneck).  The implicit-GEMM kernel (conv_igemm_impl.h) streams im2col tiles, so every
// input element is fetched, normalised and staged into LDS nine times and each K-step waits on a
// global load; on these layers it runs at 1-2.5 % MFMA (profiles/densenet121_bs256_pmc.md).
//
// Here one workgroup owns whole IMAGES: it stages the image once into LDS as a zero-bordered
// (H+2) x (W+2) pixel grid -- the prologue transform (pending BatchNorm + activation, or the
// backward pending affine of the DenseNet concat gradient) applied exactly once per element -- and
// the whole weight tensor (9 * CIN * COUT bf16, ~74 KB) next to it, then runs the complete K loop
// (9 taps x CIN) out of LDS with no global memory access: A fragments are rows of the padded grid
// (output pixel (h, w), tap (r, s) -> grid row (h + r) * (W + 2) + w + s), B fragments rows of the
// weight block.  Row strides carry 32 B of padding so the ds_read_b128 lane groups of the MFMA
// fragment layout never collide on a bank (MI355X_MICROARCH.md "LDS").
//
// Epilogues are those of conv_igemm (same ConvArgs, same numerics):
//   EPI 0 (forward): bf16 store into the output slice + per-channel shifted [sum | sumsq] of the
//          stored values (the next BatchNorm's statistics), one atomic per channel per workgroup;
//   EPI 1 (data gradient): dZ = dA * act'(mbn(mx)) stored bf16, sum(dZ) / sum(dZ * xhat) reduced
//          into gsum / gsumx; with the pending affine prologue (PRO 2) the staged operand is also
//          written once per pixel to `aout` (the side-lane weight gradient's bf16 input).
// Selected by the autotuner as conv tile TILE_IMG (conv_igemm.hip) where conv_img_ok() holds.
#include "conv_igemm.h"

// phase timestamps for tools/micro/img_phases.hip (compiled out everywhere else)
#ifndef IDC_IMG_STAMP
#define IDC_IMG_STAMP(i)
#endif

namespace idc {

namespace {

constexpr int NT = 256;

template <int CIN, int COUT>
struct ImgCfg {
  static constexpr int K = 9 * CIN;
  static constexpr int AS = CIN * 2 + 32;       // padded-grid row stride (bytes)
  static constexpr int RC = K / 8;              // 16-B chunks per weight row
  static constexpr int BS = K * 2;              // weight row stride (bytes; rows swizzled, see wswz)
  static constexpr int W_BYTES = COUT * BS;
  static constexpr int CPR = CIN / 8;           // 16-B chunks per grid row
  static constexpr int WCH = COUT * K / 8;      // 16-B weight chunks
  static constexpr int WPT = (WCH + NT - 1) / NT;
  static constexpr int CPB = COUT / 8;          // 8-channel output chunks per row
  static constexpr int CS_LD = COUT + 4;        // fp32 epilogue staging row (floats)
  static constexpr int RED_LD = 20;
};

template <int CIN, int COUT>
int img_smem_bytes(int H, int W, int rows_pad, int pro) {
  using C = ImgCfg<CIN, COUT>;
  const int grid_b = (H + 2) * (W + 2) * C::AS;
  int main_b = C::W_BYTES + grid_b;
  const int cs = rows_pad * C::CS_LD * 4;
  const int red = NT * C::RED_LD * 4;
  if (cs > main_b) main_b = cs;
  if (red > main_b) main_b = red;
  main_b = (main_b + 15) / 16 * 16;
  const int tables = (pro == 2 ? 3 * CIN : 2 * CIN) * 4 + 4 * COUT * 4;
  return main_b + tables;
}

// Weight rows are filled by LDS-DMA (global_load_lds: lane-linear destinations), so bank spreading
// is a chunk permutation within each row instead of padding.  B fragment lanes read 16 rows n at
// chunk c (+1 for the second quarter of the lanes); the permutation makes every ds_read_b128 lane
// group hit 16 distinct 16-B bank slots:
//   rows of 144 chunks (128 -> 32, slot = chunk mod 16): chunk c stored at c ^ (n & 15);
//   rows of 36 chunks (32 -> 128, slot = (4 n + chunk) mod 16): c ^ (((n >> 3) & 1) << 1).
template <int RC>
__device__ __forceinline__ int wswz(int n, int c) {
  if constexpr (RC % 16 == 0) return c ^ (n & 15);
  else return c ^ (((n >> 3) & 1) << 1);
}

typedef __attribute__((address_space(3))) void lds_void_t;

}  // namespace

// WM x WN waves (WM * WN = 4): a wave owns row fragments wr, wr + WM, ... (at most RPW) and the
// CPW = COUT / 16 / WN column fragments from wc * CPW.
template <int CIN, int COUT, int WM, int WN, int RPW, typename TA, int PRO, int EPI>
__global__ __launch_bounds__(256) void conv3x3_img_kernel(ConvArgs a, GroupArg ga) {
  IDC_IMG_STAMP(0);
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  using C = ImgCfg<CIN, COUT>;
  constexpr int CPW = COUT / 16 / WN;
  static_assert(WM * WN == 4 && CPW >= 1 && COUT % (16 * WN) == 0 && CIN % 32 == 0, "tiling");
  static_assert(NT % C::CPB == 0 && NT % (2 * COUT) == 0 && NT / (2 * COUT) <= 4, "epilogue layout");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sW = smem;
  char* sX = smem + C::W_BYTES;
  const int H = a.H, W = a.W, HW = H * W, HP = H + 2, WP = W + 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  // p / W for p < 256, W <= 13 as one multiply (exact: p * W < 2^16 / W)
  const unsigned wmul = (65536u + (unsigned)W - 1u) / (unsigned)W;
  auto divw = [&](int p) { return (int)(((unsigned)p * wmul) >> 16); };
  const int img = blockIdx.x;
  const int M = HW;                     // rows of this workgroup (one image)
  const int NR = (M + 15) / 16;         // row fragments
  const size_t row0 = (size_t)img * HW;  // first global pixel row
  // main region, then the prologue / epilogue coefficient tables
  int main_b = C::W_BYTES + HP * WP * C::AS;
  {
    const int cs = NR * 16 * C::CS_LD * 4, red = NT * C::RED_LD * 4;
    main_b = max(main_b, max(cs, red));
    main_b = (main_b + 15) / 16 * 16;
  }
  float* tA = reinterpret_cast<float*>(smem + main_b);  // PRO: scale | A
  float* tB = tA + CIN;                                 // PRO: shift | B
  float* tC = tB + CIN;                                 // PRO 2: C
  float* e0 = tA + (PRO == 2 ? 3 : 2) * CIN;            // EPI 1: sc, sh, mean, rstd
  float* e1 = e0 + COUT;
  float* e2 = e1 + COUT;
  float* e3 = e2 + COUT;

  // ---- 1. weights global -> LDS by DMA (L2-resident, shared by every workgroup), no VGPRs -----
  static_assert(C::WCH % NT == 0 && C::RC % 4 == 0, "weight DMA layout");
  const bf16_t* __restrict__ Wt = a.w;
#pragma unroll
  for (int i = 0; i < C::WPT; ++i) {
    const int d = (i * 4 + wid) * 64 + lane;  // destination chunk (lane-linear per wave instruction)
    const int n = d / C::RC, pos = d - (d / C::RC) * C::RC;
    const bf16_t* src = Wt + (size_t)n * C::K + wswz<C::RC>(n, pos) * 8;
    __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(sW + (size_t)(i * 4 + wid) * 64 * 16), 16, 0, 0);
  }
  IDC_IMG_STAMP(1);
  // ---- 2. image loads (interior pixels, 8-channel chunks), unconditional from clamped rows ----
  constexpr int MAXI = (13 * 13 * C::CPR + NT - 1) / NT;  // chunks per thread (maps up to 13 x 13)
  const int nchunk = HW * C::CPR;
  uint4 xr[MAXI];
  float4 xf0[sizeof(TA) == 4 ? MAXI : 1], xf1[sizeof(TA) == 4 ? MAXI : 1];
  uint4 xb[PRO == 2 ? MAXI : 1];
  const TA* __restrict__ X = reinterpret_cast<const TA*>(a.x);
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    const int q = tid + i * NT;
    const int qq = q < nchunk ? q : 0;
    const int p = qq / C::CPR, c8 = qq % C::CPR;
    const size_t gp = row0 + p;
    if constexpr (sizeof(TA) == 2) {
      xr[i] = *reinterpret_cast<const uint4*>(X + gp * a.ldx + c8 * 8);
    } else {
      xf0[i] = *reinterpret_cast<const float4*>(X + gp * a.ldx + c8 * 8);
      xf1[i] = *reinterpret_cast<const float4*>(X + gp * a.ldx + c8 * 8 + 4);
    }
    if constexpr (PRO == 2) xb[i] = *reinterpret_cast<const uint4*>(a.bpro.x + gp * a.bpro.ldx + c8 * 8);
  }
  IDC_IMG_STAMP(2);
  // ---- 3. coefficient tables (their loads overlap the ones above) --------------------------
  if constexpr (PRO == 1) bn_coeff_table<NT>(a.pro, CIN, tA, tB);
  if constexpr (PRO == 2) {
    bwd_aff_table<NT>(a.bpro, 0, CIN, CIN, tA, tB, tC);
    bwd_aff_fold<NT>(a.bpro);
  }
  if constexpr (EPI == 1) {
    for (int c = tid; c < COUT; c += NT) {
      float sc = 1.f, sh = 0.f, mean = 0.f, rstd = 1.f;
      if (a.mbn.mode) {
        bn_mean_rstd(a.mbn, c, mean, rstd);
        const float g = a.mbn.gamma ? a.mbn.gamma[c] : 1.f;
        const float be = a.mbn.beta ? a.mbn.beta[c] : 0.f;
        sc = g * rstd;
        sh = be - mean * sc;
      }
      e0[c] = sc; e1[c] = sh; e2[c] = mean; e3[c] = rstd;
    }
  }
  IDC_IMG_STAMP(3);
  // zero border rows of the padded grid (no loads)
  {
    const int nb = 2 * WP + 2 * H;  // border pixels
    for (int q = tid; q < nb * C::CPR; q += NT) {
      const int bp = q / C::CPR, c8 = q % C::CPR;
      int hp, wp;
      if (bp < WP) { hp = 0; wp = bp; }
      else if (bp < 2 * WP) { hp = HP - 1; wp = bp - WP; }
      else { const int k = bp - 2 * WP; hp = 1 + (k >> 1); wp = (k & 1) ? WP - 1 : 0; }
      *reinterpret_cast<uint4*>(sX + (hp * WP + wp) * C::AS + c8 * 16) = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __syncthreads();  // tables visible (and the weight DMA drained: vmcnt(0))
  IDC_IMG_STAMP(4);
  // ---- 5. transform the image once and stage it -------------------------------------------
  const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
  const bool aout_on = PRO == 2 && a.aout != nullptr;
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    const int q = tid + i * NT;
    if (q >= nchunk) continue;  // (no break: the register arrays must stay statically indexed)
    const int p = q / C::CPR, c8 = q % C::CPR;
    const int h = divw(p), w = p - h * W;
    float f[8];
    if constexpr (sizeof(TA) == 2) {
      unpack8(xr[i], f);
    } else {
      f[0] = xf0[i].x; f[1] = xf0[i].y; f[2] = xf0[i].z; f[3] = xf0[i].w;
      f[4] = xf1[i].x; f[5] = xf1[i].y; f[6] = xf1[i].z; f[7] = xf1[i].w;
    }
    uint4 v;
    if constexpr (PRO == 1) {
      affine_act8(f, tA + c8 * 8, tB + c8 * 8, lo, hi);
      v = pack8(f);
    } else if constexpr (PRO == 2) {
      float xv[8];
      unpack8(xb[i], xv);
      bwd_aff8(f, xv, tA + c8 * 8, tB + c8 * 8, tC + c8 * 8);
      v = pack8(f);
      if (aout_on) *reinterpret_cast<uint4*>(a.aout + (row0 + p) * a.ldaout + c8 * 8) = v;
    } else {
      v = sizeof(TA) == 2 ? xr[i] : pack8(f);
    }
    *reinterpret_cast<uint4*>(sX + ((h + 1) * WP + (w + 1)) * C::AS + c8 * 16) = v;
  }
  IDC_IMG_STAMP(5);
  // EPI 1: the forward input at the output positions, issued now so it lands under the K loop
  constexpr int EPP = (RPW * WM * 16 * C::CPB + NT - 1) / NT;
  uint4 ep_x[EPI == 1 ? EPP : 1];
  if constexpr (EPI == 1) {
#pragma unroll
    for (int it = 0; it < EPP; ++it) {
      const int idx = tid + it * NT;
      const int m = idx / C::CPB, c8 = idx % C::CPB;
      const int mm = m < M ? m : 0;
      ep_x[it] = *reinterpret_cast<const uint4*>(a.mx + (row0 + mm) * a.ldmx + c8 * 8);
    }
  }
  __syncthreads();

  IDC_IMG_STAMP(6);
  // ---- 6. K loop out of LDS ---------------------------------------------------------------
  int nrw = 0;  // row fragments of this wave (wave-uniform)
  int R0[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int fr = wr + WM * i;
    if (fr < NR) nrw = i + 1;
    const int m = fr * 16 + (lane & 15);
    const int h = divw(m < M ? m : 0), w = (m < M ? m : 0) - h * W;
    R0[i] = m < M ? h * WP + w : 0;  // (rows past the image read the zero border; not stored)
  }
  const int kc = lane >> 4;
  v4f acc[RPW][CPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  const int bn0 = wc * CPW * 16 + (lane & 15);  // this lane's B row for column fragment 0
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int r = tap / 3, s = tap % 3;
    const int toff = r * WP + s;
#pragma unroll
    for (int cb = 0; cb < CIN / 32; ++cb) {
      v8bf bfr[CPW];
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
        const int n = bn0 + j * 16;
        const int c = (tap * CIN + cb * 32) / 8 + kc;
        bfr[j] = *reinterpret_cast<const v8bf*>(sW + n * C::BS + wswz<C::RC>(n, c) * 16);
      }
      // every fragment slot computes (a slot past the image's fragments reads the zero border and
      // is never stored): no branch inside the unrolled loop, so the LDS reads of later steps are
      // scheduled ahead of the MFMAs instead of each read waiting on its own
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const v8bf af = *reinterpret_cast<const v8bf*>(sX + (R0[i] + toff) * C::AS + (cb * 32 + kc * 8) * 2);
#pragma unroll
        for (int j = 0; j < CPW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  IDC_IMG_STAMP(7);
  __syncthreads();  // grid and weights dead: the epilogue reuses the region
  IDC_IMG_STAMP(8);

  // ---- 7. epilogue: stage the fp32 tile, then 16-B chunks per thread -----------------------
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    if (i >= nrw) continue;
    const int fr = wr + WM * i;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int col = (wc * CPW + j) * 16 + (lane & 15);
      const int rb = fr * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) Cs[(rb + q) * C::CS_LD + col] = acc[i][j][q];
    }
  }
  __syncthreads();
  const int c8 = tid % C::CPB;
  float psum[8], psq[8], tk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    psum[j] = 0.f;
    psq[j] = 0.f;
    tk[j] = (EPI == 0 && a.stats_shift) ? a.stats_shift[c8 * 8 + j] : 0.f;
  }
  const float mlo = act_lo(a.mbn.act), mhi = act_hi(a.mbn.act);
  float t0[8], t1[8], t2[8], t3[8];  // this thread's 8 channels of the epilogue BatchNorm table
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (EPI == 1) {
      t0[j] = e0[c8 * 8 + j]; t1[j] = e1[c8 * 8 + j]; t2[j] = e2[c8 * 8 + j]; t3[j] = e3[c8 * 8 + j];
    } else {
      t0[j] = t1[j] = t2[j] = t3[j] = 0.f;
    }
  }
  constexpr int RPP = NT / C::CPB;  // rows per pass
#pragma unroll
  for (int it = 0; it < EPP; ++it) {
    const int m = tid / C::CPB + it * RPP;
    if (m >= M) continue;
    const float4 lo4 = *reinterpret_cast<const float4*>(&Cs[m * C::CS_LD + c8 * 8]);
    const float4 hi4 = *reinterpret_cast<const float4*>(&Cs[m * C::CS_LD + c8 * 8 + 4]);
    float v[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
    bf16_t* yp = reinterpret_cast<bf16_t*>(a.y) + (row0 + m) * a.ldy + c8 * 8;
    if constexpr (EPI == 0) {
      const uint4 pk = pack8(v);
      *reinterpret_cast<uint4*>(yp) = pk;
      float rr[8];
      unpack8(pk, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = rr[j] - tk[j];
        psum[j] += d;
        psq[j] += d * d;
      }
    } else {
      float xf[8], d[8];
      unpack8(ep_x[it], xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = xf[j] * t0[j] + t1[j];
        d[j] = (z > mlo && z < mhi) ? v[j] : 0.f;
      }
      const uint4 pk = pack8(d);
      *reinterpret_cast<uint4*>(yp) = pk;
      float rr[8];
      unpack8(pk, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        psum[j] += rr[j];
        psq[j] += rr[j] * (xf[j] - t2[j]) * t3[j];
      }
    }
  }
  IDC_IMG_STAMP(9);
  const bool want = EPI == 1 ? (a.gsum != nullptr || a.gsumx != nullptr) : (a.stats_out != nullptr);
  if (!want) return;
  // transposed reduction over the threads that share a chunk column, one atomic per output
  __syncthreads();
  float* s_red = reinterpret_cast<float*>(smem);
  {
    float4* d4 = reinterpret_cast<float4*>(s_red + tid * C::RED_LD);
    d4[0] = make_float4(psum[0], psum[1], psum[2], psum[3]);
    d4[1] = make_float4(psum[4], psum[5], psum[6], psum[7]);
    d4[2] = make_float4(psq[0], psq[1], psq[2], psq[3]);
    d4[3] = make_float4(psq[4], psq[5], psq[6], psq[7]);
  }
  __syncthreads();
  constexpr int Q = NT / (2 * COUT);
  constexpr int CONTRIB = NT / C::CPB;  // threads per chunk column
  const int o = tid / Q, qq = tid % Q;
  const int kind = o / COUT, col = o % COUT;
  float acc1 = 0.f;
#pragma unroll
  for (int k = qq; k < CONTRIB; k += Q)
    acc1 += s_red[((col >> 3) + C::CPB * k) * C::RED_LD + kind * 8 + (col & 7)];
  if constexpr (Q >= 2) acc1 += __shfl_xor(acc1, 1, 64);
  if constexpr (Q >= 4) acc1 += __shfl_xor(acc1, 2, 64);
  auto final_add = [&](int kind_, int col_, float v) {
    if constexpr (EPI == 0) {
      const size_t so = (size_t)(blockIdx.x % stat_slots(a.stats_slots)) * 2 * a.stats_ld;
      atomicAdd(&a.stats_out[so + (kind_ ? a.stats_ld : 0) + a.stats_off + col_], v);
    } else {
      const size_t so = (size_t)(blockIdx.x % stat_slots(a.gsum_slots)) * a.gsum_ld;
      float* g = kind_ ? a.gsumx : a.gsum;
      if (g) atomicAdd(&g[so + col_], v);
    }
  };
  // Every workgroup finishes at about the same time, so 256 float atomics per address would queue
  // at the memory side (~24 ns each, common.h "Statistics slots").  Where the op's ticket array
  // (conv_igemm.h split-K tickets, unused at ksplit 1, zeroed at build) has room, the workgroups add
  // into S private slot copies kept in it (word 0: arrival counter) and the last arrival folds the
  // copies into the real sums, re-zeroing them for the next launch.
  // The arrival count is two-level for the same reason (one counter word taking 256 arrivals would
  // serialise them): workgroup b counts in word b % 16; the last arrival of a word counts in word 16;
  // the last of those 16 is the last workgroup.  Words: [0, 17) counters, then S x 2*COUT slots.
  constexpr int NCW = 17;
  const int S = (a.tickets != nullptr && a.tickets_n > NCW) ? min(16, (a.tickets_n - NCW) / (2 * COUT)) : 0;
  // (an output whose statistics already have slot copies -- the lowering allocated them for this
  // producer -- takes the direct adds: <= 256 / slots per address, nothing to fold)
  if (S < 2 || gridDim.x < 32 || stat_slots(EPI == 0 ? a.stats_slots : a.gsum_slots) > 1) {
    if (qq == 0) final_add(kind, col, acc1);
    return;
  }
  float* slots = reinterpret_cast<float*>(a.tickets + NCW);
  if (qq == 0) atomicAdd(&slots[(blockIdx.x % S) * 2 * COUT + o], acc1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slot atomic performed
  __syncthreads();
  IDC_IMG_STAMP(10);
  int* s_last = reinterpret_cast<int*>(tA);  // (the prologue tables are dead)
  if (tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned G = gridDim.x, w1 = blockIdx.x & 15u;
    const unsigned n1 = G / 16u + (w1 < G % 16u ? 1u : 0u);  // arrivals at word w1
    const unsigned o1 = __hip_atomic_fetch_add(a.tickets + w1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = 0;
    if ((o1 + 1u) % n1 == 0u) {
      const unsigned o2 = __hip_atomic_fetch_add(a.tickets + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = ((o2 + 1u) % 16u) == 0u;
    }
    s_last[0] = last;
  }
  __syncthreads();
  IDC_IMG_STAMP(11);
  if (!s_last[0]) return;
  if (tid < 2 * COUT) {
    // every slot load in flight at once (one memory round trip), then the sum, then the re-zeroing
    float sv[16];
#pragma unroll
    for (int sl = 0; sl < 16; ++sl)
      sv[sl] = __hip_atomic_load(slots + (sl < S ? sl : 0) * 2 * COUT + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float v = 0.f;
#pragma unroll
    for (int sl = 0; sl < 16; ++sl) v += sl < S ? sv[sl] : 0.f;
#pragma unroll
    for (int sl = 0; sl < 16; ++sl)
      if (sl < S) slots[sl * 2 * COUT + tid] = 0.f;
    final_add(tid / COUT, tid % COUT, v);
  }
  if (tid < NCW) __hip_atomic_store(a.tickets + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// host side

namespace {

// which of the two supported forms a conv is: 0 none, 1 forward 128 -> 32, 2 data gradient 32 -> 128
int img_form(const ConvArgs& a, bool a_f32) {
  if (a.KH != 3 || a.KW != 3 || a.SH != 1 || a.SW != 1 || a.PT != 1 || a.PL != 1) return 0;
  if (a.H != a.Ho || a.W != a.Wo || a.H < 1 || a.W < 1 || a.N < 1) return 0;
  if (a.H * a.W > 13 * 13 || a.H > 13 || a.W > 13) return 0;  // one image per workgroup in LDS
  if (a.ksplit > 1 || (a.ldx % 8) || (a.ldy % 8)) return 0;
  if (a.Cin == 128 && a.Cout == 32 && !a_f32 && a.bpro.mode == 0 && a.epi_mode == 0 && a.out_mode == OUT_BF16 &&
      a.bias == nullptr && a.epi_act == 0 && a.aout == nullptr)
    return 1;
  if (a.Cin == 32 && a.Cout == 128 && a_f32 && a.bpro.mode == 1 && a.epi_mode == 1 && a.out_mode == OUT_BF16 &&
      a.mx != nullptr && (a.ldmx % 8) == 0 && (a.bpro.ldx % 8) == 0 && a.bpro.x != nullptr &&
      (a.aout == nullptr || (a.ldaout % 8) == 0) && a.pro.mode == 0 && a.pro.act == ACT_NONE)
    return 2;
  return 0;
}

}  // namespace

bool conv_img_ok(const ConvArgs& a, bool a_f32) { return img_form(a, a_f32) != 0; }

hipError_t conv_img(const ConvArgs& a, bool a_f32, hipStream_t st) {
  const int form = img_form(a, a_f32);
  if (!form) return hipErrorInvalidValue;
  const int NR = (a.H * a.W + 15) / 16;
  const dim3 grid = ggrid(a.N);
  if (form == 1) {
    const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
    const int rpw = (NR + 3) / 4;
    const int shm = img_smem_bytes<128, 32>(a.H, a.W, NR * 16, 1);
#define IDC_F(R, P)                                                                                          \
  hipLaunchKernelGGL((conv3x3_img_kernel<128, 32, 4, 1, R, bf16_t, P, 0>), grid, dim3(NT), shm, st, a, garg())
    if (pro) {
      if (rpw <= 1) IDC_F(1, 1); else if (rpw <= 2) IDC_F(2, 1); else IDC_F(3, 1);
    } else {
      if (rpw <= 1) IDC_F(1, 0); else if (rpw <= 2) IDC_F(2, 0); else IDC_F(3, 0);
    }
#undef IDC_F
  } else {
    const int shm = img_smem_bytes<32, 128>(a.H, a.W, NR * 16, 2);
#define IDC_D(R)                                                                                            \
  hipLaunchKernelGGL((conv3x3_img_kernel<32, 128, 1, 4, R, float, 2, 1>), grid, dim3(NT), shm, st, a, garg())
    if (NR <= 1) IDC_D(1); else if (NR <= 3) IDC_D(3); else if (NR <= 6) IDC_D(6); else IDC_D(11);
#undef IDC_D
  }
  return hipGetLastError();
}

}  // namespace idc
