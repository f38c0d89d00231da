// Large-tile implicit-GEMM convolution for the wide, plain layers (VGG16 blocks 2-5 forward and
// data gradient), gfx950.
//
// The general kernel (conv_igemm_impl.h) is built for DenseNet's small, BN-transformed layers:
// 64-128 row tiles, operands staged through VGPRs so the pending-BN prologue can transform them.
// VGG's layers have no prologue (the forward input is already ReLU(conv + bias)) and are large
// GEMMs (M up to 160k pixels, N 128-512, K 576-4608), where a 64x64 tile with 2x2 waves reads as
// many LDS bytes per MFMA as the LDS can deliver.  Here:
//
//   * 256 x BN tiles, BK = 64: BN = 128 / 256 with 8 waves as 2 (M) x 4 (N) (each wave a
//     128 x BN/4 sub-tile: 8 x BN/64 accumulators of v_mfma_f32_16x16x32_bf16, 32 or 64 MFMAs per
//     64-deep K step against 8 + BN/64 ds_read_b128 per 32-deep half), BN = 64 with 4 waves as
//     4 x 1 (64 x 64 each: 16 MFMAs per 8 fragment reads; measured slower than the general
//     kernel's 64x64 tiles on VGG block 1, so the autotuner does not offer it);
//   * both operands go global -> LDS with global_load_lds_dwordx4 (no VGPR staging): a K step is
//     one tap (r, s) and 64 consecutive input channels (Cin % 64 == 0), so every A row is one
//     contiguous 128-B line of the NHWC input; rows outside the image (padding) and past M load a
//     16-B zero block instead;
//   * the LDS image is lane-linear per wave instruction (8 rows x 128 B), so the chunk XOR
//     swizzle (chunk ^ (row & 6), conflict-free for the ds_read_b128 fragment reads) is applied to
//     the per-lane SOURCE address (guide §5.4 rule 21);
//   * two LDS buffers: tile k+1's loads are issued before tile k is computed and waited with a
//     counted s_waitcnt vmcnt (tile k's own loads only), raw s_barrier (a __syncthreads would
//     drain the in-flight DMA with vmcnt(0));
//   * epilogue per wave through a private LDS staging tile (16 rows at a time) -> 16-B coalesced
//     bf16 stores: EPI 0 bias + activation; EPI 1 (data gradient) the activation mask from the
//     saved forward input and the bias gradient sum(dZ) of the producing conv.
// Reference hot loop: the VGG16 Conv2D stack of dist_model_tf_vgg.py:119-129.
#include "common.h"
#include "conv_igemm.h"

namespace idc {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_zero_src[8];  // zero-initialised padding source

typedef __attribute__((address_space(3))) void lds_void_t;

template <int BN, int WM_, int WN_, int NBUF_>
struct BigCfg {
  static constexpr int WM = WM_, WN = WN_, NW = WM * WN;
  static constexpr int BM = 256, BK = 64, NT = NW * 64;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 16, TN = WTN / 16;
  static constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  static constexpr int BUF_ELEMS = A_ELEMS + B_ELEMS;
  // LDS buffers: 2, or 3 (two tiles in flight across each barrier: the few-workgroup, deep-K
  // layers whose K step is load-latency bound; 1-3% slower on the large-M ones)
  static constexpr int NBUF = NBUF_;
  static constexpr int LDS_MAIN = NBUF * BUF_ELEMS * 2;
  static constexpr int NGA = BM * (BK / 8) / NT;  // glds per thread per tile (A)
  static constexpr int NGB = BN * (BK / 8) / NT;  // (B)
  static constexpr int SLD = WTN + 4;
  static constexpr int STAGE = NW * 16 * SLD * 4;
  static constexpr int LDS_BYTES = (LDS_MAIN > STAGE + BN * 4 ? LDS_MAIN : STAGE + BN * 4);
};

__device__ __forceinline__ int bswz(int row, int chunk) { return chunk ^ (row & 6); }

}  // namespace

template <int BN, int WM, int WN, int NBUF_, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void conv_big_kernel(ConvArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  using C = BigCfg<BN, WM, WN, NBUF_>;
  constexpr int NW = C::NW;
  constexpr int BM = C::BM, BK = C::BK, TM = C::TM, TN = C::TN, WTN = C::WTN;
  constexpr int NGA = C::NGA, NGB = C::NGB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int wr = wid / C::WN, wc = wid % C::WN;
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.KH * a.KW * a.Cin;
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int mtiles = (M + BM - 1) / BM;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  // split-K (the under-filled small-M layers): the slices of a tile are consecutive ids
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles * nsplit);
  const int tile = bid / nsplit, slice = bid - tile * nsplit;
  const int mt = tile / ntiles, nt = tile % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk_all = K / BK;
  const int per_slice = (nk_all + nsplit - 1) / nsplit;
  const int kb = slice * per_slice;
  const int nk = max(0, min(nk_all, kb + per_slice) - kb);

  // ---- per-thread source rows (fixed for the whole K loop) ----------------------------------
  // wave instruction j covers rows (j*NW + wid)*8 .. +8; lane -> row + lane/8, LDS chunk lane%8
  const int lrow = lane >> 3, pch = lane & 7;
  const int sch = pch ^ (lrow & 6);  // swizzle on the source side (row & 6 == lrow & 6)
  int a_img[NGA], a_h0[NGA], a_w0[NGA];
  bool a_ok[NGA];
#pragma unroll
  for (int j = 0; j < NGA; ++j) {
    const int m = m0 + (j * NW + wid) * 8 + lrow;
    a_ok[j] = m < M;
    const int mm = a_ok[j] ? m : 0;
    const int wo = mm % a.Wo, t = mm / a.Wo;
    const int ho = t % a.Ho;
    a_img[j] = t / a.Ho;
    a_h0[j] = ho * a.SH - a.PT;
    a_w0[j] = wo * a.SW - a.PL;
  }
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ Wt = a.w;
  const uint4* zsrc = g_zero_src;

  auto issue = [&](int kt, int buf) {
    const int k0 = (kb + kt) * BK;
    const int rs = k0 / a.Cin, c0 = k0 - rs * a.Cin;
    const int kr = rs / a.KW, ks = rs - kr * a.KW;
    bf16_t* As = lds + buf * C::BUF_ELEMS;
    bf16_t* Bs = As + C::A_ELEMS;
#pragma unroll
    for (int j = 0; j < NGA; ++j) {
      const int h = a_h0[j] + kr, w = a_w0[j] + ks;
      const bool ok = a_ok[j] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const void* src = ok ? (const void*)(X + ((size_t)(a_img[j] * a.H + h) * a.W + w) * a.ldx + c0 + sch * 8)
                           : (const void*)zsrc;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(As + (j * NW + wid) * 8 * BK), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NGB; ++j) {
      const int n = n0 + (j * NW + wid) * 8 + lrow;
      const void* src = n < a.Cout ? (const void*)(Wt + (size_t)n * K + k0 + sch * 8) : (const void*)zsrc;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(Bs + (j * NW + wid) * 8 * BK), 16, 0, 0);
    }
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fk = lane >> 4;
  constexpr int NBUF = C::NBUF, NG = NGA + NGB;
  if (nk > 0) issue(0, 0);
  if (NBUF == 3 && nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt must have landed; the loads of the NBUF-2 tiles after it stay in flight
    const int ahead = kt + NBUF - 1;
    if (ahead < nk) {
      issue(ahead, ahead % NBUF);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 1) * NG) : "memory");
    } else if (NBUF == 3 && kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's tile-kt DMA is visible
    const bf16_t* As = lds + (kt % NBUF) * C::BUF_ELEMS;
    const bf16_t* Bs = As + C::A_ELEMS;
    // 256x128 tiles read every fragment of the K step up front (both 32-deep halves, distinct
    // registers), then issue the MFMAs: hipcc otherwise recycles two fragment registers, which
    // serialises each ds_read behind the MFMAs of the previous pair (read -> lgkmcnt(0) -> 4
    // MFMAs -> read ...).  256x256 tiles have no registers for that (it spills) and keep the
    // per-half order.
    if constexpr (TN <= 2) {
    v8bf af[BK / 32][TM], bfr[BK / 32][TN];
#pragma unroll
    for (int q = 0; q < BK / 32; ++q) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wc * WTN + j * 16 + frow;
        bfr[q][j] = *reinterpret_cast<const v8bf*>(Bs + row * BK + bswz(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wr * C::WTM + i * 16 + frow;
        af[q][i] = *reinterpret_cast<const v8bf*>(As + row * BK + bswz(row, q * 4 + fk) * 8);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < BK / 32; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q][i], bfr[q][j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
    for (int q = 0; q < BK / 32; ++q) {
      v8bf af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wr * C::WTM + i * 16 + frow;
        af[i] = *reinterpret_cast<const v8bf*>(As + row * BK + bswz(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wc * WTN + j * 16 + frow;
        bfr[j] = *reinterpret_cast<const v8bf*>(Bs + row * BK + bswz(row, q * 4 + fk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // buffer kt % NBUF free for tile kt + NBUF
  }

  // ---- split-K: publish this slice's partial tile; the tile's last arriver sums them ---------
  // (the protocol of conv_igemm_impl.h: plain stores -> vmcnt(0) -> barrier -> lane 0 agent
  //  release + relaxed ticket (modulo nsplit) -> the last arriver acquires and reads)
  if (nsplit > 1) {
    constexpr int NF = TM * TN;
    float4* slab = reinterpret_cast<float4*>(a.slab) + (size_t)tile * nsplit * NF * C::NT;
    {
      float4* mine = slab + (size_t)slice * NF * C::NT;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          mine[(i * TN + j) * C::NT + tid] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
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
    for (int sl = 0; sl < nsplit; ++sl) {
      if (sl == slice) continue;
      const float4* o = slab + (size_t)sl * NF * C::NT;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float4 q = o[(i * TN + j) * C::NT + tid];
          acc[i][j][0] += q.x;
          acc[i][j][1] += q.y;
          acc[i][j][2] += q.z;
          acc[i][j][3] += q.w;
        }
    }
  }

  // ---- epilogue: each wave stages 16 rows of its sub-tile at a time -------------------------
  constexpr int SLD = C::SLD, CPB = WTN / 8, ITER = (16 * CPB + 63) / 64;
  float* st = reinterpret_cast<float*>(smem) + wid * 16 * SLD;
  float* s_g = reinterpret_cast<float*>(smem) + NW * 16 * SLD;  // EPI 1: per-block sum(dZ)
  if constexpr (EPI == 1) {
    for (int t = tid; t < BN; t += C::NT) s_g[t] = 0.f;
  }
  __syncthreads();  // no DMA in flight any more: a plain barrier
  const float epi_lo = act_lo(a.epi_act), epi_hi = act_hi(a.epi_act);
  const float msk_lo = act_lo(a.mbn.act), msk_hi = act_hi(a.mbn.act);
  const int my_c8 = lane % CPB;
  float t_bias[8], psum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + wc * WTN + my_c8 * 8 + j;
    t_bias[j] = (EPI == 0 && a.bias && n < a.Cout) ? a.bias[n] : 0.f;
    psum[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(fk * 4 + r) * SLD + j * 16 + frow] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = lane + it * 64;
      const int rr = idx / CPB, c8 = idx % CPB;
      const int m = m0 + wr * C::WTM + i * 16 + rr;
      const int n = n0 + wc * WTN + c8 * 8;
      if (idx < 16 * CPB && m < M && n < a.Cout) {
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(st + rr * SLD + c8 * 8);
        const float4 hi = *reinterpret_cast<const float4*>(st + rr * SLD + c8 * 8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        if constexpr (EPI == 0) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = clampf(v[jj] + t_bias[jj], epi_lo, epi_hi);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (size_t)m * a.ldy + n) = pack8(v);
        } else {
          float xf[8], d[8];
          unpack8(*reinterpret_cast<const uint4*>(a.mx + (size_t)m * a.ldmx + n), xf);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) d[jj] = (xf[jj] > msk_lo && xf[jj] < msk_hi) ? v[jj] : 0.f;
          const uint4 p = pack8(d);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (size_t)m * a.ldy + n) = p;
          float rq[8];
          unpack8(p, rq);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) psum[jj] += rq[jj];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // staging tile reused by the next 16 rows
  }
  if constexpr (EPI == 1) {
    if (a.gsum) {
      wave_reduce_chunks<CPB>(psum);
      if (lane < CPB) {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) atomicAdd(&s_g[wc * WTN + lane * 8 + jj], psum[jj]);
      }
      __syncthreads();
      const size_t so = (size_t)(mt % stat_slots(a.gsum_slots)) * a.gsum_ld;
      for (int t = tid; t < BN; t += C::NT)
        if (n0 + t < a.Cout) atomicAdd(&a.gsum[so + n0 + t], s_g[t]);
    }
  }
}

bool conv_big_ok(const ConvArgs& a, bool a_f32) {
  if (a_f32) return false;
  if (a.pro.mode != 0 || a.pro.act != ACT_NONE || a.bpro.mode != 0) return false;
  if ((a.Cin % 64) || (a.ldx % 8) || (a.ldy % 8) || (a.Cout % 8)) return false;
  if (a.epi_mode == 0) return a.out_mode == OUT_BF16 && a.stats_out == nullptr;
  if (a.epi_mode == 1)
    return a.mbn.mode == 0 && a.gsumx == nullptr && a.mx != nullptr && (a.ldmx % 8) == 0;
  return false;
}

template <int BN, int WM, int WN, int NBUF>
static hipError_t big_launch(const ConvArgs& a, hipStream_t st) {
  using C = BigCfg<BN, WM, WN, NBUF>;
  const int M = a.N * a.Ho * a.Wo;
  const int tiles = ((M + C::BM - 1) / C::BM) * ((a.Cout + BN - 1) / BN);
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  if (ks > 1 && ((long long)tiles * ks * C::BM * BN > a.slab_floats || tiles > a.tickets_n)) return hipErrorInvalidValue;
  const int grid = tiles * ks;
  if (grid == 0) return hipSuccess;
  if (a.epi_mode == 0)
    hipLaunchKernelGGL((conv_big_kernel<BN, WM, WN, NBUF, 0>), ggrid(grid), dim3(C::NT), C::LDS_BYTES, st, a, garg());
  else
    hipLaunchKernelGGL((conv_big_kernel<BN, WM, WN, NBUF, 1>), ggrid(grid), dim3(C::NT), C::LDS_BYTES, st, a, garg());
  return hipGetLastError();
}

hipError_t conv_big(const ConvArgs& a, int bn, bool a_f32, hipStream_t st) {
  if (!conv_big_ok(a, a_f32)) return hipErrorInvalidValue;
  if (bn == 256) return big_launch<256, 2, 4, 2>(a, st);
  if (bn == 128) return big_launch<128, 2, 4, 2>(a, st);
  if (bn == -128) return big_launch<128, 2, 4, 3>(a, st);  // three buffers
  return big_launch<64, 4, 1, 2>(a, st);  // 4 waves of 64 x 64
}

}  // namespace idc
