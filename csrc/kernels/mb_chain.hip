// Persistent MobileNetV2 block chain, gfx950: the expand (1x1) -> depthwise (3x3) -> project (1x1)
// convs of consecutive inverted-residual blocks, their BatchNorm batch statistics and the block
// outputs BN_p(p) [+ h], in ONE work-queue launch.
//
// Reference: the MobileNetV2 base of /root/reference/dist_model_tf_mobile.py:119-121 (Keras
// Applications, include_top=False) trained at 50x50.  At batch 256 the blocks from
// 13x13 down run 32-4,096-row GEMMs and depthwise maps of a few hundred KB: as separate kernels each
// paid a launch, a ramp, a coefficient-table prologue and a drain of 10-20 us for ~1-3 us of memory
// traffic (profiles/mobilenetv2_bs256_timeline.txt).
//
// Structure.  The lowering lists PHASES in program order (per block: E = expand, D = depthwise,
// P = project; plus one TAB phase for the BatchNorm pending from before the launch).  Every phase
// has a contiguous range of TICKETS; a workgroup takes the next ticket, waits until the phase it
// depends on is READY, runs the tile, and counts itself in the phase's arrivals.  The last arrival
// FINALISES the phase: it sums the statistics slot copies once, writes the single-copy [sum|sumsq]
// the rest of the program reads (backward, moving averages, the next kernel's prologue) and the
// consumer's [scale|shift] table, then raises READY.  A consumer tile therefore reads 2*C finished
// coefficients instead of rebuilding a table from slot sums.  Every wait is on an EARLIER ticket:
// no deadlock at any residency.  Hand-off memory model and give-up path: persist.h.
//
//   MB_PW  rows x 64-column tiles: the operand chunk (rows x <= 256 channels, BN + ReLU6 of the
//          producer or the block-output BN + residual applied while staging, bf16 in LDS), B
//          fragments straight from L2 into registers, v_mfma_f32_16x16x32_bf16 (wave w owns
//          columns 16w..16w+15 of every row), bf16 output through an LDS tile (16-B coalesced
//          agent-coherent stores), per-column shifted sums reduced in-wave and added into slot
//          (tile % slots).  A block-output operand is also stored (aout: the next block's residual
//          and the expand weight gradient's input) by the first column tile.
//   MB_DW  (images x channel chunk) tiles: the chunk's whole input maps BN + ReLU6'd into LDS
//          (fp32), every output pixel from LDS (no halo exchange: a tile holds whole images),
//          statistics reduced per wave with lane shuffles, then 4-way LDS adds.
//   MB_TAB a single tile that builds a pre-launch BatchNorm's table (common.h bn_coeffs).
#include "mb_chain.h"
#include "persist.h"

namespace idc {
namespace {

using namespace persist;

constexpr int NT = 256;
constexpr int KC = 256;          // 1x1 reduction chunk staged at once
constexpr int APITCH = KC + 8;   // bf16 per staged operand row (16-B offset per row: 4-bank skew)
constexpr int YP = 64 + 8;       // bf16 per staged output row
constexpr int MAXK = 1024;       // widest 1x1 operand (its table lives in LDS)
constexpr int SMEM_LIMIT = 64 * 1024;

struct Ctl {
  int task, bad, last;
};

// per phase MB_SYNC_PER_PHASE words: 8 arrival shards (tile % 8), the shards-complete count, READY
__device__ __forceinline__ unsigned* arrive_w(unsigned* sync, int p) { return sync + 2 + MB_SYNC_PER_PHASE * p; }
__device__ __forceinline__ unsigned* ready_w(unsigned* sync, int p) { return sync + 2 + MB_SYNC_PER_PHASE * p + 9; }

// ------------------------------------------------------------------------------------------------
// 1x1 conv tile: rows [m0, m0 + TM) x columns [nb0, nb1) in 64-column chunks
template <int TM>
__device__ void pw_tile(const MbPhaseDesc& d, int t, long long go, char* smem, const float* tabs) {
  constexpr int RF = TM / 16;               // row fragments per wave
  constexpr int MAXQ = TM * KC / 8 / NT;    // staged 16-B operand chunks per thread
  constexpr int MAXT = 2 * MAXK / NT;       // table floats per thread
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = d.N * d.H * d.W, K = d.Cin, Cout = d.Cout;
  const int ctn = (Cout + d.tn - 1) / d.tn;
  const int rt = t / ctn, ct = t - rt * ctn;
  const int m0 = rt * TM, nb0 = ct * d.tn, nb1 = min(Cout, nb0 + d.tn);
  const int nkc = (K + KC - 1) / KC;
  const int pro = d.pro;
  const int ldx = d.ldx, ldy = d.ldy;
  float* sT = reinterpret_cast<float*>(smem);  // [scale | shift] over K
  bf16_t* sA = reinterpret_cast<bf16_t*>(smem + ((2 * K + 3) / 4) * 16);
  bf16_t* sY = K > KC ? sA : sA + 64 * APITCH;  // (K > KC: one column chunk, see mb_phase_smem)
  const bf16_t* __restrict__ X = gsh(d.x, go);
  const bf16_t* __restrict__ R = gsh(d.res, go);
  bf16_t* __restrict__ AO = gsh(d.aout, go);
  const bf16_t* __restrict__ Wt = gsh(d.w16, go);
  bf16_t* __restrict__ Y = gsh(d.y, go);
  const float* __restrict__ KS = gsh(d.shift, go);
  float* __restrict__ SB = gsh(d.slotbuf, go);
  const float* __restrict__ tin = tabs + (pro ? d.tab_in : 0);
  const float lo = act_lo(pro == 1 ? d.act_in : 0), hi = act_hi(pro == 1 ? d.act_in : 0);
  const bool store_a = pro == 2 && AO != nullptr && ct == 0;
  const bool use_r = pro == 2 && R != nullptr;

  uint4 va[MAXQ], vr[MAXQ];
  v8bf bq[KC / 32];
  // operand chunk kc of this tile into registers (issue only)
  auto load_a = [&](int kc) {
    const int k0 = kc * KC, kw = min(KC, K - k0), c8n = ((kw + 31) & ~31) >> 3;
    const int items = TM * c8n;
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) {
      const int q = tid + i * NT;
      const int r = q / c8n, c8 = q - r * c8n;
      const int m = min(m0 + r, M - 1), k = min(k0 + c8 * 8, K - 8);  // clamped: loads unconditional
      va[i] = q < items ? ld_coh16(X + (size_t)m * ldx + k) : make_uint4(0u, 0u, 0u, 0u);
      vr[i] = (q < items && use_r) ? ld_coh16(R + (size_t)m * K + k) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto load_b = [&](int cb, int kc) {
    const int k0 = kc * KC, kw = min(KC, K - k0), ks = (kw + 31) >> 5;
    const int col = min(cb + wid * 16 + (lane & 15), Cout - 1);
#pragma unroll
    for (int s = 0; s < KC / 32; ++s) {
      const int k = min(k0 + 32 * s + 8 * (lane >> 4), K - 8);
      bq[s] = s < ks ? *reinterpret_cast<const v8bf*>(Wt + (size_t)col * K + k) : v8bf{};
    }
  };
  // registers -> transformed bf16 operand in LDS (zero past M / K)
  auto store_a_lds = [&](int kc) {
    const int k0 = kc * KC, kw = min(KC, K - k0), c8n = ((kw + 31) & ~31) >> 3;
    const int items = TM * c8n;
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) {
      const int q = tid + i * NT;
      if (q >= items) break;
      const int r = q / c8n, c8 = q - r * c8n;
      const int m = m0 + r, k = k0 + c8 * 8;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (m < M && k < K) {
        v = va[i];
        if (pro) {
          float f[8], g[8];
          unpack8(v, f);
          unpack8(vr[i], g);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = clampf(fmaf(f[j], sT[k + j], sT[K + k + j]), lo, hi) + g[j];
          v = pack8(f);
          if (store_a) st_coh16(AO + (size_t)m * K + k, v);
        }
      }
      *reinterpret_cast<uint4*>(sA + r * APITCH + c8 * 8) = v;
    }
  };

  // ---- tile inputs: the table, the first operand chunk and the first B fragments in flight at once
  float tv[MAXT];
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    const int j = tid + i * NT;
    tv[i] = (pro && j < 2 * K) ? ld_coh(tin + j) : 0.f;
  }
  load_a(0);
  load_b(nb0, 0);
  __syncthreads();  // (the previous tile's LDS reads are done)
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    const int j = tid + i * NT;
    if (j < 2 * K) sT[j] = tv[i];
  }
  __syncthreads();
  store_a_lds(0);
  __syncthreads();

  for (int cb = nb0; cb < nb1; cb += 64) {
    v4f acc[RF];
#pragma unroll
    for (int i = 0; i < RF; ++i) acc[i] = (v4f){0.f, 0.f, 0.f, 0.f};
    const int col = cb + wid * 16 + (lane & 15);
    for (int kc = 0; kc < nkc; ++kc) {
      if (kc > 0) {  // (K > KC: one column chunk per tile)
        load_a(kc);
        load_b(cb, kc);
        __syncthreads();
        store_a_lds(kc);
        __syncthreads();
      } else if (cb != nb0) {
        load_b(cb, 0);
      }
      const int ks = (min(KC, K - kc * KC) + 31) >> 5;
#pragma unroll
      for (int s = 0; s < KC / 32; ++s) {
        if (s >= ks) break;
#pragma unroll
        for (int i = 0; i < RF; ++i) {
          const v8bf af = *reinterpret_cast<const v8bf*>(sA + (16 * i + (lane & 15)) * APITCH + 32 * s + 8 * (lane >> 4));
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[s], acc[i], 0, 0, 0);
        }
      }
    }
    // ---- epilogue: bf16 output tile, shifted column sums
    const float kk = (KS && col < Cout) ? KS[col] : 0.f;
    float ps = 0.f, pq = 0.f;
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = 16 * i + 4 * (lane >> 4) + q;
        const bf16_t h = f2bf(acc[i][q]);
        sY[rl * YP + wid * 16 + (lane & 15)] = h;
        if (m0 + rl < M) {
          const float dv = bf2f(h) - kk;
          ps += dv;
          pq += dv * dv;
        }
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    pq += __shfl_xor(pq, 16, 64);
    pq += __shfl_xor(pq, 32, 64);
    if (d.bn_mode == 1 && lane < 16 && col < Cout) {
      float* so = SB + (size_t)(t % d.slots) * 2 * Cout;
      atomicAdd(so + col, ps);
      atomicAdd(so + Cout + col, pq);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM * 8 / NT; ++i) {
      const int q = tid + i * NT, r = q >> 3, c8 = q & 7;
      const int m = m0 + r, n = cb + c8 * 8;
      if (m < M && n < Cout) st_coh16(Y + (size_t)m * ldy + n, *reinterpret_cast<const uint4*>(sY + r * YP + c8 * 8));
    }
    __syncthreads();  // sY is rewritten by the next column chunk
  }
}

// ------------------------------------------------------------------------------------------------
// depthwise 3x3 tile: images [n0, n0 + IMG) x channels [c0, c0 + CW), CW in {16, 32, 64}
template <int CG>
__device__ void dw_tile(const MbPhaseDesc& d, int t, long long go, char* smem, const float* tabs) {
  constexpr int CW = CG * 8, RW = NT / CG;  // pixel rows in flight per pass
  const int tid = threadIdx.x, lane = tid & 63;
  const int C = d.Cin, ncc = C / CW;
  const int gi = t / ncc, cc = t - gi * ncc;
  const int n0 = gi * d.tm, c0 = cc * CW;
  const int nimg = min(d.tm, d.N - n0);
  const int H = d.H, W = d.W, Ho = d.Ho, Wo = d.Wo, S = d.S, PT = d.PT, PL = d.PL;
  const int HWi = H * W, HWo = Ho * Wo;
  float* sT = reinterpret_cast<float*>(smem);  // [scale | shift] over the chunk
  float* sS = sT + 2 * CW;                      // [sum | sumsq] over the chunk
  float* sX = sS + 2 * CW;                      // [img][H][W][CW]
  const bf16_t* __restrict__ X = gsh(d.x, go);
  bf16_t* __restrict__ Y = gsh(d.y, go);
  const float* __restrict__ W32 = gsh(d.w32, go);
  const float* __restrict__ KS = gsh(d.shift, go);
  float* __restrict__ SB = gsh(d.slotbuf, go);
  const int pro = d.pro;
  const float lo = act_lo(pro ? d.act_in : 0), hi = act_hi(pro ? d.act_in : 0);
  const int tx = tid % CG, ty = tid / CG;
  // ---- tile inputs, all in flight at once: the input maps, the table, the kernel, the shift
  constexpr int MAXI = 8;  // 16-B input chunks per thread (sX <= 64 KB)
  const int items = nimg * HWi * CG;
  const size_t base = (size_t)n0 * HWi;
  uint4 xv[MAXI];
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    const int q = tid + i * NT;
    const int pix = q / CG, g = q - pix * CG;
    xv[i] = q < items ? ld_coh16(X + (base + pix) * d.ldx + c0 + g * 8) : make_uint4(0u, 0u, 0u, 0u);
  }
  float tval = tid < CW ? 1.f : 0.f;
  if (pro && tid < 2 * CW) tval = ld_coh(tabs + d.tab_in + c0 + (tid % CW) + (tid >= CW ? C : 0));
  float wk[9][8], kk[8], ps[8], pq[8];
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const float4 a0 = *reinterpret_cast<const float4*>(W32 + (size_t)r * C + c0 + tx * 8);
    const float4 a1 = *reinterpret_cast<const float4*>(W32 + (size_t)r * C + c0 + tx * 8 + 4);
    wk[r][0] = a0.x; wk[r][1] = a0.y; wk[r][2] = a0.z; wk[r][3] = a0.w;
    wk[r][4] = a1.x; wk[r][5] = a1.y; wk[r][6] = a1.z; wk[r][7] = a1.w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    kk[j] = KS ? KS[c0 + tx * 8 + j] : 0.f;
    ps[j] = 0.f;
    pq[j] = 0.f;
  }
  __syncthreads();  // (the previous tile's LDS reads are done)
  if (tid < 2 * CW) {
    sT[tid] = tval;
    sS[tid] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    const int q = tid + i * NT;
    if (q >= items) break;
    const int pix = q / CG, g = q - pix * CG;
    float f[8];
    unpack8(xv[i], f);
    affine_act8(f, sT + g * 8, sT + CW + g * 8, lo, hi);
    float* dst = sX + (size_t)pix * CW + g * 8;
    *reinterpret_cast<float4*>(dst) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
  __syncthreads();
  const int outs = nimg * HWo;
  for (int o = ty; o < outs; o += RW) {
    const int nl = o / HWo, rem = o - nl * HWo;
    const int ho = rem / Wo, wo = rem - ho * Wo;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = ho * S - PT + r;
      if ((unsigned)h >= (unsigned)H) continue;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int w = wo * S - PL + s;
        if ((unsigned)w >= (unsigned)W) continue;
        const float* src = sX + ((size_t)(nl * H + h) * W + w) * CW + tx * 8;
        const float4 a0 = *reinterpret_cast<const float4*>(src);
        const float4 a1 = *reinterpret_cast<const float4*>(src + 4);
        const float u[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(u[j], wk[r * 3 + s][j], acc[j]);
      }
    }
    const uint4 pk = pack8(acc);
    st_coh16(Y + ((size_t)(n0 + nl) * HWo + rem) * d.ldy + c0 + tx * 8, pk);
    float rv[8];
    unpack8(pk, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dv = rv[j] - kk[j];
      ps[j] += dv;
      pq[j] += dv * dv;
    }
  }
  // lanes of a wave with equal tx (= lane % CG) share channels
#pragma unroll
  for (int o = CG; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ps[j] += __shfl_xor(ps[j], o, 64);
      pq[j] += __shfl_xor(pq[j], o, 64);
    }
  if (lane < CG) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(&sS[tx * 8 + j], ps[j]);
      atomicAdd(&sS[CW + tx * 8 + j], pq[j]);
    }
  }
  __syncthreads();
  if (d.bn_mode == 1 && tid < 2 * CW) {
    float* so = SB + (size_t)(t % d.slots) * 2 * C;
    atomicAdd(so + (tid >= CW ? C : 0) + c0 + (tid % CW), sS[tid]);
  }
}

// the phase's last tile: single-copy statistics and the consumer's table.  Every load of a thread's
// (up to MAXK / NT) channels is issued before any arithmetic: one memory round trip.
__device__ void finalize(const MbPhaseDesc& d, long long go, float* tabs) {
  constexpr int CPT = MAXK / NT;
  const int C = d.Cout;
  const float* __restrict__ SB = gsh(d.slotbuf, go);
  float* __restrict__ ST = gsh(d.stats, go);
  const float* __restrict__ KS = gsh(d.shift, go);
  const float* __restrict__ G = gsh(d.gamma, go);
  const float* __restrict__ Bt = gsh(d.beta, go);
  const float* __restrict__ MM = gsh(d.mmean, go);
  const float* __restrict__ MV = gsh(d.mvar, go);
  const int S = d.slots;
  const bool batch = d.bn_mode == 1;
  float a0[CPT][MB_MAX_SLOTS], a1[CPT][MB_MAX_SLOTS], g[CPT], bt[CPT], k0[CPT], k1[CPT];
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int c = min((int)threadIdx.x + u * NT, C - 1);
#pragma unroll
    for (int s = 0; s < MB_MAX_SLOTS; ++s) {
      const size_t o = (size_t)(s < S ? s : S - 1) * 2 * C + c;
      a0[u][s] = batch ? ld_coh(SB + o) : 0.f;
      a1[u][s] = batch ? ld_coh(SB + o + C) : 0.f;
    }
    g[u] = G ? G[c] : 1.f;
    bt[u] = Bt ? Bt[c] : 0.f;
    k0[u] = batch ? (KS ? KS[c] : 0.f) : MM[c];
    k1[u] = batch ? 0.f : MV[c];
  }
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int c = threadIdx.x + u * NT;
    if (c >= C) break;
    float mean = k0[u], var = k1[u];
    if (batch) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int s = 0; s < MB_MAX_SLOTS; ++s) {
        s0 += s < S ? a0[u][s] : 0.f;
        s1 += s < S ? a1[u][s] : 0.f;
      }
      if (ST) {
        ST[c] = s0;
        ST[C + c] = s1;
      }
      shifted_mean_var(k0[u], s0, s1, d.inv_count, mean, var);
    }
    const float sc = g[u] * rsqrtf(var + d.eps);
    st_coh(tabs + d.tab_out + c, sc);
    st_coh(tabs + d.tab_out + C + c, bt[u] - mean * sc);
  }
}

// every thread's stores / atomics of the tile performed, then ONE lane counts the tile in its shard
// of the phase's arrivals; the tile that completes a shard counts the shard, and the tile that
// completes the last shard is the phase's last (it saw every other tile's count through the values
// its two adds returned).  Returns (to every thread, via LDS) whether this tile is the last.
__device__ __forceinline__ bool arrive(unsigned* arr, int t, int tiles, Ctl& s) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int sh = t & 7;
    const unsigned old = __hip_atomic_fetch_add(arr + sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool last = false;
    if ((int)old + 1 == (tiles - sh + 7) / 8) {
      const unsigned o2 = __hip_atomic_fetch_add(arr + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (int)o2 + 1 == min(tiles, 8);
    }
    s.last = last;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s.last) != 0;
}

}  // namespace

// (outside the anonymous namespace so profiles name it)
__global__ __launch_bounds__(NT) void mb_chain_kernel(MbChainArgs a, GroupArg ga) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ Ctl s;
  const long long go = goff(ga);
  unsigned* sync = gsh(a.sync, go);
  unsigned* fail = sync + 1;
  float* tabs = gsh(a.tabs, go);
  const FailSink fsink{gsh(a.err, go), gsh(a.stepflag, go), a.hostflag};
  unsigned long long* stamps = gsh(a.stamps, go);
  const unsigned max_polls = a.max_polls ? a.max_polls : DEFAULT_POLLS;
  const int tid = threadIdx.x;
  // the phase table, copied once into LDS: every descriptor field a tile reads is an LDS read (read
  // from global memory, each field was a dependent vector load on the tile's critical path)
  MbPhaseDesc* P = reinterpret_cast<MbPhaseDesc*>(smem);
  char* tsm = smem + MB_TABLE_BYTES;
  {
    const unsigned* src = reinterpret_cast<const unsigned*>(gsh(a.phases, go));
    unsigned* dst = reinterpret_cast<unsigned*>(smem);
    const int words = a.nphases * (int)sizeof(MbPhaseDesc) / 4;
    for (int i = tid; i < words; i += NT) dst[i] = src[i];
  }
  int cp = 0;
  for (;;) {
    // ticket: a thread-0 region between barriers, broadcast through LDS + readfirstlane so every
    // branch of the loop is workgroup-uniform (dense_stage.hip); the first barrier also publishes
    // the phase table
    __syncthreads();
    if (tid == 0) s.task = (int)__hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(s.task);
    if (task >= a.ntickets) return;
    while (cp + 1 < a.nphases && task >= P[cp].first + P[cp].tiles) ++cp;
    cp = __builtin_amdgcn_readfirstlane(cp);
    const MbPhaseDesc& d = P[cp];
    const int t = task - d.first;
    stamp(stamps, task, 0);
    if (d.dep >= 0) {
      if (tid == 0) s.bad = !wait_count(ready_w(sync, d.dep), 1u, fail, fsink, max_polls);
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s.bad)) return;
    }
    stamp(stamps, task, 1);
    const int kind = d.kind;
    if (kind == MB_PW) {
      if (d.tm == 64) pw_tile<64>(d, t, go, tsm, tabs);
      else pw_tile<32>(d, t, go, tsm, tabs);
    } else if (kind == MB_DW) {
      const int cw = d.tn;
      if (cw == 64) dw_tile<8>(d, t, go, tsm, tabs);
      else if (cw == 32) dw_tile<4>(d, t, go, tsm, tabs);
      else dw_tile<2>(d, t, go, tsm, tabs);
    } else {  // MB_TAB
      BnArgs b = d.pre;
      gshift(b, go);
      for (int c = tid; c < d.Cout; c += NT) {
        float sc, sh;
        bn_coeffs(b, c, sc, sh);
        st_coh(tabs + d.tab_out + c, sc);
        st_coh(tabs + d.tab_out + d.Cout + c, sh);
      }
    }
    stamp(stamps, task, 2);
    if (arrive(arrive_w(sync, cp), t, d.tiles, s)) {
      if (kind != MB_TAB && d.tab_out >= 0) finalize(d, go, tabs);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(ready_w(sync, cp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(stamps, task, 3);
  }
}

namespace {

}  // namespace

int mb_smem_limit() { return SMEM_LIMIT - MB_TABLE_BYTES; }

// tile LDS: PW = table + operand chunk (+ the output staging tile, which aliases the operand when
// K > KC: one column chunk, operand dead after its last MFMA); DW = tables + input maps
int mb_phase_smem(const MbPhaseDesc& d) {
  if (d.kind == MB_PW) return ((2 * d.Cin + 3) / 4) * 16 + 64 * APITCH * 2 + (d.Cin > KC ? 0 : 64 * YP * 2);
  if (d.kind == MB_DW) return (4 * d.tn + d.tm * d.H * d.W * d.tn) * 4;
  return 0;
}

// host-side shape rules of one phase (the Python lowering checks every descriptor with this
// before it emits the launch: a tile never indexes past what these allow)
bool mb_phase_ok(const MbPhaseDesc& d) {
  if (d.tiles < 1 || d.first < 0 || d.N < 1 || d.Cout < 1) return false;
  if (d.kind == MB_TAB) return d.tiles == 1 && d.tab_out >= 0 && d.Cout <= 4096;
  if (d.pro && d.tab_in < 0) return false;
  if (d.bn_mode == 1 && (d.slots < 1 || d.slots > MB_MAX_SLOTS || d.slotbuf == nullptr)) return false;
  if (d.Cout > MAXK) return false;
  if (d.bn_mode && d.tab_out < 0) return false;
  if (d.kind == MB_PW) {
    const int M = d.N * d.H * d.W;
    if (d.tm != 32 && d.tm != 64) return false;
    if (d.tn < 64 || d.tn % 64 || (d.Cin > KC && d.tn != 64)) return false;
    if (d.Cin % 8 || d.Cin > MAXK || d.Cout % 8 || d.ldx % 8 || d.ldy % 8 || d.ldx < d.Cin || d.ldy < d.Cout) return false;
    if (d.pro == 2 && d.act_in != 0) return false;
    if (d.pro == 0 && (d.res || d.aout)) return false;
    const int tiles = ((M + d.tm - 1) / d.tm) * ((d.Cout + d.tn - 1) / d.tn);
    return d.tiles == tiles && d.H == d.Ho && d.W == d.Wo && mb_phase_smem(d) <= mb_smem_limit();
  }
  if (d.kind == MB_DW) {
    if (d.tn != 16 && d.tn != 32 && d.tn != 64) return false;
    if (d.Cin != d.Cout || d.Cin % d.tn || d.tm < 1 || (d.S != 1 && d.S != 2)) return false;
    if (d.ldx % 8 || d.ldy % 8 || d.ldx < d.Cin || d.ldy < d.Cin || d.PT < 0 || d.PL < 0 || d.PT > 1 || d.PL > 1)
      return false;
    if ((d.Ho - 1) * d.S - d.PT + 2 < 0 || d.Ho < 1 || d.Wo < 1) return false;
    const int tiles = ((d.N + d.tm - 1) / d.tm) * (d.Cin / d.tn);
    return d.tiles == tiles && mb_phase_smem(d) <= mb_smem_limit() &&
           d.tm * d.H * d.W * (d.tn / 8) <= 8 * NT;  // (dw_tile MAXI)
  }
  return false;
}

hipError_t mb_chain(const MbChainArgs& a, int grid, int smem, hipStream_t st) {
  if (a.phases == nullptr || a.sync == nullptr || a.tabs == nullptr || a.nphases < 1 ||
      a.nphases > MB_MAX_PHASES || a.ntickets < 1 || smem < 0 || smem > mb_smem_limit())
    return hipErrorInvalidValue;
  smem += MB_TABLE_BYTES;
  if (grid <= 0) grid = 512;
  const int k = launch_groups().k;
  if (k > 1) grid = grid / k > 8 ? grid / k : 8;
  if (grid > a.ntickets) grid = a.ntickets;
  hipLaunchKernelGGL(mb_chain_kernel, ggrid(grid), dim3(NT), smem, st, a, garg());
  return hipGetLastError();
}

}  // namespace idc
