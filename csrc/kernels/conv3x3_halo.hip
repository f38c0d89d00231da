// Direct 3x3 / stride 1 / 'same' convolution for SMALL images, one image per workgroup, gfx950.
//
// DenseNet at 50x50 runs its 58 growth convs (3x3, Cin=128 -> Cout=32) and their data gradients
// (3x3, 32 -> 128) on 13x13, 6x6, 3x3 and 1x1 feature maps.  As implicit GEMMs those are skinny
// (N = 32), re-read every input pixel 9x through the im2col gather and need 18+ dependent K steps
// per tile: latency-bound at ~5% of MFMA peak.  Here a workgroup owns a whole image instead:
//
//   1. stage the zero-padded (H+2)x(W+2)xCin halo of its image in LDS ONCE — pending BN + act
//      applied on the way in, padding inserted AFTER the activation (Keras semantics) — together
//      with all 9 taps of the bf16 weights (re-laid out as [tap][Cout][Cin] in LDS);
//   2. every wave sweeps its 16-row output tiles over 9 taps x Cin/32 K-steps with
//      v_mfma_f32_16x16x32_bf16, A fragments read straight out of the halo (the tap is just an
//      LDS address offset — no im2col), B fragments cached in registers across its tiles;
//   3. epilogue per wave through a private LDS staging tile: 16-B coalesced bf16 stores into the
//      (channel-sliced) destination plus either the next BN's [sum|sumsq] (EPI 0) or the
//      BN-backward terms dZ = dA*act'(z), sum dZ, sum dZ*xhat (EPI 1), reduced in LDS then one
//      global atomic per channel per workgroup.
//
// Per-pixel LDS stride is Cin+8 elements: 16 consecutive pixels then start on 16 distinct 4-bank
// groups, so the ds_read_b128 fragment reads are conflict-free.  All global loads of the staging
// phase are issued in batches before any LDS write (RU independent loads in flight per thread).
#include "common.h"
#include "conv_igemm.h"

namespace idc {

namespace {

constexpr int NT = 256;

struct HaloGeom {
  int H, W, Hp, Wp, CinP, npix, mtiles;
  size_t halo_bytes, w_bytes, stage_bytes, table_bytes;
};

__host__ __device__ inline HaloGeom halo_geom(int H, int W, int Cin, int Cout, int pro, int epi) {
  HaloGeom g;
  g.H = H; g.W = W; g.Hp = H + 2; g.Wp = W + 2;
  g.CinP = Cin + 8;
  g.npix = H * W;
  g.mtiles = (g.npix + 15) / 16;
  g.halo_bytes = (size_t)g.Hp * g.Wp * g.CinP * 2;
  g.w_bytes = (size_t)9 * Cout * g.CinP * 2;
  g.stage_bytes = (size_t)4 * 16 * (Cout + 4) * 4;
  g.table_bytes = (size_t)(2 * (pro ? Cin : 0) + 2 * Cout + (epi ? 4 * Cout : 0)) * 4;
  return g;
}

}  // namespace

template <int COUT, int MT, typename TA, int PRO, int EPI>
__global__ __launch_bounds__(NT) void conv3x3_halo_kernel(ConvArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  constexpr int NTL = COUT / 16;  // n tiles (16 output channels each)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const HaloGeom g = halo_geom(a.H, a.W, a.Cin, COUT, PRO, EPI);
  bf16_t* s_halo = reinterpret_cast<bf16_t*>(smem);
  bf16_t* s_w = reinterpret_cast<bf16_t*>(smem + g.halo_bytes);
  float* s_stage = reinterpret_cast<float*>(smem + g.halo_bytes + g.w_bytes);
  float* s_tab = reinterpret_cast<float*>(smem + g.halo_bytes + g.w_bytes + g.stage_bytes);
  float* s_scale = s_tab;                       // [Cin]   (PRO)
  float* s_shift = s_scale + (PRO ? a.Cin : 0);  // [Cin]   (PRO)
  float* s_sum = s_shift + (PRO ? a.Cin : 0);    // [COUT]
  float* s_sq = s_sum + COUT;                    // [COUT]
  float* s_e = s_sq + COUT;                      // [4][COUT] (EPI 1)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int img = blockIdx.x;
  const int Cin = a.Cin, CinP = g.CinP, C8 = Cin / 8;

  // ---- tables --------------------------------------------------------------------------
  if constexpr (PRO) {
    for (int c = tid; c < Cin; c += NT) {
      float sc, sh;
      bn_coeffs(a.pro, c, sc, sh);
      s_scale[c] = sc;
      s_shift[c] = sh;
    }
  }
  for (int c = tid; c < COUT; c += NT) {
    s_sum[c] = 0.f;
    s_sq[c] = 0.f;
    if constexpr (EPI == 1) {
      float sc, sh, mean = 0.f, rstd = 1.f;
      bn_coeffs(a.mbn, c, sc, sh);
      if (a.mbn.mode) bn_mean_rstd(a.mbn, c, mean, rstd);
      s_e[c] = sc; s_e[COUT + c] = sh; s_e[2 * COUT + c] = mean; s_e[3 * COUT + c] = rstd;
    }
  }

  // ---- weights: global [Cout][3][3][Cin] -> LDS [tap][Cout][CinP] ------------------------
  {
    const int nchunk = COUT * 9 * C8;
    constexpr int RU = 8;
    for (int base = tid; base < nchunk; base += NT * RU) {
      uint4 v[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        int q = base + u * NT;
        q = q < nchunk ? q : nchunk - 1;
        v[u] = *reinterpret_cast<const uint4*>(a.w + (size_t)q * 8);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        int q = base + u * NT;
        if (q >= nchunk) break;
        int c8 = q % C8, t = q / C8, tap = t % 9, n = t / 9;
        *reinterpret_cast<uint4*>(s_w + ((size_t)tap * COUT + n) * CinP + c8 * 8) = v[u];
      }
    }
  }
  __syncthreads();  // BN tables visible before the halo transform

  // ---- halo: interior pixels (BN + act applied), zero ring --------------------------------
  {
    const int nchunk = g.npix * C8;
    const size_t img_off = (size_t)img * g.npix;
    const float pro_lo = act_lo(a.pro.act), pro_hi = act_hi(a.pro.act);
    constexpr int RU = 4;
    for (int base = tid; base < nchunk; base += NT * RU) {
      float v[RU][8];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        int q = base + u * NT;
        q = q < nchunk ? q : nchunk - 1;
        int c8 = q % C8, p = q / C8;
        const size_t off = (img_off + p) * a.ldx + c8 * 8;
        if constexpr (sizeof(TA) == 4) {
          const float* xp = reinterpret_cast<const float*>(a.x) + off;
          float4 lo = *reinterpret_cast<const float4*>(xp);
          float4 hi = *reinterpret_cast<const float4*>(xp + 4);
          v[u][0] = lo.x; v[u][1] = lo.y; v[u][2] = lo.z; v[u][3] = lo.w;
          v[u][4] = hi.x; v[u][5] = hi.y; v[u][6] = hi.z; v[u][7] = hi.w;
        } else {
          unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.x) + off), v[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        int q = base + u * NT;
        if (q >= nchunk) break;
        int c8 = q % C8, p = q / C8;
        int h = p / a.W, w = p - h * a.W;
        if constexpr (PRO) affine_act8(v[u], s_scale + c8 * 8, s_shift + c8 * 8, pro_lo, pro_hi);
        *reinterpret_cast<uint4*>(s_halo + ((size_t)(h + 1) * g.Wp + (w + 1)) * CinP + c8 * 8) = pack8(v[u]);
      }
    }
    // zero ring: rows 0 and Hp-1, columns 0 and Wp-1
    const int ring = 2 * g.Wp + 2 * a.H;
    for (int q = tid; q < ring * C8; q += NT) {
      int c8 = q % C8, r = q / C8, hh, ww;
      if (r < g.Wp) { hh = 0; ww = r; }
      else if (r < 2 * g.Wp) { hh = g.Hp - 1; ww = r - g.Wp; }
      else if (r < 2 * g.Wp + a.H) { hh = r - 2 * g.Wp + 1; ww = 0; }
      else { hh = r - 2 * g.Wp - a.H + 1; ww = g.Wp - 1; }
      *reinterpret_cast<uint4*>(s_halo + ((size_t)hh * g.Wp + ww) * CinP + c8 * 8) = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();

  // ---- MFMA sweep ------------------------------------------------------------------------
  const int frow = lane & 15, fk = lane >> 4;
  v4f acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  int hbase[MT];  // halo element offset of this lane's output pixel, tap (0,0)
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int mt = wid + 4 * i;
    int p = mt * 16 + frow;
    p = p < g.npix ? p : g.npix - 1;  // padding rows: computed, never stored
    int h = p / a.W, w = p - h * a.W;
    hbase[i] = (h * g.Wp + w) * CinP + fk * 8;
  }
  const bool active0 = wid < g.mtiles;
  if (active0) {
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap - r * 3;
      const int toff = (r * g.Wp + s) * CinP;
      const bf16_t* wt = s_w + (size_t)tap * COUT * CinP + frow * CinP + fk * 8;
      for (int ks = 0; ks < Cin; ks += 32) {
        v8bf bfr[NTL];
#pragma unroll
        for (int j = 0; j < NTL; ++j) bfr[j] = *reinterpret_cast<const v8bf*>(wt + j * 16 * CinP + ks);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          if (wid + 4 * i >= g.mtiles) break;
          v8bf af = *reinterpret_cast<const v8bf*>(s_halo + hbase[i] + toff + ks);
#pragma unroll
          for (int j = 0; j < NTL; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: per wave, one 16-row tile at a time through its private staging tile -------
  constexpr int SLD = COUT + 4;
  float* st = s_stage + wid * 16 * SLD;
  constexpr int CPB = COUT / 8;             // 16-B chunks per row
  constexpr int ITER = (16 * CPB + 63) / 64;
  float psum[8], psq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { psum[j] = 0.f; psq[j] = 0.f; }
  const int my_c8 = lane % CPB;
  float t_k[8];  // statistics shift of this lane's chunk (common.h "Shifted statistics")
#pragma unroll
  for (int j = 0; j < 8; ++j) t_k[j] = (EPI == 0 && a.stats_shift) ? a.stats_shift[my_c8 * 8 + j] : 0.f;
  const float epi_lo = act_lo(a.epi_act), epi_hi = act_hi(a.epi_act);
  const float msk_lo = act_lo(a.mbn.act), msk_hi = act_hi(a.mbn.act);
  const size_t out_img = (size_t)img * g.npix;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int mt = wid + 4 * i;
    if (mt >= g.mtiles) break;
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(fk * 4 + r) * SLD + j * 16 + frow] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = lane + it * 64;
      const int lrow = idx / CPB, c8 = idx % CPB;
      const int p = mt * 16 + lrow;
      if (idx < 16 * CPB && p < g.npix) {
        const int n = c8 * 8;
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(st + lrow * SLD + n);
        const float4 hi = *reinterpret_cast<const float4*>(st + lrow * SLD + n + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        const size_t m = out_img + p;
        if constexpr (EPI == 0) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = fminf(fmaxf(v[jj], epi_lo), epi_hi);
          uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + m * a.ldy + n) = pk;
          float rr[8];
          unpack8(pk, rr);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const float dj = rr[jj] - t_k[jj];
            psum[jj] += dj;
            psq[jj] += dj * dj;
          }
        } else {
          float xf[8], d[8];
          unpack8(*reinterpret_cast<const uint4*>(a.mx + m * a.ldmx + n), xf);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            float z = xf[jj] * s_e[n + jj] + s_e[COUT + n + jj];
            d[jj] = (z > msk_lo && z < msk_hi) ? v[jj] : 0.f;
          }
          uint4 pk = pack8(d);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + m * a.ldy + n) = pk;
          float rr[8];
          unpack8(pk, rr);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            psum[jj] += rr[jj];
            psq[jj] += rr[jj] * (xf[jj] - s_e[2 * COUT + n + jj]) * s_e[3 * COUT + n + jj];
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // staging tile reused by the next m tile
  }
  const bool want = (EPI == 1) || (a.stats_out != nullptr);
  if (want) {
    wave_reduce_chunks<CPB < 64 ? CPB : 64>(psum);
    wave_reduce_chunks<CPB < 64 ? CPB : 64>(psq);
    if (lane < CPB) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        atomicAdd(&s_sum[my_c8 * 8 + jj], psum[jj]);
        atomicAdd(&s_sq[my_c8 * 8 + jj], psq[jj]);
      }
    }
    __syncthreads();
    // one workgroup per image: the image index picks the statistics slot
    const size_t so = EPI == 0 ? (size_t)(blockIdx.x % stat_slots(a.stats_slots)) * 2 * a.stats_ld
                               : (size_t)(blockIdx.x % stat_slots(a.gsum_slots)) * a.gsum_ld;
    for (int c = tid; c < COUT; c += NT) {
      if constexpr (EPI == 0) {
        atomicAdd(&a.stats_out[so + a.stats_off + c], s_sum[c]);
        atomicAdd(&a.stats_out[so + a.stats_ld + a.stats_off + c], s_sq[c]);
      } else {
        if (a.gsum) atomicAdd(&a.gsum[so + c], s_sum[c]);
        if (a.gsumx) atomicAdd(&a.gsumx[so + c], s_sq[c]);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
bool conv3x3_halo_ok(const ConvArgs& a) {
  if (a.KH != 3 || a.KW != 3 || a.SH != 1 || a.SW != 1 || a.PT != 1 || a.PL != 1) return false;
  if (a.Ho != a.H || a.Wo != a.W || (a.Cin % 32) || (a.ldx % 8) || (a.ldy % 8)) return false;
  if (a.Cout != 32 && a.Cout != 64 && a.Cout != 128) return false;
  if (a.bpro.mode != 0 || a.epi_mode > 1) return false;  // backward-affine forms: igemm only
  if (a.epi_mode == 0 && (a.bias != nullptr || a.out_mode != OUT_BF16)) return false;
  const int mtiles = (a.H * a.W + 15) / 16;
  if (mtiles > 16) return false;
  const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  HaloGeom g = halo_geom(a.H, a.W, a.Cin, a.Cout, pro, a.epi_mode);
  return g.halo_bytes + g.w_bytes + g.stage_bytes + g.table_bytes <= 160 * 1024;
}

template <int COUT, typename TA, int PRO, int EPI>
static hipError_t halo_launch_mt(const ConvArgs& a, int mt, size_t shm, hipStream_t st) {
  dim3 grid(a.N), block(NT);
  switch (mt) {
    case 1: hipLaunchKernelGGL((conv3x3_halo_kernel<COUT, 1, TA, PRO, EPI>), ggrid(grid), block, shm, st, a, garg()); break;
    case 2: hipLaunchKernelGGL((conv3x3_halo_kernel<COUT, 2, TA, PRO, EPI>), ggrid(grid), block, shm, st, a, garg()); break;
    case 3: hipLaunchKernelGGL((conv3x3_halo_kernel<COUT, 3, TA, PRO, EPI>), ggrid(grid), block, shm, st, a, garg()); break;
    default: hipLaunchKernelGGL((conv3x3_halo_kernel<COUT, 4, TA, PRO, EPI>), ggrid(grid), block, shm, st, a, garg()); break;
  }
  return hipGetLastError();
}

template <int COUT>
static hipError_t halo_launch(const ConvArgs& a, bool a_f32, int pro, int mt, size_t shm, hipStream_t st) {
  if (a_f32) {
    if (pro) return hipErrorInvalidValue;
    return a.epi_mode ? halo_launch_mt<COUT, float, 0, 1>(a, mt, shm, st)
                      : halo_launch_mt<COUT, float, 0, 0>(a, mt, shm, st);
  }
  if (pro)
    return a.epi_mode ? halo_launch_mt<COUT, bf16_t, 1, 1>(a, mt, shm, st)
                      : halo_launch_mt<COUT, bf16_t, 1, 0>(a, mt, shm, st);
  return a.epi_mode ? halo_launch_mt<COUT, bf16_t, 0, 1>(a, mt, shm, st)
                    : halo_launch_mt<COUT, bf16_t, 0, 0>(a, mt, shm, st);
}

hipError_t conv3x3_halo(const ConvArgs& a, bool a_f32, hipStream_t st) {
  if (!conv3x3_halo_ok(a)) return hipErrorInvalidValue;
  if (a.N == 0) return hipSuccess;
  const int pro = (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  HaloGeom g = halo_geom(a.H, a.W, a.Cin, a.Cout, pro, a.epi_mode);
  const size_t shm = g.halo_bytes + g.w_bytes + g.stage_bytes + g.table_bytes;
  const int mt = (g.mtiles + 3) / 4;
  switch (a.Cout) {
    case 32: return halo_launch<32>(a, a_f32, pro, mt, shm, st);
    case 64: return halo_launch<64>(a, a_f32, pro, mt, shm, st);
    default: return halo_launch<128>(a, a_f32, pro, mt, shm, st);
  }
}

}  // namespace idc
