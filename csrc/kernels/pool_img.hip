// Image-resident overlapping max pool, gfx950: DenseNet's stem pool (3x3 / 2, pad 1, 25x25 -> 13x13
// on 50x50 patches; Keras DenseNet121's pool1 after ZeroPadding2D, which the reference builds through
// keras.applications in /root/reference/dist_model_tf_dense.py), forward and backward.
//
// The row kernels (nn_kernels.hip pool_fwd_kernel / pool_bwd_kernel) give every thread one
// 8-channel chunk of a few pixels and grid-stride over the map: the forward re-reads each input
// chunk ~2.25 times (9 taps per window at stride 2) and re-applies the pending BatchNorm to it each
// time; the backward gathers, for every input pixel, the <= 4 windows containing it -- dy, the
// argmax bytes and the later BatchNorm's pending-affine input per window, so each window's
// operands are loaded and transformed 4 times.  Both ran as latency chains of several dependent
// memory round trips per thread (bench profile, round 5: 29 us forward, 59 us backward on 20 MB of
// activations).
//
// Here a workgroup owns ONE image x 16 channels:
//   forward:  the activated input map (BN + act applied once per element) goes to LDS as fp32
//             (H*W*16*4 B: 40 KB at 25x25), then every window reads its taps from LDS -- one global
//             round trip per workgroup, every load issued before any arithmetic;
//   backward: every window's transformed gradient dy' (pending affine applied once) and argmax
//             bytes go to LDS (Ho*Wo*16*5 B: 13.5 KB at 13x13), then every input pixel gathers its
//             windows from LDS in the row kernel's order (same sums, same rounding), applies the
//             backward of the BN+act that fed the pool and reduces its sums.
// Statistics / gradient sums are reduced per workgroup (16 channels) and added once per channel,
// into slot copy (image % slots): the workgroups of one channel group spread over every copy.
#include "nn_kernels.h"

#include <cstdlib>

namespace idc {

namespace {

constexpr int NT = 256;
constexpr int CG = 16;          // channels per workgroup (two 8-channel chunks)
constexpr int FWD_LDS = 48 * 1024;
constexpr int BWD_LDS = 48 * 1024;

__device__ __forceinline__ void load8(const void* base, int f32, size_t off, float* v) {
  if (f32) {
    const float* p = reinterpret_cast<const float*>(base) + off;
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(base) + off), v);
  }
}

// per-channel block totals of the (chunk = tid & 1) partials: lanes of equal parity within the
// wave, then the 4 waves through LDS; thread t < 16 returns channel t's totals
__device__ __forceinline__ void reduce16(float (&pa)[8], float (&pb)[8], float* red, float& ra, float& rb) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int sh = 2; sh < 64; sh <<= 1) {
      pa[j] += __shfl_xor(pa[j], sh, 64);
      pb[j] += __shfl_xor(pb[j], sh, 64);
    }
  }
  __syncthreads();  // (red may alias LDS the caller just finished reading)
  if (lane < 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wid * 2 + lane) * 16 + j] = pa[j];
      red[(wid * 2 + lane) * 16 + 8 + j] = pb[j];
    }
  }
  __syncthreads();
  ra = rb = 0.f;
  if (tid < CG) {
    const int u = tid >> 3, j = tid & 7;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      ra += red[(w * 2 + u) * 16 + j];
      rb += red[(w * 2 + u) * 16 + 8 + j];
    }
  }
}

}  // namespace

// (outside the anonymous namespace so profiles name them)
__global__ __launch_bounds__(NT) void maxpool_img_fwd_kernel(PoolArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(PoolArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  const int tid = threadIdx.x;
  const int G = a.C / CG;
  const int img = blockIdx.x / G, c0 = (blockIdx.x - img * G) * CG;
  const int HW = a.H * a.W, HWo = a.Ho * a.Wo;
  float* sv = smem_f;                 // [HW][16] activated input
  float* s_sc = sv + HW * CG;         // [16]
  float* s_sh = s_sc + CG;
  float* red = s_sh + CG;             // [8][16]
  const bf16_t* __restrict__ X = a.x + (size_t)img * HW * a.ldx + c0;

  // the whole map's loads first (up to 5 chunks per thread at 25x25), then the coefficient table
  // (its loads overlap them), then the activation into LDS
  constexpr int RU = 5;
  const int items = HW * 2;
  if (tid < CG) {
    float sc, sh;
    bn_coeffs(a.pro, c0 + tid, sc, sh);
    s_sc[tid] = sc;
    s_sh[tid] = sh;
  }
  const int npass = (items + RU * NT - 1) / (RU * NT);  // (uniform: the first pass holds a barrier)
  for (int pass = 0; pass < npass; ++pass) {
    const int i0 = pass * RU * NT + tid;
    uint4 raw[RU];
#pragma unroll
    for (int r = 0; r < RU; ++r) {
      const int i = min(i0 + r * NT, items - 1);
      raw[r] = *reinterpret_cast<const uint4*>(X + (size_t)(i >> 1) * a.ldx + (i & 1) * 8);
    }
    if (pass == 0) __syncthreads();  // the coefficient table
#pragma unroll
    for (int r = 0; r < RU; ++r) {
      const int i = i0 + r * NT;
      if (i >= items) break;
      const int u = i & 1;
      float v[8];
      unpack8(raw[r], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j] * s_sc[u * 8 + j] + s_sh[u * 8 + j], a.pro.act);
      float4* d = reinterpret_cast<float4*>(sv + (size_t)(i >> 1) * CG + u * 8);
      d[0] = make_float4(v[0], v[1], v[2], v[3]);
      d[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
  __syncthreads();

  const int u = tid & 1;  // this thread's chunk in every window item (NT is even)
  float kk[8], ps[8], pq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    kk[j] = a.stats_shift ? a.stats_shift[c0 + u * 8 + j] : 0.f;
    ps[j] = pq[j] = 0.f;
  }
  const int k = a.k;
  for (int o = tid; o < HWo * 2; o += NT) {
    const int po = o >> 1;
    const int ho = po / a.Wo, wo = po - ho * a.Wo;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -3.4e38f; arg[j] = 0; }
    for (int q = 0; q < k * k; ++q) {
      const int r = q / k, s2 = q - r * k;
      const int h = ho * a.s - a.pt + r, w = wo * a.s - a.pl + s2;
      float v[8];
      if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
        const float4* p = reinterpret_cast<const float4*>(sv + (size_t)(h * a.W + w) * CG + u * 8);
        const float4 lo = p[0], hi = p[1];
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;  // Keras ZeroPadding before the pool
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j] > best[j]) { best[j] = v[j]; arg[j] = (uint8_t)q; }
    }
    const uint4 p = pack8(best);
    const size_t orow = (size_t)img * HWo + po;
    *reinterpret_cast<uint4*>(a.y + orow * a.ldy + c0 + u * 8) = p;
    if (a.argmax) {
      uint2 ar;
      ar.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
      ar.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
      *reinterpret_cast<uint2*>(a.argmax + orow * a.C + c0 + u * 8) = ar;
    }
    if (a.stats) {
      float out[8];
      unpack8(p, out);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dj = out[j] - kk[j];
        ps[j] += dj;
        pq[j] += dj * dj;
      }
    }
  }
  if (a.stats) {
    float ra, rb;
    reduce16(ps, pq, red, ra, rb);
    if (tid < CG) {
      float* so = a.stats + (size_t)(img % stat_slots(a.stats_slots)) * 2 * a.stats_ld + a.stats_off;
      atomicAdd(so + c0 + tid, ra);
      atomicAdd(so + a.stats_ld + c0 + tid, rb);
    }
  }
}

__global__ __launch_bounds__(NT) void maxpool_img_bwd_kernel(PoolBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(PoolBwdArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  const int tid = threadIdx.x;
  const int G = a.C / CG;
  const int img = blockIdx.x / G, c0 = (blockIdx.x - img * G) * CG;
  const int HW = a.H * a.W, HWo = a.Ho * a.Wo;
  float* sd = smem_f;                                           // [HWo][16] dy'
  float* s_sc = sd + HWo * CG;                                  // epilogue BN: scale, shift, mean, rstd
  float* s_sh = s_sc + CG;
  float* s_mu = s_sh + CG;
  float* s_rs = s_mu + CG;
  float* s_da = s_rs + CG;                                      // dy affine A, B, C
  float* s_db = s_da + CG;
  float* s_dc = s_db + CG;
  float* red = s_dc + CG;                                       // [8][16]
  uint8_t* sam = reinterpret_cast<uint8_t*>(red + 8 * CG);      // [HWo][16] argmax bytes
  const bool epi = (a.bn.mode != 0 || a.bn.act != ACT_NONE);
  const bool dyaff = a.dyaff.mode != 0;

  // ---- window operands: loads first (<= 2 items per thread at 13x13), tables meanwhile
  constexpr int RW = 2;
  const int witems = HWo * 2;
  const size_t wrow0 = (size_t)img * HWo;
  if (tid < CG) {
    const int c = c0 + tid;
    float sc = 1.f, sh = 0.f, mean = 0.f, rstd = 1.f;
    if (a.bn.mode) {
      bn_mean_rstd(a.bn, c, mean, rstd);
      const float g = a.bn.gamma ? a.bn.gamma[c] : 1.f;
      const float be = a.bn.beta ? a.bn.beta[c] : 0.f;
      sc = g * rstd;
      sh = be - mean * sc;
    }
    s_sc[tid] = sc; s_sh[tid] = sh; s_mu[tid] = mean; s_rs[tid] = rstd;
  }
  if (dyaff) {
    bwd_aff_table<NT>(a.dyaff, c0, CG, a.C, s_da, s_db, s_dc);
    bwd_aff_fold<NT>(a.dyaff);
  }
  __syncthreads();
  for (int o0 = tid; o0 < witems; o0 += RW * NT) {
    float d[RW][8];
    uint4 xo[RW];
    uint2 am[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int o = min(o0 + r * NT, witems - 1);
      const size_t row = wrow0 + (o >> 1);
      const int c = c0 + (o & 1) * 8;
      load8(a.dy, a.dy_f32, row * a.lddy + c, d[r]);
      if (dyaff) xo[r] = *reinterpret_cast<const uint4*>(a.dyaff.x + row * a.dyaff.ldx + c);
      am[r] = *reinterpret_cast<const uint2*>(a.argmax + row * a.C + c);
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int o = o0 + r * NT;
      if (o >= witems) break;
      const int u = o & 1;
      if (dyaff) {
        float xf[8];
        unpack8(xo[r], xf);
        bwd_aff8(d[r], xf, s_da + u * 8, s_db + u * 8, s_dc + u * 8);
      }
      float4* dst = reinterpret_cast<float4*>(sd + (size_t)(o >> 1) * CG + u * 8);
      dst[0] = make_float4(d[r][0], d[r][1], d[r][2], d[r][3]);
      dst[1] = make_float4(d[r][4], d[r][5], d[r][6], d[r][7]);
      *reinterpret_cast<uint2*>(sam + (size_t)(o >> 1) * CG + u * 8) = am[r];
    }
  }
  __syncthreads();

  // ---- input pixels: gather the <= 2 x 2 windows containing each (the row kernel's order)
  constexpr int RU = 5;
  const int items = HW * 2;
  const int u = tid & 1;
  const float lo = act_lo(a.bn.act), hi = act_hi(a.bn.act);
  float ps[8], px[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ps[j] = px[j] = 0.f;
  const size_t irow0 = (size_t)img * HW;
  for (int i0 = tid; i0 < items; i0 += RU * NT) {
    uint4 xr[RU];
    if (epi) {
#pragma unroll
      for (int r = 0; r < RU; ++r) {
        const int i = min(i0 + r * NT, items - 1);
        xr[r] = *reinterpret_cast<const uint4*>(a.x + (irow0 + (i >> 1)) * a.ldx + c0 + (i & 1) * 8);
      }
    }
#pragma unroll
    for (int r = 0; r < RU; ++r) {
      const int i = i0 + r * NT;
      if (i >= items) break;
      const int p = i >> 1;
      const int h = p / a.W, w = p - h * a.W;
      int oh_lo = h + a.pt - a.k + 1 + a.s - 1;
      oh_lo = oh_lo < 0 ? 0 : oh_lo / a.s;
      int oh_hi = (h + a.pt) / a.s;
      int ow_lo = w + a.pl - a.k + 1 + a.s - 1;
      ow_lo = ow_lo < 0 ? 0 : ow_lo / a.s;
      int ow_hi = (w + a.pl) / a.s;
      oh_hi = oh_hi < a.Ho - 1 ? oh_hi : a.Ho - 1;
      ow_hi = ow_hi < a.Wo - 1 ? ow_hi : a.Wo - 1;
      float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int dw = 0; dw < 2; ++dw) {
          const int oh = oh_lo + dh, ow = ow_lo + dw;
          if (oh > oh_hi || ow > ow_hi) continue;
          const int po = oh * a.Wo + ow;
          const uint8_t mine = (uint8_t)((h - (oh * a.s - a.pt)) * a.k + (w - (ow * a.s - a.pl)));
          const float4* dp = reinterpret_cast<const float4*>(sd + (size_t)po * CG + u * 8);
          const float4 d0 = dp[0], d1 = dp[1];
          const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
          const uint2 ar = *reinterpret_cast<const uint2*>(sam + (size_t)po * CG + u * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t word = j < 4 ? ar.x : ar.y;
            const uint8_t b = (uint8_t)(word >> (8 * (j & 3)));
            g[j] += (b == mine) ? dv[j] : 0.f;
          }
        }
      const size_t orow = irow0 + p;
      if (epi) {
        float x[8];
        unpack8(xr[r], x);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cj = u * 8 + j;
          const float z = x[j] * s_sc[cj] + s_sh[cj];
          g[j] = (z > lo && z < hi) ? g[j] : 0.f;
        }
        if (a.dx_f32) {
          float o8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int cj = u * 8 + j;
            o8[j] = s_sc[cj] * g[j];
            ps[j] += g[j];
            px[j] += g[j] * (x[j] - s_mu[cj]) * s_rs[cj];
          }
          float* q = reinterpret_cast<float*>(a.dx) + orow * a.lddx + c0 + u * 8;
          *reinterpret_cast<float4*>(q) = make_float4(o8[0], o8[1], o8[2], o8[3]);
          *reinterpret_cast<float4*>(q + 4) = make_float4(o8[4], o8[5], o8[6], o8[7]);
        } else {
          const uint4 pk = pack8(g);
          *reinterpret_cast<uint4*>(a.dx + orow * a.lddx + c0 + u * 8) = pk;
          unpack8(pk, g);  // reduce exactly what was stored
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int cj = u * 8 + j;
            ps[j] += g[j];
            px[j] += g[j] * (x[j] - s_mu[cj]) * s_rs[cj];
          }
        }
      } else {
        *reinterpret_cast<uint4*>(a.dx + orow * a.lddx + c0 + u * 8) = pack8(g);
      }
    }
  }
  if (epi && (a.gsum || a.gsumx)) {
    float ra, rb;
    reduce16(ps, px, red, ra, rb);
    if (tid < CG) {
      const size_t so = (size_t)(img % stat_slots(a.gsum_slots)) * a.gsum_ld;
      if (a.gsum) atomicAdd(a.gsum + so + c0 + tid, ra);
      if (a.gsumx) atomicAdd(a.gsumx + so + c0 + tid, rb);
    }
  }
}

namespace {

bool pool_img_on() {
  static const bool on = [] {
    const char* e = std::getenv("IDC_POOL_IMG");
    return !(e && e[0] == '0');
  }();
  return on;
}

size_t fwd_lds(const PoolArgs& a) { return ((size_t)a.H * a.W * CG + 2 * CG + 8 * CG) * 4; }
size_t bwd_lds(const PoolBwdArgs& a) { return ((size_t)a.Ho * a.Wo * CG + 7 * CG + 8 * CG) * 4 + (size_t)a.Ho * a.Wo * CG; }

}  // namespace

bool maxpool_img_fwd_ok(const PoolArgs& a) {
  // overlapping windows only (k > s: the stem pool): the non-overlapping VGG16 pools read every
  // input once already and measured faster on the row kernel (2.396 vs 2.438 ms/step)
  return pool_img_on() && a.k > a.s && a.C % CG == 0 && a.ldx % 8 == 0 && a.ldy % 8 == 0 && a.k >= 1 && a.k * a.k <= 255 &&
         a.s >= 1 && a.pt >= 0 && a.pl >= 0 && a.Ho > 0 && a.Wo > 0 && fwd_lds(a) <= FWD_LDS &&
         (a.stats == nullptr || a.stats_slots <= MAX_STAT_SLOTS);
}

bool maxpool_img_bwd_ok(const PoolBwdArgs& a) {
  const bool epi = a.bn.mode != 0 || a.bn.act != ACT_NONE;
  // k <= 2s: at most 2 x 2 windows contain an input pixel
  return pool_img_on() && !a.is_avg && a.argmax != nullptr && a.C % CG == 0 && a.k <= 2 * a.s && a.k * a.k <= 255 &&
         a.lddy % 8 == 0 && a.lddx % 8 == 0 && (!epi || a.ldx % 8 == 0) && (a.dx_f32 ? epi : true) &&
         (a.dyaff.mode == 0 || (a.dyaff.x != nullptr && a.dyaff.ldx % 8 == 0)) && bwd_lds(a) <= BWD_LDS &&
         (!epi || !(a.gsum || a.gsumx) || a.gsum_slots <= MAX_STAT_SLOTS);
}

hipError_t maxpool_img_fwd(const PoolArgs& a, hipStream_t st) {
  if (!maxpool_img_fwd_ok(a)) return hipErrorInvalidValue;
  const int grid = a.N * (a.C / CG);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(maxpool_img_fwd_kernel, ggrid(grid), dim3(NT), fwd_lds(a), st, a, garg());
  return hipGetLastError();
}

hipError_t maxpool_img_bwd(const PoolBwdArgs& a, hipStream_t st) {
  if (!maxpool_img_bwd_ok(a)) return hipErrorInvalidValue;
  const int grid = a.N * (a.C / CG);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(maxpool_img_bwd_kernel, ggrid(grid), dim3(NT), bwd_lds(a), st, a, garg());
  return hipGetLastError();
}

}  // namespace idc
