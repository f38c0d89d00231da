// Depthwise 3x3 convolution for MobileNetV2 (stride 1 'same', stride 2 with Keras correct_pad
// asymmetric padding), NHWC bf16, gfx950.  Pure bandwidth (9 FMAs per loaded element): a thread
// owns one output pixel x 8 channels with 16-B vector loads; the pending BN+ReLU6 of the producer
// (expand conv) is applied on load, output statistics for the depthwise BN are reduced in the
// epilogue, so neither BN needs its own pass.  Backward data is a gather over the (<= 9) output
// positions that read each input pixel, with the BN-backward epilogue (dZ, sum dZ, sum dZ*xhat);
// weight grad reduces over pixels per (tap, channel) with one atomic per block and channel.
#include "common.h"
#include "dwconv.h"

namespace idc {

namespace {
struct Map8 {
  int C8, R, tx, ty;
  __device__ Map8(int C) {
    C8 = C / 8;
    R = 256 / C8;
    if (R < 1) R = 1;
    tx = threadIdx.x % C8;
    ty = threadIdx.x / C8;
  }
};
inline int nblocks(long long rows, int C, int rows_per_thread) {
  int C8 = C / 8, R = 256 / C8;
  if (R < 1) R = 1;
  long long b = (rows + (long long)R * rows_per_thread - 1) / ((long long)R * rows_per_thread);
  if (b > 4096) b = 4096;
  return b < 1 ? 1 : (int)b;
}
}  // namespace

__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sf = sh + a.C;
  float* s_a = sh + 2 * a.C;
  float* s_b = sh + 3 * a.C;
  const bool ident = a.pro.mode == 0 && a.pro.act == ACT_NONE;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    bn_coeffs(a.pro, c, s_sc[c], s_sf[c]);
    s_a[c] = 0.f;
    s_b[c] = 0.f;
  }
  __syncthreads();
  Map8 mp(a.C);
  const int Mo = a.N * a.Ho * a.Wo;
  if (mp.ty < mp.R) {
    const int c = mp.tx * 8;
    float ps[8] = {0}, pq[8] = {0};
    for (int o = blockIdx.x * mp.R + mp.ty; o < Mo; o += gridDim.x * mp.R) {
      int wo = o % a.Wo, t = o / a.Wo, ho = t % a.Ho, n = t / a.Ho;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int r = 0; r < a.KH; ++r) {
        int h = ho * a.S - a.PT + r;
        if ((unsigned)h >= (unsigned)a.H) continue;
        for (int s = 0; s < a.KW; ++s) {
          int w = wo * a.S - a.PL + s;
          if ((unsigned)w >= (unsigned)a.W) continue;
          float v[8];
          unpack8(*reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.ldx + c), v);
          const float* wp = a.w + (size_t)(r * a.KW + s) * a.C + c;
          float4 w0 = *reinterpret_cast<const float4*>(wp);
          float4 w1 = *reinterpret_cast<const float4*>(wp + 4);
          float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float u = ident ? v[j] : apply_act(v[j] * s_sc[c + j] + s_sf[c + j], a.pro.act);
            acc[j] += u * wk[j];
          }
        }
      }
      uint4 p = pack8(acc);
      *reinterpret_cast<uint4*>(a.y + (size_t)o * a.ldy + c) = p;
      if (a.stats) {
        unpack8(p, acc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dj = acc[j] - (a.stats_shift ? a.stats_shift[c + j] : 0.f);
          ps[j] += dj;
          pq[j] += dj * dj;
        }
      }
    }
    if (a.stats) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { atomicAdd(&s_a[c + j], ps[j]); atomicAdd(&s_b[c + j], pq[j]); }
    }
  }
  if (a.stats) {
    __syncthreads();
    float* so = a.stats + (size_t)(blockIdx.x % stat_slots(a.stats_slots)) * 2 * a.stats_ld;
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      atomicAdd(&so[c], s_a[c]);
      atomicAdd(&so[a.stats_ld + c], s_b[c]);
    }
  }
}

__global__ __launch_bounds__(256) void dw_bwd_data_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sf = sh + a.C;
  float* s_mu = sh + 2 * a.C;
  float* s_rs = sh + 3 * a.C;
  float* s_a = sh + 4 * a.C;
  float* s_b = sh + 5 * a.C;
  const bool epi = !(a.pro.mode == 0 && a.pro.act == ACT_NONE);
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    bn_coeffs(a.pro, c, s_sc[c], s_sf[c]);
    float mean = 0.f, rstd = 1.f;
    if (a.pro.mode) bn_mean_rstd(a.pro, c, mean, rstd);
    s_mu[c] = mean; s_rs[c] = rstd; s_a[c] = 0.f; s_b[c] = 0.f;
  }
  __syncthreads();
  Map8 mp(a.C);
  const int Mi = a.N * a.H * a.W;
  if (mp.ty < mp.R) {
    const int c = mp.tx * 8;
    float ps[8] = {0}, px[8] = {0};
    for (int i = blockIdx.x * mp.R + mp.ty; i < Mi; i += gridDim.x * mp.R) {
      int w = i % a.W, t = i / a.W, h = t % a.H, n = t / a.H;
      float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int r = 0; r < a.KH; ++r) {
        int th = h + a.PT - r;
        if (th < 0 || th % a.S) continue;
        int ho = th / a.S;
        if (ho >= a.Ho) continue;
        for (int s = 0; s < a.KW; ++s) {
          int tw = w + a.PL - s;
          if (tw < 0 || tw % a.S) continue;
          int wo = tw / a.S;
          if (wo >= a.Wo) continue;
          float d[8];
          unpack8(*reinterpret_cast<const uint4*>(a.dy + ((size_t)(n * a.Ho + ho) * a.Wo + wo) * a.lddy + c), d);
          const float* wp = a.w + (size_t)(r * a.KW + s) * a.C + c;
          float4 w0 = *reinterpret_cast<const float4*>(wp);
          float4 w1 = *reinterpret_cast<const float4*>(wp + 4);
          float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] += d[j] * wk[j];
        }
      }
      if (epi) {
        float x[8];
        unpack8(*reinterpret_cast<const uint4*>(a.x + (size_t)i * a.ldx + c), x);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] *= act_mask(x[j] * s_sc[c + j] + s_sf[c + j], a.pro.act);
        uint4 p = pack8(g);
        *reinterpret_cast<uint4*>(a.dx + (size_t)i * a.lddx + c) = p;
        unpack8(p, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) { ps[j] += g[j]; px[j] += g[j] * (x[j] - s_mu[c + j]) * s_rs[c + j]; }
      } else {
        *reinterpret_cast<uint4*>(a.dx + (size_t)i * a.lddx + c) = pack8(g);
      }
    }
    if (epi) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { atomicAdd(&s_a[c + j], ps[j]); atomicAdd(&s_b[c + j], px[j]); }
    }
  }
  if (epi) {
    __syncthreads();
    const size_t so = (size_t)(blockIdx.x % stat_slots(a.gsum_slots)) * a.gsum_ld;
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      if (a.gsum) atomicAdd(&a.gsum[so + c], s_a[c]);
      if (a.gsumx) atomicAdd(&a.gsumx[so + c], s_b[c]);
    }
  }
}

__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sf = sh + a.C;
  float* s_acc = sh + 2 * a.C;  // [KH*KW][C]
  const int T = a.KH * a.KW;
  const bool ident = a.pro.mode == 0 && a.pro.act == ACT_NONE;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) bn_coeffs(a.pro, c, s_sc[c], s_sf[c]);
  for (int k = threadIdx.x; k < T * a.C; k += blockDim.x) s_acc[k] = 0.f;
  __syncthreads();
  Map8 mp(a.C);
  const int Mo = a.N * a.Ho * a.Wo;
  if (mp.ty < mp.R) {
    const int c = mp.tx * 8;
    float acc[9][8];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
    for (int o = blockIdx.x * mp.R + mp.ty; o < Mo; o += gridDim.x * mp.R) {
      int wo = o % a.Wo, t = o / a.Wo, ho = t % a.Ho, n = t / a.Ho;
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(a.dy + (size_t)o * a.lddy + c), d);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        int h = ho * a.S - a.PT + r;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          int w = wo * a.S - a.PL + s;
          if (r >= a.KH || s >= a.KW) continue;
          if ((unsigned)h >= (unsigned)a.H || (unsigned)w >= (unsigned)a.W) continue;
          float v[8];
          unpack8(*reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.ldx + c), v);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float u = ident ? v[j] : apply_act(v[j] * s_sc[c + j] + s_sf[c + j], a.pro.act);
            acc[r * 3 + s][j] += u * d[j];
          }
        }
      }
    }
    for (int r = 0; r < a.KH; ++r)
      for (int s = 0; s < a.KW; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(&s_acc[(r * a.KW + s) * a.C + c + j], acc[r * 3 + s][j]);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < T * a.C; k += blockDim.x) atomicAdd(&a.dw[k], s_acc[k]);
}

// ---- 3x3 strip kernels -------------------------------------------------------------------
// A thread owns one 8-channel chunk and a strip of P consecutive pixels along W: the 3 x
// ((P-1)*S + 3) input vectors of the strip are loaded once and feed every output that reads
// them (stride 1: 18 loads for 4 outputs instead of 36), the chunk's 9 taps and BN coefficients
// sit in registers for the whole grid-stride loop, the pending BN + activation is a branch-free
// clamp, and padding taps are masked after the activation (Keras pads the activated tensor).
constexpr int kDwStrip = 4;

// Strip-kernel geometry: a block owns c8b 8-channel chunks (c8b = the largest divisor of C/8 that
// is <= 8: 64, 48 or fewer channels) x R = 256 / c8b strips in flight, blockIdx.y = channel
// chunk.  A block holding ALL C channels (C/8 chunks x 256/(C/8) rows) left MobileNetV2's deep
// layers (C 384-960: 2-5 strip rows per block) with a few dozen long-running blocks on 256 CUs.
struct DwChunks {
  int c8b, nchunk, R;
};
__host__ __device__ inline DwChunks dw_chunks(int C) {
  const int C8 = C / 8;
  int b = C8 < 8 ? C8 : 8;
  while (b > 1 && C8 % b) --b;
  if (b < 1) b = 1;
  DwChunks d;
  d.c8b = b;
  d.nchunk = C8 / b;
  d.R = 256 / b;
  return d;
}
constexpr int kDwTargetBlocks = 2048;  // ~8 blocks per CU across the chunks
// pixel blocks (gridDim.x) of a strip kernel: >= 1 strip per thread row, ~kDwTargetBlocks total
inline int dw_pblocks(long long strips, const DwChunks& d) {
  long long b = (strips + d.R - 1) / d.R;
  long long cap = kDwTargetBlocks / d.nchunk;
  if (cap < 1) cap = 1;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

template <int S>
__global__ __launch_bounds__(256) void dw_fwd3_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  constexpr int P = kDwStrip, NCOL = (P - 1) * S + 3;
  extern __shared__ float sh[];
  const int CBX = dw_chunks(a.C).c8b * 8;  // table stride: the block's channels
  float* s_sc = sh;
  float* s_sf = sh + CBX;
  float* s_a = sh + 2 * CBX;
  float* s_b = sh + 3 * CBX;
  const DwChunks dc = dw_chunks(a.C);
  const int CB = dc.c8b * 8, cb = blockIdx.y * CB;  // this block's channels [cb, cb + CB)
  for (int i = threadIdx.x; i < CB; i += blockDim.x) {
    bn_coeffs(a.pro, cb + i, s_sc[i], s_sf[i]);
    s_a[i] = 0.f;
    s_b[i] = 0.f;
  }
  __syncthreads();
  const int tx = threadIdx.x % dc.c8b, ty = threadIdx.x / dc.c8b;
  const int WS = (a.Wo + P - 1) / P;
  const int strips = a.N * a.Ho * WS;
  float ps[8] = {0}, pq[8] = {0};
  if (ty < dc.R) {
    const int cl = tx * 8, c = cb + cl;
    float wk[9][8], sc[8], sf[8];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c);
      const float4 w1 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c + 4);
      wk[t][0] = w0.x; wk[t][1] = w0.y; wk[t][2] = w0.z; wk[t][3] = w0.w;
      wk[t][4] = w1.x; wk[t][5] = w1.y; wk[t][6] = w1.z; wk[t][7] = w1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = s_sc[cl + j]; sf[j] = s_sf[cl + j]; }
    const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
    float kk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) kk[j] = a.stats_shift ? a.stats_shift[c + j] : 0.f;
    for (int st = blockIdx.x * dc.R + ty; st < strips; st += gridDim.x * dc.R) {
      const int ws = st % WS, t = st / WS, ho = t % a.Ho, n = t / a.Ho;
      const int wo0 = ws * P;
      float acc[P][8];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[p][j] = 0.f;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int h = ho * S - a.PT + r;
        const bool hv = (unsigned)h < (unsigned)a.H;
        uint4 xv[NCOL];
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          const int w = wo0 * S - a.PL + q;
          const bool v = hv && (unsigned)w < (unsigned)a.W;
          const size_t pix = v ? ((size_t)(n * a.H + h) * a.W + w) : 0;
          xv[q] = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c);
        }
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          const int w = wo0 * S - a.PL + q;
          const float m = (hv && (unsigned)w < (unsigned)a.W) ? 1.f : 0.f;
          float u[8];
          unpack8(xv[q], u);
#pragma unroll
          for (int j = 0; j < 8; ++j) u[j] = fminf(fmaxf(fmaf(u[j], sc[j], sf[j]), lo), hi) * m;
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const int s = q - p * S;
            if (s >= 0 && s < 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[p][j] = fmaf(u[j], wk[r * 3 + s][j], acc[p][j]);
            }
          }
        }
      }
      const size_t ob = (size_t)(n * a.Ho + ho) * a.Wo;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        if (wo0 + p >= a.Wo) break;
        const uint4 pk = pack8(acc[p]);
        *reinterpret_cast<uint4*>(a.y + (ob + wo0 + p) * a.ldy + c) = pk;
        float r8[8];
        unpack8(pk, r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dj = r8[j] - kk[j];
          ps[j] += dj;
          pq[j] += dj * dj;
        }
      }
    }
  }
  if (a.stats) {
    chunk_sums(CB, dc.R, tx, ty, ps, pq, sh + 4 * CBX, s_a, s_b);
    __syncthreads();
    float* so = a.stats + (size_t)(blockIdx.x % stat_slots(a.stats_slots)) * 2 * a.stats_ld;
    for (int i = threadIdx.x; i < CB; i += blockDim.x) {
      atomicAdd(&so[cb + i], s_a[i]);
      atomicAdd(&so[a.stats_ld + cb + i], s_b[i]);
    }
  }
}

// backward data, stride 1: dx[h, w] = sum_{r,s} dy[h+PT-r, w+PL-s] * w[r, s]; a strip of P input
// pixels reads P+2 dy columns per tap row.  Stride 2 gathers per pixel (the taps that hit an
// output position depend on parity).  Epilogue: dZ = g * act'(bn(x)), sum dZ, sum dZ*xhat.
// Stride 2 with left pad PL2 (0 or 1, Keras correct_pad): for a strip of P input pixels starting
// at an even w0, dy column (w0 >> 1) - 1 + q feeds pixel p through tap s = p + PL2 + 2 - 2q, so
// which (pixel, column) pairs meet is known at compile time; PL2 < 0 gathers per pixel.
template <int S, int PL2, bool AFF>
__global__ __launch_bounds__(256) void dw_bwd3_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  constexpr bool STRIP = S == 1 || PL2 >= 0;
  constexpr int P = STRIP ? kDwStrip : 1;
  constexpr int NCOL = S == 1 ? P + 2 : (PL2 >= 0 ? (P + PL2 + 2) / 2 + 1 : 3);
  extern __shared__ float sh[];
  const int CBX = dw_chunks(a.C).c8b * 8;  // table stride: the block's channels
  float* s_sc = sh;
  float* s_sf = sh + CBX;
  float* s_mu = sh + 2 * CBX;
  float* s_rs = sh + 3 * CBX;
  float* s_a = sh + 4 * CBX;
  float* s_b = sh + 5 * CBX;
  float* s_fA = sh + 6 * CBX;  // AFF: dy' = A*dy + B*x + C
  float* s_fB = sh + 7 * CBX;
  float* s_fC = sh + 8 * CBX;
  const bool epi = !(a.pro.mode == 0 && a.pro.act == ACT_NONE);
  const DwChunks dc = dw_chunks(a.C);
  const int CB = dc.c8b * 8, cb = blockIdx.y * CB;  // this block's channels [cb, cb + CB)
  for (int i = threadIdx.x; i < CB; i += blockDim.x) {
    const int c = cb + i;
    bn_coeffs(a.pro, c, s_sc[i], s_sf[i]);
    float mean = 0.f, rstd = 1.f;
    if (a.pro.mode) bn_mean_rstd(a.pro, c, mean, rstd);
    s_mu[i] = mean; s_rs[i] = rstd; s_a[i] = 0.f; s_b[i] = 0.f;
  }
  if constexpr (AFF) {
    bwd_aff_table<256>(a.dyaff, cb, CB, a.C, s_fA, s_fB, s_fC);
    bwd_aff_fold<256>(a.dyaff);
  }
  __syncthreads();
  const int tx = threadIdx.x % dc.c8b, ty = threadIdx.x / dc.c8b;
  const int WS = (a.W + P - 1) / P;
  const int strips = a.N * a.H * WS;
  float ps[8] = {0}, px[8] = {0};
  if (ty < dc.R) {
    const int cl = tx * 8, c = cb + cl;
    float wk[9][8], sc[8], sf[8], mu[8], rs[8], fA[8], fB[8], fC[8];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c);
      const float4 w1 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c + 4);
      wk[t][0] = w0.x; wk[t][1] = w0.y; wk[t][2] = w0.z; wk[t][3] = w0.w;
      wk[t][4] = w1.x; wk[t][5] = w1.y; wk[t][6] = w1.z; wk[t][7] = w1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = s_sc[cl + j]; sf[j] = s_sf[cl + j]; mu[j] = s_mu[cl + j]; rs[j] = s_rs[cl + j];
      if constexpr (AFF) { fA[j] = s_fA[cl + j]; fB[j] = s_fB[cl + j]; fC[j] = s_fC[cl + j]; }
    }
    const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
    for (int st = blockIdx.x * dc.R + ty; st < strips; st += gridDim.x * dc.R) {
      const int ws = st % WS, t = st / WS, h = t % a.H, n = t / a.H;
      const int w0 = ws * P;
      float g[P][8];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) g[p][j] = 0.f;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int th = h + a.PT - r;
        int ho;
        bool hv;
        if constexpr (S == 1) {
          ho = th;
          hv = (unsigned)th < (unsigned)a.Ho;
        } else {
          ho = th >> 1;
          hv = th >= 0 && !(th & 1) && ho < a.Ho;
        }
        uint4 dv[NCOL], xv[AFF ? NCOL : 1];
        float m[NCOL];
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          int wo;
          bool v;
          if constexpr (S == 1) {
            wo = w0 + a.PL - 2 + q;  // column q feeds pixel p through tap s = p + 2 - q
            v = hv && (unsigned)wo < (unsigned)a.Wo;
          } else if constexpr (PL2 >= 0) {
            wo = (w0 >> 1) - 1 + q;
            v = hv && (unsigned)wo < (unsigned)a.Wo;
          } else {
            const int tw = w0 + a.PL - q;  // tap s = q
            wo = tw >> 1;
            v = hv && tw >= 0 && !(tw & 1) && wo < a.Wo;
          }
          m[q] = v ? 1.f : 0.f;
          const size_t o = v ? ((size_t)(n * a.Ho + ho) * a.Wo + wo) : 0;
          dv[q] = *reinterpret_cast<const uint4*>(a.dy + o * a.lddy + c);
          if constexpr (AFF) xv[q] = *reinterpret_cast<const uint4*>(a.dyaff.x + o * a.dyaff.ldx + c);
        }
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          float d[8];
          unpack8(dv[q], d);
          if constexpr (AFF) {
            float xd[8];
            unpack8(xv[q], xd);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = fmaf(fA[j], d[j], fmaf(fB[j], xd[j], fC[j]));
          }
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const int s = S == 1 ? p + 2 - q : (PL2 >= 0 ? p + PL2 + 2 - 2 * q : q);
            if (s >= 0 && s < 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) g[p][j] = fmaf(d[j] * m[q], wk[r * 3 + s][j], g[p][j]);
            }
          }
        }
      }
      const size_t ib = (size_t)(n * a.H + h) * a.W;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        if (w0 + p >= a.W) break;
        const size_t i = ib + w0 + p;
        if (epi) {
          float x[8];
          unpack8(*reinterpret_cast<const uint4*>(a.x + i * a.ldx + c), x);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = fmaf(x[j], sc[j], sf[j]);
            g[p][j] = (z > lo && z < hi) ? g[p][j] : 0.f;
          }
          const uint4 pk = pack8(g[p]);
          *reinterpret_cast<uint4*>(a.dx + i * a.lddx + c) = pk;
          float r8[8];
          unpack8(pk, r8);
#pragma unroll
          for (int j = 0; j < 8; ++j) { ps[j] += r8[j]; px[j] += r8[j] * (x[j] - mu[j]) * rs[j]; }
        } else {
          *reinterpret_cast<uint4*>(a.dx + i * a.lddx + c) = pack8(g[p]);
        }
      }
    }
  }
  if (epi) {
    chunk_sums(CB, dc.R, tx, ty, ps, px, sh + 9 * CBX, s_a, s_b);
    __syncthreads();
    const size_t so = (size_t)(blockIdx.x % stat_slots(a.gsum_slots)) * a.gsum_ld;
    for (int i = threadIdx.x; i < CB; i += blockDim.x) {
      if (a.gsum) atomicAdd(&a.gsum[so + cb + i], s_a[i]);
      if (a.gsumx) atomicAdd(&a.gsumx[so + cb + i], s_b[i]);
    }
  }
}


// Stride-1 depthwise 3x3 backward, data AND weight gradients in one pass over the same operands
// (VERDICT r5 item 5a).  A thread's strip of P pixels x 8 channels loads the 3 x (P+2) window of
// dY (the data gradient's gather, as dw_bwd3_kernel) and the 3 x (P+2) window of the raw input x
// (the weight gradient's taps, as dw_wgrad3_part_kernel): 36 loads per strip where the two kernels
// issue 22 + 22, the strip's own dY row and x row are shared, and one launch replaces two.  The
// data gradient's epilogue (act' mask of the pending BN + activation, the BN-backward sums) is
// dw_bwd3_kernel's; the weight-gradient partials are reduced per block into ws[block][9][C] like
// dw_wgrad3_part_kernel's and summed by dwconv_wgrad_sum (a separate, side-lane launch).
__global__ __launch_bounds__(256) void dw_bwd3_fused_kernel(DwArgs a, GroupArg ga) {
  gshift(a, goff(ga));
  constexpr int P = kDwStrip, NCOL = P + 2;
  extern __shared__ float sh[];
  const DwChunks dc = dw_chunks(a.C);
  const int CB = dc.c8b * 8, cb = blockIdx.y * CB;
  float* s_sc = sh;
  float* s_sf = sh + CB;
  float* s_mu = sh + 2 * CB;
  float* s_rs = sh + 3 * CB;
  float* s_a = sh + 4 * CB;
  float* s_b = sh + 5 * CB;
  float* s_tmp = sh + 6 * CB;  // chunk_sums scratch (2 x 256 x 8) / weight-gradient rows (256 x 24)
  const bool epi = !(a.pro.mode == 0 && a.pro.act == ACT_NONE);
  for (int i = threadIdx.x; i < CB; i += blockDim.x) {
    const int c = cb + i;
    bn_coeffs(a.pro, c, s_sc[i], s_sf[i]);
    float mean = 0.f, rstd = 1.f;
    if (a.pro.mode) bn_mean_rstd(a.pro, c, mean, rstd);
    s_mu[i] = mean; s_rs[i] = rstd; s_a[i] = 0.f; s_b[i] = 0.f;
  }
  __syncthreads();
  const int tx = threadIdx.x % dc.c8b, ty = threadIdx.x / dc.c8b;
  const int WS = (a.W + P - 1) / P;
  const int strips = a.N * a.H * WS;
  float ps[8] = {0}, px[8] = {0};
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  if (ty < dc.R) {
    const int cl = tx * 8, c = cb + cl;
    float wk[9][8], sc[8], sf[8], mu[8], rs[8];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w0 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c);
      const float4 w1 = *reinterpret_cast<const float4*>(a.w + (size_t)t * a.C + c + 4);
      wk[t][0] = w0.x; wk[t][1] = w0.y; wk[t][2] = w0.z; wk[t][3] = w0.w;
      wk[t][4] = w1.x; wk[t][5] = w1.y; wk[t][6] = w1.z; wk[t][7] = w1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = s_sc[cl + j]; sf[j] = s_sf[cl + j]; mu[j] = s_mu[cl + j]; rs[j] = s_rs[cl + j]; }
    const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
    for (int st = blockIdx.x * dc.R + ty; st < strips; st += gridDim.x * dc.R) {
      const int ws = st % WS, t = st / WS, h = t % a.H, n = t / a.H;
      const int w0 = ws * P;
      float g[P][8], dcen[P][8], xcen[P][8];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) { g[p][j] = 0.f; dcen[p][j] = 0.f; xcen[p][j] = 0.f; }
      // the centre rows first: the strip's own dY (weight gradient) and x (data-gradient mask)
      constexpr int RORD[3] = {1, 0, 2};
#pragma unroll
      for (int ri = 0; ri < 3; ++ri) {
        const int r = RORD[ri];
        const int ho = h + a.PT - r;                  // dY row feeding this strip through tap row r
        const bool hv = (unsigned)ho < (unsigned)a.Ho;
        const int hx = h - a.PT + r;                  // x row under tap row r of the strip's outputs
        const bool xv_ok = (unsigned)hx < (unsigned)a.H;
        uint4 dv[NCOL], xv[NCOL];
        float md[NCOL], mx[NCOL];
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          const int wo = w0 + a.PL - 2 + q;  // column q feeds pixel p through tap s = p + 2 - q
          const bool v = hv && (unsigned)wo < (unsigned)a.Wo;
          md[q] = v ? 1.f : 0.f;
          const size_t o = v ? ((size_t)(n * a.Ho + ho) * a.Wo + wo) : 0;
          dv[q] = *reinterpret_cast<const uint4*>(a.dy + o * a.lddy + c);
          const int wx = w0 - a.PL + q;      // input column q: tap s = q - p of output pixel p
          const bool vx = xv_ok && (unsigned)wx < (unsigned)a.W;
          mx[q] = vx ? 1.f : 0.f;
          const size_t pix = vx ? ((size_t)(n * a.H + hx) * a.W + wx) : 0;
          xv[q] = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c);
        }
        if (r == 1) {  // stride 1, PT = PL = 1: dY column q = p + 1 is output pixel p; x column q = p + 1 is pixel p
#pragma unroll
          for (int p = 0; p < P; ++p) {
            float d[8], xx[8];
            unpack8(dv[p + 1], d);
            unpack8(xv[p + 1], xx);
            const float vo = (w0 + p < a.W) ? md[p + 1] : 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) { dcen[p][j] = d[j] * vo; xcen[p][j] = xx[j]; }
          }
        }
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          float d[8], u[8];
          unpack8(dv[q], d);
          unpack8(xv[q], u);
#pragma unroll
          for (int j = 0; j < 8; ++j) u[j] = clampf(fmaf(u[j], sc[j], sf[j]), lo, hi) * mx[q];
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const int sd = p + 2 - q;  // data gradient: dY column q through tap (r, sd) into pixel p
            if (sd >= 0 && sd < 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) g[p][j] = fmaf(d[j] * md[q], wk[r * 3 + sd][j], g[p][j]);
            }
            const int sw = q - p;      // weight gradient: x column q under tap (r, sw) of pixel p
            if (sw >= 0 && sw < 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[r * 3 + sw][j] = fmaf(u[j], dcen[p][j], acc[r * 3 + sw][j]);
            }
          }
        }
      }
      const size_t ib = (size_t)(n * a.H + h) * a.W;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        if (w0 + p >= a.W) break;
        const size_t i = ib + w0 + p;
        if (epi) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = fmaf(xcen[p][j], sc[j], sf[j]);
            g[p][j] = (z > lo && z < hi) ? g[p][j] : 0.f;
          }
          const uint4 pk = pack8(g[p]);
          *reinterpret_cast<uint4*>(a.dx + i * a.lddx + c) = pk;
          float r8[8];
          unpack8(pk, r8);
#pragma unroll
          for (int j = 0; j < 8; ++j) { ps[j] += r8[j]; px[j] += r8[j] * (xcen[p][j] - mu[j]) * rs[j]; }
        } else {
          *reinterpret_cast<uint4*>(a.dx + i * a.lddx + c) = pack8(g[p]);
        }
      }
    }
  }
  if (epi) {
    chunk_sums(CB, dc.R, tx, ty, ps, px, s_tmp, s_a, s_b);
    __syncthreads();
    const size_t so = (size_t)(blockIdx.x % stat_slots(a.gsum_slots)) * a.gsum_ld;
    for (int i = threadIdx.x; i < CB; i += blockDim.x) {
      if (a.gsum) atomicAdd(&a.gsum[so + cb + i], s_a[i]);
      if (a.gsumx) atomicAdd(&a.gsumx[so + cb + i], s_b[i]);
    }
  }
  // weight-gradient partials of this block: one tap row per round through LDS, summed in order
  float* out = a.ws + (size_t)blockIdx.x * 9 * a.C + cb;
  const int C8 = dc.c8b;
  const bool act = ty < dc.R;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    __syncthreads();
    float4* d = reinterpret_cast<float4*>(s_tmp + threadIdx.x * 24);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const float* v = acc[r * 3 + s];
      d[2 * s] = act ? make_float4(v[0], v[1], v[2], v[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
      d[2 * s + 1] = act ? make_float4(v[4], v[5], v[6], v[7]) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < 3 * CB; o += blockDim.x) {
      const int s = o / CB, c = o - s * CB, cx = c >> 3, j = c & 7;
      float sum = 0.f;
      for (int y = 0; y < dc.R; ++y) sum += s_tmp[(y * C8 + cx) * 24 + s * 8 + j];
      out[(r * 3 + s) * a.C + c] = sum;
    }
  }
}

hipError_t dwconv_fwd(const DwArgs& a, hipStream_t st) {
  if (a.KH == 3 && a.KW == 3 && (a.S == 1 || a.S == 2) && a.C % 8 == 0 && a.C <= 2048) {
    const long long strips = (long long)a.N * a.Ho * ((a.Wo + kDwStrip - 1) / kDwStrip);
    const DwChunks dc = dw_chunks(a.C);
    const dim3 g(dw_pblocks(strips, dc), dc.nchunk);
    const size_t shm = (4 * dc.c8b * 8 + 2 * 256 * 8) * 4;  // tables + chunk_sums scratch
    if (a.S == 1)
      hipLaunchKernelGGL(dw_fwd3_kernel<1>, ggrid(g), dim3(256), shm, st, a, garg());
    else
      hipLaunchKernelGGL(dw_fwd3_kernel<2>, ggrid(g), dim3(256), shm, st, a, garg());
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dw_fwd_kernel, ggrid(dim3(nblocks((long long)a.N * a.Ho * a.Wo, a.C, 4))), dim3(256),
                     4 * a.C * 4, st, a, garg());
  return hipGetLastError();
}

hipError_t dwconv_bwd_data(const DwArgs& a, hipStream_t st) {
  const bool aff = a.dyaff.mode != 0;
  if (a.KH == 3 && a.KW == 3 && (a.S == 1 || a.S == 2) && a.C % 8 == 0 && a.C <= 2048) {
    const DwChunks dc = dw_chunks(a.C);
    const size_t shm = (9 * dc.c8b * 8 + 2 * 256 * 8) * 4;  // tables + chunk_sums scratch
    const long long strips4 = (long long)a.N * a.H * ((a.W + kDwStrip - 1) / kDwStrip);
    const dim3 g4(dw_pblocks(strips4, dc), dc.nchunk), g1(dw_pblocks((long long)a.N * a.H * a.W, dc), dc.nchunk);
#define IDC_DWB(S_, PL_, G_)                                                                      \
  if (aff) hipLaunchKernelGGL((dw_bwd3_kernel<S_, PL_, true>), ggrid(G_), dim3(256), shm, st, a, garg()); \
  else hipLaunchKernelGGL((dw_bwd3_kernel<S_, PL_, false>), ggrid(G_), dim3(256), shm, st, a, garg());
    if (a.S == 1) {
      IDC_DWB(1, -1, g4)
    } else if (a.PL == 0) {
      IDC_DWB(2, 0, g4)
    } else if (a.PL == 1) {
      IDC_DWB(2, 1, g4)
    } else {
      IDC_DWB(2, -1, g1)
    }
#undef IDC_DWB
    return hipGetLastError();
  }
  if (aff) return hipErrorInvalidValue;  // the backward affine prologue is 3x3-only
  hipLaunchKernelGGL(dw_bwd_data_kernel, ggrid(dim3(nblocks((long long)a.N * a.H * a.W, a.C, 4))), dim3(256),
                     6 * a.C * 4, st, a, garg());
  return hipGetLastError();
}

namespace {
inline bool dw_fused_ok(const DwArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.S == 1 && a.PT == 1 && a.PL == 1 && a.H == a.Ho && a.W == a.Wo &&
         a.C % 8 == 0 && a.C <= 2048 && a.dyaff.mode == 0 && a.ws != nullptr && a.dw != nullptr;
}
inline int dw_fused_blocks(const DwArgs& a) {
  const long long strips = (long long)a.N * a.H * ((a.W + kDwStrip - 1) / kDwStrip);
  return dw_pblocks(strips, dw_chunks(a.C));
}
}  // namespace

bool dwconv_bwd_fused_ok(const DwArgs& a) { return dw_fused_ok(a); }

hipError_t dwconv_bwd_fused(const DwArgs& a, hipStream_t st) {
  if (!dw_fused_ok(a)) return hipErrorInvalidValue;
  const DwChunks dc = dw_chunks(a.C);
  const size_t shm = (6 * dc.c8b * 8 + (2 * 256 * 8 > 256 * 24 ? 2 * 256 * 8 : 256 * 24)) * 4;
  const dim3 g(dw_fused_blocks(a), dc.nchunk);
  hipLaunchKernelGGL(dw_bwd3_fused_kernel, ggrid(g), dim3(256), shm, st, a, garg());
  return hipGetLastError();
}

// ---- two-stage weight gradient ---------------------------------------------------------
// Stage 1: a block owns a contiguous range of output pixels and ALL channels (one 16-B channel
// chunk per thread, R pixel rows in flight per block, two rows per iteration for ILP); its
// 9 x C partial sums are reduced in LDS and stored (plain stores) into ws[block][tap][C].
// Stage 2: one thread per (tap, c) sums the column over blocks.  No global atomics: the
// single-stage kernel's few long-running blocks (and the atomic alternative's contention on
// 9*C addresses) made this the MobileNetV2 step's longest kernel.
namespace {
constexpr int kDwRowsPerThread = 16;
inline int dw_wgrad_blocks(long long M, int C) {
  int C8 = C / 8, R = 256 / C8;
  if (R < 1) R = 1;
  long long b = (M + (long long)R * kDwRowsPerThread - 1) / ((long long)R * kDwRowsPerThread);
  if (b > 1024) b = 1024;
  return b < 1 ? 1 : (int)b;
}
}  // namespace

long long dwconv_wgrad_ws_floats(long long M, int C, int taps) {
  // the larger of the general two-stage grid and the strip kernel's pixel blocks (strips <= M)
  const long long a = dw_wgrad_blocks(M, C), b = dw_pblocks(M, dw_chunks(C));
  return (a > b ? a : b) * taps * C;
}

__global__ __launch_bounds__(256) void dw_wgrad_part_kernel(DwArgs a, int rows_per_block, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sf = sh + a.C;
  float* s_acc = sh + 2 * a.C;  // [KH*KW][C]
  const int T = a.KH * a.KW;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) bn_coeffs(a.pro, c, s_sc[c], s_sf[c]);
  for (int k = threadIdx.x; k < T * a.C; k += blockDim.x) s_acc[k] = 0.f;
  __syncthreads();
  Map8 mp(a.C);
  const int Mo = a.N * a.Ho * a.Wo;
  const int o0 = blockIdx.x * rows_per_block;
  const int o1 = min(Mo, o0 + rows_per_block);
  const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
  if (mp.ty < mp.R) {
    const int c = mp.tx * 8;
    float sc[8], sf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = s_sc[c + j]; sf[j] = s_sf[c + j]; }
    float acc[9][8];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
    for (int o = o0 + mp.ty; o < o1; o += mp.R) {
      int wo = o % a.Wo, t = o / a.Wo, ho = t % a.Ho, n = t / a.Ho;
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(a.dy + (size_t)o * a.lddy + c), d);
      uint4 xv[9];
      bool ok[9];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          int h = ho * a.S - a.PT + r, w = wo * a.S - a.PL + s;
          bool v = r < a.KH && s < a.KW && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
          ok[r * 3 + s] = v;
          h = v ? h : 0;
          w = v ? w : 0;  // clamped address: the load stays unconditional
          xv[r * 3 + s] = *reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.ldx + c);
        }
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float v[8];
        unpack8(xv[k], v);
        const float m = ok[k] ? 1.f : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float u = fminf(fmaxf(fmaf(v[j], sc[j], sf[j]), lo), hi);
          acc[k][j] = fmaf(u * m, d[j], acc[k][j]);
        }
      }
    }
    for (int r = 0; r < a.KH; ++r)
      for (int s = 0; s < a.KW; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(&s_acc[(r * a.KW + s) * a.C + c + j], acc[r * 3 + s][j]);
  }
  __syncthreads();
  float* out = a.ws + (size_t)blockIdx.x * T * a.C;
  for (int k = threadIdx.x; k < T * a.C; k += blockDim.x) out[k] = s_acc[k];
}

// 3x3 weight-gradient partials over strips of P output pixels: the strip's 3 x ((P-1)*S+3) input
// vectors are loaded once and multiplied into every tap they meet (stride 1: 18 loads and 4 dy
// loads per 4 outputs instead of 40); block b owns strips [b*spb, (b+1)*spb).
template <int S, bool AFF>
__global__ __launch_bounds__(256) void dw_wgrad3_part_kernel(DwArgs a, int spb, GroupArg ga) {
  gshift(a, goff(ga));
  constexpr int P = kDwStrip, NCOL = (P - 1) * S + 3;
  extern __shared__ float sh[];
  const DwChunks dc = dw_chunks(a.C);
  const int CB = dc.c8b * 8, cb = blockIdx.y * CB;  // this block's channels [cb, cb + CB)
  float* s_sc = sh;
  float* s_sf = sh + CB;
  float* s_fA = sh + 2 * CB;   // AFF: dy' = A*dy + B*x + C
  float* s_fB = sh + 3 * CB;
  float* s_fC = sh + 4 * CB;
  float* s_red = sh + 5 * CB;  // [256 threads][3 taps][8]: one tap row per reduction round
  for (int i = threadIdx.x; i < CB; i += blockDim.x) bn_coeffs(a.pro, cb + i, s_sc[i], s_sf[i]);
  if constexpr (AFF) bwd_aff_table<256>(a.dyaff, cb, CB, a.C, s_fA, s_fB, s_fC);
  __syncthreads();
  const int tx = threadIdx.x % dc.c8b, ty = threadIdx.x / dc.c8b;
  const int WS = (a.Wo + P - 1) / P;
  const int strips = a.N * a.Ho * WS;
  const int s0 = blockIdx.x * spb, s1 = min(strips, s0 + spb);
  const float lo = act_lo(a.pro.act), hi = act_hi(a.pro.act);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  if (ty < dc.R) {
    const int cl = tx * 8, c = cb + cl;
    float sc[8], sf[8], fA[8], fB[8], fC[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = s_sc[cl + j]; sf[j] = s_sf[cl + j];
      if constexpr (AFF) { fA[j] = s_fA[cl + j]; fB[j] = s_fB[cl + j]; fC[j] = s_fC[cl + j]; }
    }
    for (int st = s0 + ty; st < s1; st += dc.R) {
      const int ws = st % WS, t = st / WS, ho = t % a.Ho, n = t / a.Ho;
      const int wo0 = ws * P;
      float d[P][8];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const bool v = wo0 + p < a.Wo;
        const size_t o = v ? ((size_t)(n * a.Ho + ho) * a.Wo + wo0 + p) : 0;
        unpack8(*reinterpret_cast<const uint4*>(a.dy + o * a.lddy + c), d[p]);
        if constexpr (AFF) {
          float xd[8];
          unpack8(*reinterpret_cast<const uint4*>(a.dyaff.x + o * a.dyaff.ldx + c), xd);
#pragma unroll
          for (int j = 0; j < 8; ++j) d[p][j] = fmaf(fA[j], d[p][j], fmaf(fB[j], xd[j], fC[j]));
        }
        if (!v) {
#pragma unroll
          for (int j = 0; j < 8; ++j) d[p][j] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int h = ho * S - a.PT + r;
        const bool hv = (unsigned)h < (unsigned)a.H;
        uint4 xv[NCOL];
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          const int w = wo0 * S - a.PL + q;
          const bool v = hv && (unsigned)w < (unsigned)a.W;
          const size_t pix = v ? ((size_t)(n * a.H + h) * a.W + w) : 0;
          xv[q] = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c);
        }
#pragma unroll
        for (int q = 0; q < NCOL; ++q) {
          const int w = wo0 * S - a.PL + q;
          const float m = (hv && (unsigned)w < (unsigned)a.W) ? 1.f : 0.f;
          float u[8];
          unpack8(xv[q], u);
#pragma unroll
          for (int j = 0; j < 8; ++j) u[j] = fminf(fmaxf(fmaf(u[j], sc[j], sf[j]), lo), hi) * m;
#pragma unroll
          for (int p = 0; p < P; ++p) {
            const int s = q - p * S;
            if (s >= 0 && s < 3) {
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[r * 3 + s][j] = fmaf(u[j], d[p][j], acc[r * 3 + s][j]);
            }
          }
        }
      }
    }
  }
  // block reduction over the R thread rows of each chunk, one tap row (3 taps) per round:
  // every thread's 24 partials to LDS, then each (tap, channel) output sums its R entries in
  // order (the per-address LDS atomics this replaces serialised R-way on small C)
  float* out = a.ws + (size_t)blockIdx.x * 9 * a.C + cb;
  const int C8 = dc.c8b;
  const bool act = ty < dc.R;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    if (r) __syncthreads();
    float4* d = reinterpret_cast<float4*>(s_red + threadIdx.x * 24);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const float* v = acc[r * 3 + s];
      d[2 * s] = act ? make_float4(v[0], v[1], v[2], v[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
      d[2 * s + 1] = act ? make_float4(v[4], v[5], v[6], v[7]) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < 3 * CB; o += blockDim.x) {
      const int s = o / CB, c = o - s * CB, cx = c >> 3, j = c & 7;
      float sum = 0.f;
      for (int y = 0; y < dc.R; ++y) sum += s_red[(y * C8 + cx) * 24 + s * 8 + j];
      out[(r * 3 + s) * a.C + c] = sum;
    }
  }
}

// column sums of the per-block partials: blockIdx.y splits the blocks so the sum is spread over
// many workgroups (a single pass per column was a few long latency chains on a handful of CUs)
__global__ __launch_bounds__(256) void dw_wgrad_sum_kernel(const float* __restrict__ ws, int nblk, int n,
                                                           float* __restrict__ dw, GroupArg ga) {
  const long long go = goff(ga);
  ws = gsh(ws, go);
  dw = gsh(dw, go);
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int per = (nblk + gridDim.y - 1) / gridDim.y;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = b0;
  for (; b + 4 <= b1; b += 4) {
    s0 += ws[(size_t)b * n + k];
    s1 += ws[(size_t)(b + 1) * n + k];
    s2 += ws[(size_t)(b + 2) * n + k];
    s3 += ws[(size_t)(b + 3) * n + k];
  }
  for (; b < b1; ++b) s0 += ws[(size_t)b * n + k];
  const float v = (s0 + s1) + (s2 + s3);
  if (gridDim.y == 1) dw[k] += v;
  else atomicAdd(&dw[k], v);
}

hipError_t dwconv_wgrad(const DwArgs& a, hipStream_t st) {
  if (a.KH > 3 || a.KW > 3) return hipErrorInvalidValue;
  const long long Mo = (long long)a.N * a.Ho * a.Wo;
  const int T = a.KH * a.KW;
  if (a.ws) {
    int nblk = dw_wgrad_blocks(Mo, a.C);
    const bool aff = a.dyaff.mode != 0;
    if (a.KH == 3 && a.KW == 3 && (a.S == 1 || a.S == 2) && a.C % 8 == 0) {
      const long long strips = (long long)a.N * a.Ho * ((a.Wo + kDwStrip - 1) / kDwStrip);
      const DwChunks dc = dw_chunks(a.C);
      nblk = dw_pblocks(strips, dc);
      const int spb = (int)((strips + nblk - 1) / nblk);
      nblk = (int)((strips + spb - 1) / spb);
      const size_t shm = (5 * dc.c8b * 8 + 256 * 24) * 4;
      const dim3 g(nblk, dc.nchunk);
      if (a.S == 1) {
        if (aff) hipLaunchKernelGGL((dw_wgrad3_part_kernel<1, true>), ggrid(g), dim3(256), shm, st, a, spb, garg());
        else hipLaunchKernelGGL((dw_wgrad3_part_kernel<1, false>), ggrid(g), dim3(256), shm, st, a, spb, garg());
      } else {
        if (aff) hipLaunchKernelGGL((dw_wgrad3_part_kernel<2, true>), ggrid(g), dim3(256), shm, st, a, spb, garg());
        else hipLaunchKernelGGL((dw_wgrad3_part_kernel<2, false>), ggrid(g), dim3(256), shm, st, a, spb, garg());
      }
    } else if (aff) {
      return hipErrorInvalidValue;
    } else {
      const int rpb = (int)((Mo + nblk - 1) / nblk);
      hipLaunchKernelGGL(dw_wgrad_part_kernel, ggrid(dim3(nblk)), dim3(256), (2 + T) * a.C * 4, st, a, rpb, garg());
    }
    const int n = T * a.C;
    const int cols = (n + 255) / 256;
    int split = (nblk + 31) / 32;  // ~32 partials per thread, enough workgroups to fill the chip
    if (split > 64) split = 64;
    if (split < 1) split = 1;
    hipLaunchKernelGGL(dw_wgrad_sum_kernel, ggrid(dim3(cols, split)), dim3(256), 0, st, a.ws, nblk, n, a.dw, garg());
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dw_wgrad_kernel, ggrid(dim3(nblocks(Mo, a.C, 32))), dim3(256), (2 + T) * a.C * 4, st, a, garg());
  return hipGetLastError();
}

// column sums of dw_bwd3_fused_kernel's per-block weight-gradient partials (side lane)
hipError_t dwconv_wgrad_sum(const DwArgs& a, hipStream_t st) {
  if (!dw_fused_ok(a)) return hipErrorInvalidValue;
  const int nblk = dw_fused_blocks(a);
  const int n = 9 * a.C;
  const int cols = (n + 255) / 256;
  int split = (nblk + 31) / 32;
  if (split > 64) split = 64;
  if (split < 1) split = 1;
  hipLaunchKernelGGL(dw_wgrad_sum_kernel, ggrid(dim3(cols, split)), dim3(256), 0, st, a.ws, nblk, n, a.dw, garg());
  return hipGetLastError();
}

}  // namespace idc
