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

__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
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
        for (int j = 0; j < 8; ++j) { ps[j] += acc[j]; pq[j] += acc[j] * acc[j]; }
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

__global__ __launch_bounds__(256) void dw_bwd_data_kernel(DwArgs a) {
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

__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwArgs a) {
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

hipError_t dwconv_fwd(const DwArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(nblocks((long long)a.N * a.Ho * a.Wo, a.C, 4)), dim3(256), 4 * a.C * 4,
                     st, a);
  return hipGetLastError();
}

hipError_t dwconv_bwd_data(const DwArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(dw_bwd_data_kernel, dim3(nblocks((long long)a.N * a.H * a.W, a.C, 4)), dim3(256),
                     6 * a.C * 4, st, a);
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
constexpr int kDwRowsPerThread = 4;
inline int dw_wgrad_blocks(long long M, int C) {
  int C8 = C / 8, R = 256 / C8;
  if (R < 1) R = 1;
  long long b = (M + (long long)R * kDwRowsPerThread - 1) / ((long long)R * kDwRowsPerThread);
  if (b > 2048) b = 2048;
  return b < 1 ? 1 : (int)b;
}
}  // namespace

long long dwconv_wgrad_ws_floats(long long M, int C, int taps) {
  return (long long)dw_wgrad_blocks(M, C) * taps * C;
}

__global__ __launch_bounds__(256) void dw_wgrad_part_kernel(DwArgs a, int rows_per_block) {
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

__global__ __launch_bounds__(256) void dw_wgrad_sum_kernel(const float* __restrict__ ws, int nblk, int n,
                                                           float* __restrict__ dw) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = 0;
  for (; b + 4 <= nblk; b += 4) {
    s0 += ws[(size_t)b * n + k];
    s1 += ws[(size_t)(b + 1) * n + k];
    s2 += ws[(size_t)(b + 2) * n + k];
    s3 += ws[(size_t)(b + 3) * n + k];
  }
  for (; b < nblk; ++b) s0 += ws[(size_t)b * n + k];
  dw[k] += (s0 + s1) + (s2 + s3);
}

hipError_t dwconv_wgrad(const DwArgs& a, hipStream_t st) {
  if (a.KH > 3 || a.KW > 3) return hipErrorInvalidValue;
  const long long Mo = (long long)a.N * a.Ho * a.Wo;
  const int T = a.KH * a.KW;
  if (a.ws) {
    const int nblk = dw_wgrad_blocks(Mo, a.C);
    const int rpb = (int)((Mo + nblk - 1) / nblk);
    hipLaunchKernelGGL(dw_wgrad_part_kernel, dim3(nblk), dim3(256), (2 + T) * a.C * 4, st, a, rpb);
    const int n = T * a.C;
    hipLaunchKernelGGL(dw_wgrad_sum_kernel, dim3((n + 255) / 256), dim3(256), 0, st, a.ws, nblk, n, a.dw);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dw_wgrad_kernel, dim3(nblocks(Mo, a.C, 32)), dim3(256), (2 + T) * a.C * 4, st, a);
  return hipGetLastError();
}

}  // namespace idc
