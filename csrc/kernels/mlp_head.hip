// Fused tiny-CNN head (secure_fed_model.py:90-95): dropout + Dense + ReLU + dropout + Dense + loss,
// forward and backward, one 256-thread workgroup per sample (the secure-FL batch is 32 x 128
// features: the whole head is a few thousand FMAs, so the point is ONE launch instead of eight).
#include "mlp_head.h"

namespace idc {

namespace {
__device__ __forceinline__ uint32_t philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0 = __umulhi(M0, c0), l0 = M0 * c0;
    uint32_t h1 = __umulhi(M1, c2), l1 = M1 * c2;
    uint32_t n0 = h1 ^ c1 ^ k0, n1 = l1, n2 = h0 ^ c3 ^ k1, n3 = l0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0;
    k1 += W1;
  }
  return c0;
}

// keep factor of element `i` of layer `layer` for sample n: 0 (dropped) or 1/(1-p)
__device__ __forceinline__ float keep(const Mlp2Args& a, int layer, int n, int i, float p, unsigned int step) {
  if (!a.training || p <= 0.f) return 1.f;
  uint32_t r = philox_w0((uint32_t)i, (uint32_t)n, (uint32_t)layer, step, (uint32_t)a.seed,
                         (uint32_t)(a.seed >> 32));
  float u = (r >> 8) * (1.f / 16777216.f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}
}  // namespace

__global__ __launch_bounds__(256) void mlp2_fwd_kernel(Mlp2Args a, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_x = sh;               // [D0] dropped input
  float* s_h = s_x + a.D0;       // [D1] dropped hidden
  float* s_red = s_h + a.D1;     // [4]
  const int n = blockIdx.x;
  const unsigned int step = a.step ? *a.step : 0u;
  for (int i = threadIdx.x; i < a.D0; i += blockDim.x)
    s_x[i] = bf2f(a.x[(size_t)n * a.D0 + i]) * keep(a, 0, n, i, a.p0, step);
  __syncthreads();
  for (int j = threadIdx.x; j < a.D1; j += blockDim.x) {
    float acc = a.b1 ? a.b1[j] : 0.f;
    for (int i = 0; i < a.D0; ++i) acc = fmaf(s_x[i], a.w1[(size_t)i * a.D1 + j], acc);
    acc = fmaxf(acc, 0.f);
    a.h1[(size_t)n * a.D1 + j] = acc;
    s_h[j] = acc * keep(a, 1, n, j, a.p1, step);
  }
  __syncthreads();
  // logits + loss (U small: one block-wide dot per output)
  float lsum = 0.f, zmax = -INFINITY;
  for (int u = 0; u < a.U; ++u) {
    float part = 0.f;
    for (int j = threadIdx.x; j < a.D1; j += blockDim.x) part += s_h[j] * a.w2[(size_t)j * a.U + u];
    float z = block_sum(part, s_red) + (a.b2 ? a.b2[u] : 0.f);
    if (threadIdx.x == 0) a.logits[(size_t)n * a.U + u] = z;
    zmax = fmaxf(zmax, z);
  }
  if (threadIdx.x != 0) return;
  const float* z = a.logits + (size_t)n * a.U;
  if (a.U == 1) {
    float y = a.labels[n], x = z[0];
    float l = fmaxf(x, 0.f) - x * y + log1pf(expf(-fabsf(x)));
    lsum = l;
    if (a.dlogits) a.dlogits[n] = (1.f / (1.f + expf(-x)) - y) * a.dl_scale;
  } else {
    float se = 0.f;
    for (int u = 0; u < a.U; ++u) se += expf(z[u] - zmax);
    float lse = zmax + logf(se);
    for (int u = 0; u < a.U; ++u) {
      float y = a.labels[(size_t)n * a.U + u];
      lsum += y * (lse - z[u]);
      if (a.dlogits) a.dlogits[(size_t)n * a.U + u] = (expf(z[u] - lse) - y) * a.dl_scale;
    }
  }
  atomicAdd(a.loss, lsum * a.loss_scale);
}

__global__ __launch_bounds__(256) void mlp2_bwd_kernel(Mlp2Args a, GroupArg ga) {
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_x = sh;               // [D0] dropped input (recomputed)
  float* s_dh = s_x + a.D0;      // [D1] gradient at the hidden pre-activation
  float* s_hd = s_dh + a.D1;     // [D1] dropped hidden
  const int n = blockIdx.x;
  const unsigned int step = a.step ? *a.step : 0u;
  for (int i = threadIdx.x; i < a.D0; i += blockDim.x)
    s_x[i] = bf2f(a.x[(size_t)n * a.D0 + i]) * keep(a, 0, n, i, a.p0, step);
  for (int j = threadIdx.x; j < a.D1; j += blockDim.x) {
    float h = a.h1[(size_t)n * a.D1 + j];
    float k1 = keep(a, 1, n, j, a.p1, step);
    s_hd[j] = h * k1;
    float g = 0.f;
    for (int u = 0; u < a.U; ++u) g += a.dlogits[(size_t)n * a.U + u] * a.w2[(size_t)j * a.U + u];
    s_dh[j] = h > 0.f ? g * k1 : 0.f;
  }
  __syncthreads();
  // dense 2: dW2[j][u] += hd[j] * dl[u], db2[u] += dl[u]
  for (int t = threadIdx.x; t < a.D1 * a.U; t += blockDim.x) {
    int j = t / a.U, u = t - j * a.U;
    atomicAdd(&a.dw2[t], s_hd[j] * a.dlogits[(size_t)n * a.U + u]);
  }
  for (int u = threadIdx.x; u < a.U; u += blockDim.x) atomicAdd(&a.db2[u], a.dlogits[(size_t)n * a.U + u]);
  // dense 1: dW1[i][j] += x[i] * dh[j], db1[j] += dh[j]
  for (int t = threadIdx.x; t < a.D0 * a.D1; t += blockDim.x) {
    int i = t / a.D1, j = t - i * a.D1;
    atomicAdd(&a.dw1[t], s_x[i] * s_dh[j]);
  }
  for (int j = threadIdx.x; j < a.D1; j += blockDim.x) atomicAdd(&a.db1[j], s_dh[j]);
  if (a.dx) {
    for (int i = threadIdx.x; i < a.D0; i += blockDim.x) {
      float g = 0.f;
      for (int j = 0; j < a.D1; ++j) g = fmaf(s_dh[j], a.w1[(size_t)i * a.D1 + j], g);
      a.dx[(size_t)n * a.D0 + i] = g * keep(a, 0, n, i, a.p0, step);
    }
  }
}

__global__ void mlp2_step_kernel(unsigned int* step, GroupArg ga) { gsh(step, goff(ga))[0] += 1u; }

hipError_t mlp2_fwd(const Mlp2Args& a, hipStream_t st) {
  if (a.N == 0) return hipSuccess;
  hipLaunchKernelGGL(mlp2_fwd_kernel, ggrid(a.N), dim3(256), (a.D0 + a.D1 + 4) * 4, st, a, garg());
  return hipGetLastError();
}

hipError_t mlp2_bwd(const Mlp2Args& a, hipStream_t st) {
  if (a.N == 0) return hipSuccess;
  hipLaunchKernelGGL(mlp2_bwd_kernel, ggrid(a.N), dim3(256), (a.D0 + 2 * a.D1) * 4, st, a, garg());
  return hipGetLastError();
}

hipError_t mlp2_step(unsigned int* step, hipStream_t st) {
  hipLaunchKernelGGL(mlp2_step_kernel, ggrid(1), dim3(1), 0, st, step, garg());
  return hipGetLastError();
}

}  // namespace idc
