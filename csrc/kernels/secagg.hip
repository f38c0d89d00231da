// Secure aggregation: fixed-point quantisation + pairwise Philox masks, dequantisation.
//
// Replaces the reference's per-element Python Paillier encryption (secure_fed_model.py:109-129,
// 3072-bit modexp per weight on the CPU) with one bandwidth-bound kernel: each element gets
// K-1 counter-based Philox4x32-10 masks keyed by the unordered client pair and the round, added
// with opposite signs by the two members of the pair, so the uint32 ring sum over all K clients
// equals the plain fixed-point sum bit-exactly.
#include "secagg.h"

namespace idc {

__device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }

// Philox4x32-10, returns the first word
__device__ __forceinline__ uint32_t philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                           uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0 = mulhi(M0, c0), l0 = M0 * c0;
    uint32_t h1 = mulhi(M1, c2), l1 = M1 * c2;
    uint32_t n0 = h1 ^ c1 ^ k0, n1 = l1, n2 = h0 ^ c3 ^ k1, n3 = l0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0;
    k1 += W1;
  }
  return c0;
}

__global__ void secagg_mask_kernel(const float* __restrict__ x, uint32_t* __restrict__ out, long long n,
                                   float scale, float clip, int K, int rank, unsigned long long seed,
                                   unsigned long long rnd, unsigned long long alive) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float v = x[i] * scale;
    v = fminf(fmaxf(v, -clip), clip);
    int32_t q = (int32_t)rintf(v);
    uint32_t acc = (uint32_t)q;
    for (int j = 0; j < K; ++j) {
      if (j == rank || !((alive >> j) & 1ull)) continue;  // dropped clients: re-keyed round
      int lo = j < rank ? j : rank, hi = j < rank ? rank : j;
      uint32_t k0 = (uint32_t)seed ^ (uint32_t)(lo * 0x9E3779B1u);
      uint32_t k1 = (uint32_t)(seed >> 32) ^ (uint32_t)(hi * 0x85EBCA77u);
      uint32_t m = philox((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)rnd, (uint32_t)(rnd >> 32), k0, k1);
      acc += (rank == lo) ? m : (0u - m);
    }
    out[i] = acc;
  }
}

__global__ void secagg_unmask_kernel(const uint32_t* __restrict__ s, float* __restrict__ out, long long n,
                                     float inv_scale_div) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = (float)(int32_t)s[i] * inv_scale_div;
}

hipError_t secagg_quantize_mask(const float* x, uint32_t* out, long long n, float scale, float clip, int K,
                                int rank, unsigned long long seed, unsigned long long rnd, unsigned long long alive,
                                hipStream_t st) {
  if (K > 64) return hipErrorInvalidValue;
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(secagg_mask_kernel, dim3((int)b), dim3(256), 0, st, x, out, n, scale, clip, K, rank, seed,
                     rnd, alive);
  return hipGetLastError();
}

hipError_t secagg_dequantize(const uint32_t* sum, float* out, long long n, float scale, int K, float divisor,
                             hipStream_t st) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(secagg_unmask_kernel, dim3((int)b), dim3(256), 0, st, sum, out, n,
                     1.f / (scale * divisor));
  return hipGetLastError();
}

}  // namespace idc
