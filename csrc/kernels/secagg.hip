// Secure aggregation: fixed-point quantisation + pairwise Philox masks, dequantisation.
//
// Replaces the reference's per-element Python Paillier encryption (secure_fed_model.py:109-129,
// 3072-bit modexp per weight on the CPU) with one bandwidth-bound kernel: each element gets
// K-1 counter-based Philox4x32-10 masks keyed by the pair's Diffie-Hellman-derived key (one key
// table entry per peer, loaded once per thread into registers) and counted by (round, index),
// added with opposite signs by the two members of the pair, so the uint32 ring sum over all K
// clients equals the plain fixed-point sum bit-exactly.  Each protected tensor has its own
// fixed-point scale (segment table), so small kernels keep their resolution next to large BN
// variances.
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

// segment of element i at or after segment `from` (seg_end ascending, seg_end[nseg-1] == n)
__device__ __forceinline__ int segment_from(long long i, const long long* seg_end, int from, int nseg) {
  int lo = from, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (i < seg_end[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// Grid-stride over elements: consecutive lanes own consecutive elements, so every load and store
// is one coalesced 256-B wave access.  A thread's index only grows, so its segment index only moves
// forward: it is re-searched (binary, from the current segment) only when the element leaves it.
__global__ __launch_bounds__(256) void secagg_mask_kernel(const float* __restrict__ x, uint32_t* __restrict__ out,
                                                          long long n, const float* __restrict__ seg_scale,
                                                          const long long* __restrict__ seg_end, int nseg,
                                                          float clip, int K, int rank,
                                                          const uint32_t* __restrict__ keys, unsigned long long rnd,
                                                          unsigned long long alive, int accumulate) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int s = segment_from(i, seg_end, 0, nseg);
  float sc = seg_scale[s];
  for (; i < n; i += stride) {
    if (i >= seg_end[s]) {
      s = segment_from(i, seg_end, s, nseg);
      sc = seg_scale[s];
    }
    float v = x[i] * sc;
    v = fminf(fmaxf(v, -clip), clip);
    uint32_t acc = (uint32_t)(int32_t)rintf(v);
    for (int j = 0; j < K; ++j) {
      if (j == rank || !((alive >> j) & 1ull)) continue;  // dropped clients: re-keyed round
      const uint32_t m = philox((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)rnd, (uint32_t)(rnd >> 32),
                                keys[2 * j], keys[2 * j + 1]);
      acc += (rank < j) ? m : (0u - m);
    }
    // accumulate: add into the running masked sum of this rank's clients (uint32 wraps mod 2^32,
    // exactly the ring the all-reduce sums in), no per-client int32 temporary and no host-side
    // widen / add / modulo passes
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

__global__ __launch_bounds__(256) void secagg_unmask_kernel(const uint32_t* __restrict__ s, float* __restrict__ out,
                                                            long long n, const float* __restrict__ seg_scale,
                                                            const long long* __restrict__ seg_end, int nseg,
                                                            float divisor) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int g = segment_from(i, seg_end, 0, nseg);
  float inv = 1.f / (seg_scale[g] * divisor);
  for (; i < n; i += stride) {
    if (i >= seg_end[g]) {
      g = segment_from(i, seg_end, g, nseg);
      inv = 1.f / (seg_scale[g] * divisor);
    }
    out[i] = (float)(int32_t)s[i] * inv;
  }
}

// Per-segment max |x| (the quantisation ranges of secure aggregation), OR-ed into out[] as float
// bits (non-negative floats order like their bit patterns): block b owns the contiguous chunk
// [b*per, (b+1)*per), each thread keeps one running max per segment it walks through and merges it
// into the block's LDS bins when it leaves the segment; the block then adds its bins to out[] with
// one global atomic per segment it touched (a handful per block, not one per element).
constexpr int kAbsMaxBins = 4096;
__global__ __launch_bounds__(256) void secagg_absmax_kernel(const float* __restrict__ x, long long n,
                                                            const long long* __restrict__ seg_end, int nseg,
                                                            unsigned* __restrict__ out) {
  __shared__ unsigned bins[kAbsMaxBins];
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long c0 = blockIdx.x * per, c1 = c0 + per < n ? c0 + per : n;
  if (c0 >= c1) return;  // block-uniform
  const int s0 = segment_from(c0, seg_end, 0, nseg);
  const int s1 = segment_from(c1 - 1, seg_end, s0, nseg);
  const int nb = s1 - s0 + 1;
  for (int j = threadIdx.x; j < nb && j < kAbsMaxBins; j += blockDim.x) bins[j] = 0u;
  __syncthreads();
  auto flush = [&](int sg, unsigned m) {
    if (m == 0u) return;
    if (sg - s0 < kAbsMaxBins) atomicMax(&bins[sg - s0], m);
    else atomicMax(&out[sg], m);
  };
  long long i = c0 + threadIdx.x;
  int sg = s0;
  unsigned m = 0u;
  for (; i < c1; i += blockDim.x) {
    if (i >= seg_end[sg]) {
      flush(sg, m);
      m = 0u;
      sg = segment_from(i, seg_end, sg, nseg);
    }
    const unsigned b = __float_as_uint(fabsf(x[i]));
    m = b > m ? b : m;
  }
  flush(sg, m);
  __syncthreads();
  for (int j = threadIdx.x; j < nb && j < kAbsMaxBins; j += blockDim.x)
    if (bins[j]) atomicMax(&out[s0 + j], bins[j]);
}

static int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  return b < 1 ? 1 : (int)b;
}

hipError_t secagg_quantize_mask(const float* x, uint32_t* out, long long n, const float* seg_scale,
                                const long long* seg_end, int nseg, float clip, int K, int rank,
                                const uint32_t* keys, unsigned long long rnd, unsigned long long alive,
                                hipStream_t st, int accumulate) {
  if (K > 64 || nseg < 1 || (K > 1 && keys == nullptr)) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(secagg_mask_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, out, n, seg_scale, seg_end, nseg,
                     clip, K, rank, keys, rnd, alive, accumulate);
  return hipGetLastError();
}

hipError_t secagg_absmax(const float* x, long long n, const long long* seg_end, int nseg, unsigned* out,
                         hipStream_t st) {
  if (nseg < 1) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(secagg_absmax_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, n, seg_end, nseg, out);
  return hipGetLastError();
}

hipError_t secagg_dequantize(const uint32_t* sum, float* out, long long n, const float* seg_scale,
                             const long long* seg_end, int nseg, float divisor, hipStream_t st) {
  if (nseg < 1) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(secagg_unmask_kernel, dim3(grid_for(n)), dim3(256), 0, st, sum, out, n, seg_scale, seg_end,
                     nseg, divisor);
  return hipGetLastError();
}

}  // namespace idc
