// Microbenchmark: cost of per-block same-address float atomics (the BN-statistics flush pattern).
// G blocks each add C floats (consecutive lanes -> one request per cache line) to ONE C-float array.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void flush(float* g, int C) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&g[c], 1.0f);
}
__global__ void flush_spread(float* g, int C, int copies) {
  float* d = g + (size_t)(blockIdx.x % copies) * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&d[c], 1.0f);
}
__global__ void nop(float* g) { if (threadIdx.x == 9999) g[0] = 1; }
int main() {
  float* g; hipMalloc(&g, 64 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int C : {64, 128, 256, 1024}) for (int G : {256, 676, 1024, 2500, 4096}) {
    float best = 1e9, bests = 1e9, bestn = 1e9;
    for (int r = 0; r < 20; ++r) {
      hipMemset(g, 0, 64 << 20);
      hipEventRecord(a); hipLaunchKernelGGL(flush, dim3(G), dim3(256), 0, 0, g, C); hipEventRecord(b);
      hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
      hipEventRecord(a); hipLaunchKernelGGL(flush_spread, dim3(G), dim3(256), 0, 0, g, C, 32); hipEventRecord(b);
      hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); if (ms < bests) bests = ms;
      hipEventRecord(a); hipLaunchKernelGGL(nop, dim3(G), dim3(256), 0, 0, g); hipEventRecord(b);
      hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); if (ms < bestn) bestn = ms;
    }
    printf("C=%5d G=%5d  same-address %7.2f us   32 copies %7.2f us   empty kernel %6.2f us\n", C, G, best * 1e3, bests * 1e3, bestn * 1e3);
  }
  return 0;
}
