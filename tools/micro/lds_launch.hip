// Launch-to-launch cost of a trivial 256 x 256-thread kernel vs its dynamic LDS size (does a large
// LDS allocation per workgroup cost time at dispatch?).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_launch tools/micro/lds_launch.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void touch(float* out, int n) {
  extern __shared__ float s[];
  s[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && out) out[blockIdx.x] = s[(threadIdx.x + 1) % 256] + n;
}

int main() {
  float* out = nullptr;
  (void)hipMalloc(&out, 1 << 20);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int sizes[] = {1024, 16384, 32768, 65536, 81920, 98304, 131072, 143360, 163840};
  for (int grid : {256, 512}) {
    for (int sz : sizes) {
      for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(touch, dim3(grid), dim3(256), sz, 0, out, sz);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(touch, dim3(grid), dim3(256), sz, 0, out, sz);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("grid %d LDS %6d B: %.2f us/launch (%s)\n", grid, sz, ms * 1e3 / 50, hipGetErrorString(hipGetLastError()));
    }
  }
  return 0;
}
