// Instruction-fetch cost of straight-line code: a kernel whose waves execute R unrolled
// independent v_fma_f32 (8 B each, VOP3) once, vs the same count of FMAs in a 16-instruction
// loop.  Durations come from rocprofv3 --kernel-trace (dispatch order = the order printed).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/icache tools/micro/icache.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int R>
__global__ __launch_bounds__(256) void straight(float* out, float s) {
  float a = threadIdx.x * s, b = s, c = 1.f, d = 2.f;
#pragma unroll
  for (int i = 0; i < R / 4; ++i) {
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(b) : "v"(c), "v"(d));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(a));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(d) : "v"(a), "v"(b));
  }
  if (a + b + c + d == 12345.f) out[threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void looped(float* out, float s, int R) {
  float a = threadIdx.x * s, b = s, c = 1.f, d = 2.f;
  for (int i = 0; i < R / 16; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(b) : "v"(c), "v"(d));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(a));
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(d) : "v"(a), "v"(b));
    }
  }
  if (a + b + c + d == 12345.f) out[threadIdx.x] = a;
}

template <int R>
void run(float* out, int grid, const char* tag) {
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(straight<R>, dim3(grid), dim3(256), 0, 0, out, 1e-7f);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(looped, dim3(grid), dim3(256), 0, 0, out, 1e-7f, R);
  hipDeviceSynchronize();
  printf("%s R=%d (%d KB straight) grid=%d\n", tag, R, R * 8 / 1024, grid);
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  for (int grid : {1, 256, 1024}) {
    run<128>(out, grid, "case");
    run<1024>(out, grid, "case");
    run<2048>(out, grid, "case");
    run<4096>(out, grid, "case");
    run<6144>(out, grid, "case");
  }
  hipFree(out);
  return 0;
}
