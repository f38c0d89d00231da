// Cost of one cross-workgroup barrier of the persistent launches (persist.h) on MI355X: 256
// workgroups of 512 threads, one per CU (LDS-sized), ITERS barriers back to back, variants:
//   SLOTS: the BatchNorm-statistics pattern (slot atomics before the publish, slot sums after)
//   SLEEP: s_sleep between polls (0: spin)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels -o /tmp/barrier_cost tools/micro/barrier_cost.hip
#include "persist.h"
#include <cstdio>

using namespace idc;
using namespace idc::persist;

constexpr int ITERS = 200;

template <bool ATOM, bool READ, int S, int SLEEP>
__global__ __launch_bounds__(512) void barrier_kernel(unsigned* sync, float* slots, unsigned* fail, float* out) {
  extern __shared__ float lds[];
  __shared__ int s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int gi = blockIdx.x, G = gridDim.x;
  const FailSink fs{nullptr, nullptr, nullptr};
  float acc = 0.f;
  for (int it = 0; it < ITERS; ++it) {
    float* sl = slots + (size_t)it * 64 * 256;
    if (ATOM && tid < 256) atomicAdd(&sl[(gi % S) * 256 + tid], 1.f);
    unsigned* cnt = sync + it * 8;
    publish_shard(cnt, gi);
    if (wid == 0) {
      bool ok;
      if (SLEEP) {
        ok = wait_sum8(cnt, (unsigned)G, fail, fs, 1u << 20);
      } else {
        ok = false;
        for (unsigned p = 0; p < (1u << 24); ++p) {
          unsigned v = lane < 8 ? __hip_atomic_load(cnt + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          v += __shfl_xor(v, 4, 64);
          if (__builtin_amdgcn_readfirstlane(v) >= (unsigned)G) { ok = true; break; }
        }
      }
      if (lane == 0) s_bad = !ok;
    }
    __syncthreads();
    if (s_bad) return;
    if (READ && tid < 128) {
      float s0, s1;
      slot_sum<S>(sl, 128, tid, s0, s1);
      lds[tid] = s0 + s1;
    }
    __syncthreads();
    acc += lds[tid & 127];
  }
  if (tid == 0) out[gi] = acc;
}

template <bool ATOM, bool READ, int S, int SLEEP>
static void run(const char* name) {
  unsigned* sync;
  float* slots;
  unsigned* fail;
  float* out;
  hipMalloc(&sync, ITERS * 8 * 4);
  hipMalloc(&slots, (size_t)ITERS * 64 * 256 * 4);
  hipMalloc(&fail, 4);
  hipMalloc(&out, 256 * 4);
  const size_t smem = 100 * 1024;  // one workgroup per CU
  hipFuncSetAttribute((const void*)barrier_kernel<ATOM, READ, S, SLEEP>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipMemset(sync, 0, ITERS * 8 * 4);
    hipMemset(slots, 0, (size_t)ITERS * 64 * 256 * 4);
    hipMemset(fail, 0, 4);
    hipDeviceSynchronize();
    hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL((barrier_kernel<ATOM, READ, S, SLEEP>), dim3(256), dim3(512), smem, nullptr, sync, slots, fail, out);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  unsigned f = 0;
  hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
  printf("%-34s %.2f us per barrier (launch %.1f us, fail %u, %s)\n", name, best * 1e3 / ITERS, best * 1e3, f,
         hipGetErrorString(hipGetLastError()));
}

int main() {
  run<false, false, 8, 1>("barrier only");
  run<true, false, 8, 1>("slot atomics (8 copies) + barrier");
  run<false, true, 8, 1>("barrier + slot sums (8 copies)");
  run<true, true, 8, 1>("both, 8 copies");
  run<true, true, 32, 1>("both, 32 copies");
  run<true, true, 64, 1>("both, 64 copies");
  return 0;
}
