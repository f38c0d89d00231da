// Cross-workgroup hand-off primitives of the persistent work-queue kernels (dense_stage.hip,
// dense_stage_bwd.hip) on gfx950.
//
// Memory model: every byte a launch produces for another workgroup of the SAME launch is stored
// and loaded with agent-scope atomic accesses (global_* sc1: never a stale line of another XCD's
// L2 or of this CU's L1), the producer drains them (s_waitcnt vmcnt(0)) before ONE lane's counter
// increment, and the consumer loads after its poll matched and a workgroup barrier
// (MI355X_MICROARCH.md, "Valid forms", first table row).  Counters are polled with sc1 loads from
// one lane, an s_sleep apart: an atomic read-modify-write poll by ~200 workgroups contends with the
// producers' increments on the same word.
#pragma once
#include "common.h"

namespace idc {
namespace persist {

__device__ __forceinline__ uint4 ld_coh16(const void* p) {
  unsigned long long* q = (unsigned long long*)p;
  const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ float4 ld_coh_f4(const float* p) {
  const uint4 v = ld_coh16(p);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float ld_coh(const float* p) {
  return __hip_atomic_load((float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh8(void* p, uint32_t x, uint32_t y) {
  __hip_atomic_store((unsigned long long*)p, ((unsigned long long)y << 32) | x, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh16(void* p, const uint4& v) {
  st_coh8(p, v.x, v.y);
  st_coh8((unsigned long long*)p + 1, v.z, v.w);
}

constexpr unsigned DEFAULT_POLLS = 1u << 19;  // ~0.5-1 s of polling

// A launch gave up: the first workgroup to set the fail flag counts the launch in the persistent
// error counter and raises bit 1 of the program's per-step guard word (the flag the optimizer's
// skip test reads: the step's update is dropped, its stale outputs never reach the weights; the
// host sees the counter after the step, runtime/program.py FusedStep.check_persistent).
// ``hostflag`` (nullable) is a word of pinned host memory the runtime polls without a device
// synchronisation: a plain system-scope store of 1.
struct FailSink {
  int* err;
  int* stepflag;
  int* hostflag;
};
__device__ inline void note_fail(unsigned* fail, const FailSink& fs) {
  const unsigned old = __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == 0) {
    if (fs.err) atomicAdd(fs.err, 1);
    if (fs.stepflag) atomicOr(fs.stepflag, 2);
    if (fs.hostflag) __hip_atomic_store(fs.hostflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// thread 0: wait until *cnt >= need.  Every 256 polls the fail flag is checked.  On a timeout (or
// when another workgroup already failed) returns false; the workgroup that first sets the fail
// flag counts the launch in the persistent error counter.
__device__ inline bool wait_count(const unsigned* cnt, unsigned need, unsigned* fail, const FailSink& fs,
                                  unsigned max_polls) {
  unsigned polls = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(1);
    if ((++polls & 255u) == 0 || polls >= max_polls) {
      if (polls >= max_polls || __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        note_fail(fail, fs);
        return false;
      }
    }
  }
  return true;
}

// every thread's stores / atomics of this tile performed, then ONE lane's counter increment;
// returns (to thread 0) the counter's previous value
__device__ __forceinline__ unsigned publish(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned old = 0;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return old;
}

// Sharded completion counters: a phase's producers add into shard (tile % NSHARD) of an
// NSHARD-word counter so no word takes more than ~1/NSHARD of the arrivals (255 arrivals on one
// device-scope word serialise for ~3 us, MI355X_MICROARCH.md "fanin"); a consumer polls all
// shards with one 8-lane load and compares their sum.
constexpr int NSHARD = 8;

__device__ __forceinline__ unsigned publish_shard(unsigned* cnt8, int tile) {
  return publish(cnt8 + (tile & (NSHARD - 1)));
}

// called by ALL lanes of ONE wave: wait until the shards of cnt8 sum to >= need; returns a
// wave-uniform result (false: timeout or fail flag, counted like wait_count)
__device__ inline bool wait_sum8(const unsigned* cnt8, unsigned need, unsigned* fail, const FailSink& fs,
                                 unsigned max_polls) {
  const int lane = threadIdx.x & 63;
  unsigned polls = 0;
  for (;;) {
    unsigned v = lane < NSHARD ? __hip_atomic_load(cnt8 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if (__builtin_amdgcn_readfirstlane(v) >= need) return true;
    __builtin_amdgcn_s_sleep(1);
    ++polls;
    if ((polls & 255u) == 0 || polls >= max_polls) {
      unsigned f = lane == 0 ? __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      f = __builtin_amdgcn_readfirstlane(f);
      if (polls >= max_polls || f != 0) {
        if (lane == 0) note_fail(fail, fs);
        return false;
      }
    }
  }
}

constexpr int NSTAMP = 8;  // s_memrealtime stamps per work item (diagnostics)
__device__ __forceinline__ void stamp(unsigned long long* st, int task, int k) {
  if (st && threadIdx.x == 0) st[(size_t)task * NSTAMP + k] = __builtin_amdgcn_s_memrealtime();
}

// [sum, sumsq] of channel c over the S slot copies of a [S][2][C] statistics scratch (all loads
// issued before the adds)
template <int S>
__device__ __forceinline__ void slot_sum(const float* slots, int C, int c, float& s0, float& s1) {
  float a0[S], a1[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    a0[s] = ld_coh(slots + (size_t)s * 2 * C + c);
    a1[s] = ld_coh(slots + (size_t)s * 2 * C + C + c);
  }
  s0 = 0.f;
  s1 = 0.f;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    s0 += a0[s];
    s1 += a1[s];
  }
}

}  // namespace persist
}  // namespace idc
