// Persistent dense-stage forward for DenseNet (gfx950): all dense layers of one stage in ONE launch.
//
// A dense layer is  y = conv3x3(ReLU(BN2(conv1x1(ReLU(BN1(x[:, :cin]))))))  written into channels
// [cin, cin+32) of the stage buffer (reference: /root/reference/dist_model_tf_dense.py:131-133
// builds DenseNet-121 through Keras Applications).  In the late stages (bs 256:
// 3x3 and 1x1 maps, M = 2,304 / 256 pixels) every such conv is a few hundred MFLOP that the
// per-layer implicit GEMM runs in 7-15 us, almost all of it launch ramp, the serial K loop and the
// BN tables' memory round trips, while 40 layers x 2 convs = 80 launches sit on the critical path.
//
// Here one launch walks the whole stage as a WORK QUEUE of tiles:
//     [layer 0: 1x1 tiles][layer 0: 3x3 tiles][layer 1: 1x1 tiles] ...
// A workgroup takes the next ticket (one agent-scope atomic), and before it reads anything the
// previous phase produced it waits until that phase's completion counter is full.  Tickets are
// handed out in queue order, so every tile a waiting workgroup depends on was taken earlier by a
// workgroup that is already running (or done): the queue cannot deadlock whatever number of
// workgroups is resident (no co-residency assumption, no cooperative launch), and each wait has a
// bounded poll count besides (a per-launch fail flag: every workgroup then leaves, and the launch
// is counted in a persistent error counter), so a bug can never hang the GPU.  Weight fragments do
// not depend on earlier phases and are loaded BEFORE the wait, so a workgroup that took a ticket of
// the next phase early has its B operand in registers when the dependency clears.
//
// Hand-off between phases (DenseStageArgs::coh): by default the outputs are stored and the
// operands / statistics produced in this launch are loaded with agent-coherent (sc1) accesses, so
// no phase boundary pays an L2 writeback (release) or invalidate (acquire); with coh = 0 the
// counters are guarded by agent-scope release/acquire fences instead (~2.5 us per boundary).
//
// Tile shapes (64-wide waves, v_mfma_f32_16x16x32_bf16, operands straight from global/L2 into
// registers -- no LDS staging, a wave's K range in flight at once, in chunks for cin > 512):
//   1x1 phase: 32 rows x 64 output channels per tile (2 tiles across the 128 channels), the K
//              range (cin <= 1024) split over the 4 waves in chunks, partial tiles summed in LDS;
//   3x3 phase: 16 rows x all 32 output channels, the 9 taps x 128 channels split over the waves.
// Both phases apply the pending BatchNorm + ReLU of their operand in registers from a per-tile
// coefficient table computed from the shifted batch statistics (common.h), store bf16 and add the
// shifted statistics of the stored (rounded) values into the consumer's [sum|sumsq] arrays, exactly
// the contract of the per-layer kernels (conv_igemm_impl.h EPI 0), so the backward is unchanged.
#include "dense_stage.h"

namespace idc {
namespace {

constexpr int NT = 256;
constexpr int KC = 4;    // 1x1 phase: k-steps of 32 per wave per chunk (cin <= 512: one chunk)
constexpr int KB = 9;    // 3x3 phase: 9 taps x 128 channels / 32 / 4 waves
constexpr int RLD = 33;  // LDS partial-tile row stride of the 3x3 phase (floats)
constexpr int RLDA = 65; // ... of the 1x1 phase (64 columns)
constexpr unsigned MAX_POLLS = 1u << 19;  // ~0.5-1 s of polling

struct Smem {
  float sc[1024];
  float sh[1024];
  float red[4][32 * RLDA];
  int task;
  int bad;
};

// Agent-coherent loads of data other workgroups of this launch produced (sc1: never served from a
// stale line of this XCD's L2), so a consumer needs no L2-invalidating acquire fence
__device__ __forceinline__ uint4 ld_coh16(const void* p) {
  unsigned long long* q = (unsigned long long*)p;
  const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ float ld_coh(const float* p) {
  return __hip_atomic_load((float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0: wait until *cnt >= need (then acquire), or give up after MAX_POLLS / when another
// workgroup already gave up.  Returns false on a timeout.
__device__ bool wait_count(unsigned* cnt, unsigned need, unsigned* fail, bool coherent_loads) {
  // the counter is read with an atomic RMW (add 0): performed at the same coherence point as the
  // producers' increments whatever XCD / L2 this workgroup runs on.  The bound is a poll count
  // (each poll is a memory round trip plus an s_sleep), not a clock reading.
  unsigned polls = 0;
  while (__hip_atomic_fetch_add(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(2);
    if ((++polls & 255u) == 0 &&
        (polls > MAX_POLLS || __hip_atomic_fetch_add(fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  if (!coherent_loads) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// every thread's stores / atomics of this tile performed, then one agent-scope release + count
__device__ __forceinline__ void publish(unsigned* cnt, bool coherent_stores) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!coherent_stores) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// BN scale/shift for channels [0, C) (C <= 1024) from shifted [sum|sumsq] statistics (row length
// ld), all loads of a thread issued before any arithmetic
__device__ __forceinline__ void bn_table(const float* st, int ld, const float* shift, const float* g,
                                         const float* b, float inv_n, float eps, int C, float* sc, float* sh,
                                         bool coh) {
  const int tid = threadIdx.x;
  float s0[4], s1[4], k[4], gg[4], bb[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + u * NT;
    const int cc = c < C ? c : 0;
    s0[u] = coh ? ld_coh(st + cc) : st[cc];
    s1[u] = coh ? ld_coh(st + ld + cc) : st[ld + cc];
    k[u] = shift ? shift[cc] : 0.f;
    gg[u] = g[cc];
    bb[u] = b[cc];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + u * NT;
    if (c < C) {
      float mean, var;
      shifted_mean_var(k[u], s0[u], s1[u], inv_n, mean, var);
      const float r = gg[u] * rsqrtf(var + eps);
      sc[c] = r;
      sh[c] = bb[u] - mean * r;
    }
  }
}

__device__ __forceinline__ v8bf bn_act8(const uint4& x, const float* sc, const float* sh, float lo, float hi,
                                        bool keep) {
  float f[8];
  unpack8(x, f);
  const float4 a0 = *reinterpret_cast<const float4*>(sc), a1 = *reinterpret_cast<const float4*>(sc + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(sh), b1 = *reinterpret_cast<const float4*>(sh + 4);
  const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = keep ? clampf(f[j] * av[j] + bv[j], lo, hi) : 0.f;
  return __builtin_bit_cast(v8bf, pack8(f));
}

}  // namespace

// (outside the anonymous namespace so profiles name it: idc::dense_stage_kernel)
__global__ __launch_bounds__(NT) void dense_stage_kernel(DenseStageArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(DenseStageArgs) + sizeof(GroupArg)>();
  const long long go = goff(ga);
  bf16_t* __restrict__ buf = gsh(a.buf, go);
  float* __restrict__ sstats = gsh(a.sstats, go);
  const float* __restrict__ sshift = gsh(a.sshift, go);
  const DenseLayerDesc* __restrict__ layers = gsh(a.layers, go);
  unsigned* sync = gsh(a.sync, go);
  unsigned* fail = sync + 1 + 2 * a.nlayers;  // this launch gave up (zeroed with the counters)
  int* err = gsh(a.err, go);

  __shared__ __attribute__((aligned(16))) Smem s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int HW = a.H * a.W, M = a.N * HW;
  const int mtA = (M + 31) / 32, nA = mtA * 2;
  const int nB = (M + 15) / 16;
  const int per = nA + nB, total = per * a.nlayers;
  const int taps = a.k2 * a.k2, pad = a.k2 >> 1;
  const float lo1 = act_lo(a.act1), hi1 = act_hi(a.act1);
  const float lo2 = act_lo(a.act2), hi2 = act_hi(a.act2);
  const bool coh = (a.coh & 2) != 0;  // coherent loads, no acquire fence (dense_stage.h)

  for (;;) {
    // The ticket fetch is a thread-0 region enclosed by barriers on both sides.  Without the
    // leading barrier hipcc merged it with the previous tile's thread-0 publish (no convergent op
    // between them) and structurised the loop so that the other lanes of wave 0 and waves 1-3 went
    // round again to the barrier before thread 0 had fetched the next ticket: they re-ran the stale
    // tile forever (observed as a hang).
    __syncthreads();
    if (tid == 0) s.task = (int)__hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    // LDS broadcasts read through readfirstlane: the compiler then knows every control decision of
    // the loop is workgroup-uniform (scalar branches), so no barrier ever sits in exec-masked flow
    const int task = __builtin_amdgcn_readfirstlane(s.task);
    if (task >= total) {
      // the last workgroup out reports a failed launch into the persistent error counter
      if (tid == 0 && err && task == total + (int)gridDim.x - 1 &&
          __hip_atomic_fetch_add(fail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
        atomicAdd(err, 1);
      return;
    }
    const int l = task / per, r = task - l * per;
    DenseLayerDesc d = layers[l];
    const bf16_t* __restrict__ w1 = gsh(d.w1, go);
    const bf16_t* __restrict__ w2 = gsh(d.w2, go);
    bf16_t* __restrict__ tb = gsh(d.t, go);
    float* __restrict__ tst = gsh(d.tstats, go);
    const float* __restrict__ tsh = gsh(d.tshift, go);

    if (r < nA) {
      // ------------------------------------------------ 1x1 phase: t = conv1x1(relu(bn1(x)))
      // 32 rows x 64 channels per tile (2 tiles across the 128 channels: a 2,304-row stage is 144
      // tiles, one round on 256 CUs); each wave owns every 4th k-step and runs them in chunks of
      // KC, a chunk's A and B fragments all in flight at once (cin <= 512: one chunk)
      const int mt = r >> 1, n0 = (r & 1) * 64, m0 = mt * 32;
      const int cin = d.cin, nks = cin >> 5;
      v8bf bq[KC][4];
      auto load_b = [&](int c0k) {
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const int ks = wid + 4 * (c0k + i);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bq[i][j] = ks < nks ? *reinterpret_cast<const v8bf*>(w1 + (size_t)(n0 + j * 16 + fr) * cin + ks * 32 + fk)
                                : v8bf{};
        }
      };
      uint4 ar[KC][2];
      auto load_a = [&](int c0k) {
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const int ks = wid + 4 * (c0k + i);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int m = m0 + h * 16 + fr;
            const bf16_t* src = buf + (size_t)m * a.ld + ks * 32 + fk;
            ar[i][h] = (ks < nks && m < M) ? (coh ? ld_coh16(src) : *reinterpret_cast<const uint4*>(src))
                                           : make_uint4(0, 0, 0, 0);
          }
        }
      };
      load_b(0);  // weights do not depend on earlier phases: in flight before the wait
      const int erow = tid >> 3, ecol = (tid & 7) * 8;
      float kq[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) kq[q] = tsh ? tsh[n0 + ecol + q] : 0.f;
      if (l > 0) {
        if (tid == 0) s.bad = !wait_count(&sync[2 * l], (unsigned)nB, fail, coh);  // 3x3 phase of layer l-1
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s.bad)) return;
      }
      load_a(0);
      bn_table(sstats, a.ld, sshift, gsh(d.g1, go), gsh(d.b1, go), a.inv_count, d.eps1, cin, s.sc, s.sh, coh);
      __syncthreads();
      v4f acc[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][j] = v4f{0.f, 0.f, 0.f, 0.f};
      const int nchunks = (nks + 4 * KC - 1) / (4 * KC);
      for (int ch = 0; ch < nchunks; ++ch) {
        if (ch > 0) {
          load_b(ch * KC);
          load_a(ch * KC);
        }
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const int ks = wid + 4 * (ch * KC + i);
          if (ks < nks) {
            const int c0 = ks * 32 + fk;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const v8bf af = bn_act8(ar[i][h], s.sc + c0, s.sh + c0, lo1, hi1, true);
#pragma unroll
              for (int j = 0; j < 4; ++j)
                acc[h][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[i][j], acc[h][j], 0, 0, 0);
            }
          }
        }
      }
      float* red = s.red[wid];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) red[(h * 16 + (lane >> 4) * 4 + q) * RLDA + j * 16 + fr] = acc[h][j][q];
      __syncthreads();
      {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int o = erow * RLDA + ecol + q;
          v[q] = s.red[0][o] + s.red[1][o] + s.red[2][o] + s.red[3][o];
        }
        const int m = m0 + erow;
        const uint4 pk = pack8(v);
        if (m < M) {
          uint32_t* o = reinterpret_cast<uint32_t*>(tb + (size_t)m * 128 + n0 + ecol);
          if ((a.coh & 1)) {  // agent-coherent (sc1) stores: no release fence needed
            unsigned long long* o2 = reinterpret_cast<unsigned long long*>(o);
            __hip_atomic_store(o2, ((unsigned long long)pk.y << 32) | pk.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(o2 + 1, ((unsigned long long)pk.w << 32) | pk.z, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          } else {
            *reinterpret_cast<uint4*>(o) = pk;
          }
        }
        float rv[8];
        unpack8(pk, rv);
#pragma unroll
        for (int q = 0; q < 8; ++q) s.red[0][erow * RLDA + ecol + q] = m < M ? rv[q] - kq[q] : 0.f;
      }
      __syncthreads();
      if (tid < 128) {
        const int c = tid & 63, which = tid >> 6;
        float sum = 0.f;
#pragma unroll 8
        for (int row = 0; row < 32; ++row) {
          const float x = s.red[0][row * RLDA + c];
          sum += which ? x * x : x;
        }
        atomicAdd(&tst[which * 128 + n0 + c], sum);
      }
      publish(&sync[1 + 2 * l], (a.coh & 1));
    } else {
      // ------------------------------------------------ 3x3 phase: buf[:, cin:cin+32] = conv3x3(relu(bn2(t)))
      const int m0 = (r - nA) * 16;
      const int cin = d.cin, Kc = taps * 128, nks = taps * 4;
      v8bf bq[KB][2];
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int ks = wid + 4 * i;
        const int tap = ks >> 2, c = (ks & 3) * 32 + fk;
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bq[i][j] = ks < nks ? *reinterpret_cast<const v8bf*>(w2 + (size_t)(j * 16 + fr) * Kc + tap * 128 + c)
                              : v8bf{};
      }
      const int erow = tid >> 4, ecol = (tid & 15) * 2;
      float kq[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) kq[q] = sshift ? sshift[cin + ecol + q] : 0.f;
      const int m = m0 + fr;
      const int mm = m < M ? m : M - 1;
      const int img = mm / HW, rem = mm - img * HW;
      const int ph = rem / a.W, pw = rem - ph * a.W;
      if (tid == 0) s.bad = !wait_count(&sync[1 + 2 * l], (unsigned)nA, fail, coh);  // 1x1 phase of layer l
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s.bad)) return;
      uint4 ar[KB];
      bool okr[KB];
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int ks = wid + 4 * i;
        const int tap = ks >> 2;
        const int kr = tap / a.k2, kc = tap - kr * a.k2;
        const int hh = ph + kr - pad, ww = pw + kc - pad;
        okr[i] = ks < nks && m < M && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
        const bf16_t* src = tb + ((size_t)(img * a.H + hh) * a.W + ww) * 128 + (ks & 3) * 32 + fk;
        ar[i] = okr[i] ? (coh ? ld_coh16(src) : *reinterpret_cast<const uint4*>(src)) : make_uint4(0, 0, 0, 0);
      }
      if (tid < 128) {
        // 128 channels: one per thread (the 4-way table builder's other slots stay idle)
        const int c = tid;
        float mean, var;
        shifted_mean_var(tsh ? tsh[c] : 0.f, coh ? ld_coh(tst + c) : tst[c], coh ? ld_coh(tst + 128 + c) : tst[128 + c],
                         a.inv_count, mean, var);
        const float rr = gsh(d.g2, go)[c] * rsqrtf(var + d.eps2);
        s.sc[c] = rr;
        s.sh[c] = gsh(d.b2, go)[c] - mean * rr;
      }
      __syncthreads();
      v4f acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int ks = wid + 4 * i;
        if (ks < nks) {
          const int c0 = (ks & 3) * 32 + fk;
          // zero padding is applied AFTER the activation (Keras 'same' conv of relu(bn(t)))
          const v8bf af = bn_act8(ar[i], s.sc + c0, s.sh + c0, lo2, hi2, okr[i]);
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[i][j], acc[j], 0, 0, 0);
        }
      }
      float* red = s.red[wid];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[((lane >> 4) * 4 + q) * RLD + j * 16 + fr] = acc[j][q];
      __syncthreads();
      {
        float v[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int o = erow * RLD + ecol + q;
          v[q] = s.red[0][o] + s.red[1][o] + s.red[2][o] + s.red[3][o];
        }
        const int mo = m0 + erow;
        const uint32_t p = pack2bf(v[0], v[1]);
        if (mo < M) {
          uint32_t* o = reinterpret_cast<uint32_t*>(buf + (size_t)mo * a.ld + cin + ecol);
          if ((a.coh & 1)) __hip_atomic_store(o, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else *o = p;
        }
        const float rv[2] = {__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
#pragma unroll
        for (int q = 0; q < 2; ++q) s.red[0][erow * RLD + ecol + q] = mo < M ? rv[q] - kq[q] : 0.f;
      }
      __syncthreads();
      if (tid < 64) {
        const int c = tid & 31, which = tid >> 5;
        float sum = 0.f;
#pragma unroll
        for (int row = 0; row < 16; ++row) {
          const float x = s.red[0][row * RLD + c];
          sum += which ? x * x : x;
        }
        atomicAdd(&sstats[which * a.ld + cin + c], sum);
      }
      publish(&sync[2 + 2 * l], (a.coh & 1));
    }
  }
}

int dense_stage_tasks(const DenseStageArgs& a) {
  const long long M = (long long)a.N * a.H * a.W;
  return (int)(a.nlayers * (((M + 31) / 32) * 2 + (M + 15) / 16));
}

hipError_t dense_stage_fwd(const DenseStageArgs& a, int grid, hipStream_t st) {
  if (a.nlayers < 1 || (a.k2 != 1 && a.k2 != 3) || a.ld % 8 != 0 || a.N < 1 || a.H < 1 || a.W < 1 ||
      a.buf == nullptr || a.sstats == nullptr || a.layers == nullptr || a.sync == nullptr)
    return hipErrorInvalidValue;
  const int tasks = dense_stage_tasks(a);
  if (grid <= 0) grid = 256;
  // a grouped launch (K copies, each with its own queue) shares the CUs: one resident workgroup
  // per CU (256 VGPRs), so K copies of a full-chip grid would run one copy after another
  const int k = launch_groups().k;
  if (k > 1) grid = grid / k > 8 ? grid / k : 8;
  if (grid > tasks) grid = tasks;
  hipLaunchKernelGGL(dense_stage_kernel, ggrid(grid), dim3(NT), 0, st, a, garg());
  return hipGetLastError();
}

}  // namespace idc
