// Common device helpers for the idc_models_amd gfx950 (MI355X / CDNA4) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16 with an explicit per-pixel stride `ld` (elements) so a kernel can
//     read/write a channel SLICE of a wider buffer (DenseNet's concat-free stage buffers);
//   * all reductions accumulate in fp32; per-channel statistics are fp32 [sum | sumsq] arrays;
//   * wave = 64 lanes; every block size is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace idc {

typedef uint16_t bf16_t;  // raw bf16 bits
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// round-to-nearest-even; NaN kept a NaN (hipcc emits v_cvt_pk_bf16_f32 for the cast form)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
typedef float v2f_t __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (the scalar-cast form compiles to two
// single-lane converts plus a shift and an or)
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  v2f_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, v2bf_t));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2 };

// Activations are evaluated branch-free as a clamp to [lo, hi] (ReLU: [0,inf), ReLU6: [0,6],
// linear: (-inf,inf)); with `act` a kernel argument the bounds are loop-invariant selects, so the
// hot loops carry no per-element branches (a switch here compiled to per-element s_cbranch).
__device__ __forceinline__ float act_lo(int act) { return act ? 0.f : -INFINITY; }
__device__ __forceinline__ float act_hi(int act) { return act == ACT_RELU6 ? 6.f : INFINITY; }

// clamp to [lo, hi] in one v_med3_f32
__device__ __forceinline__ float clampf(float v, float lo, float hi) {
  return __builtin_amdgcn_fmed3f(v, lo, hi);
}

__device__ __forceinline__ float apply_act(float v, int act) {
  return clampf(v, act_lo(act), act_hi(act));
}

// derivative mask of the activation evaluated at pre-activation value z (TF: relu' = z > 0,
// relu6' = 0 < z < 6)
__device__ __forceinline__ float act_mask(float z, int act) {
  return (z > act_lo(act) && z < act_hi(act)) ? 1.f : 0.f;
}

// y[j] = act(x[j]*sc[j] + sh[j]) for 8 channels; sc/sh 32-B aligned LDS tables
__device__ __forceinline__ void affine_act8(float* v, const float* sc, const float* sh, float lo,
                                            float hi) {
  const float4 s0 = *reinterpret_cast<const float4*>(sc);
  const float4 s1 = *reinterpret_cast<const float4*>(sc + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(sh);
  const float4 h1 = *reinterpret_cast<const float4*>(sh + 4);
  const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = clampf(fmaf(v[j], s[j], h[j]), lo, hi);
}

// Sum 8 per-lane column partials over the lanes of a wave that own the same 8-column chunk
// (lane % CPB): afterwards every lane holds its chunk's wave total.  Used before the per-block
// statistics flush so LDS sees CPB-way instead of (64/CPB)-way same-address float atomics.
template <int CPB>
__device__ __forceinline__ void wave_reduce_chunks(float* v) {
#pragma unroll
  for (int o = CPB; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += __shfl_xor(v[j], o, 64);
  }
}

// Per-channel block totals of per-thread 8-channel partials: thread (tx, ty) owns channels
// [8tx, 8tx+8) of a CB-channel block for row group ty < R (threadIdx = ty * (CB/8) + tx).  The
// partials are transposed through `tmp` (2 * 256 * 8 floats) and summed down the row groups, so no
// LDS address has more than one writer: per-thread LDS float atomics on the same few addresses
// serialise R ways (R = 256 / (CB/8) = 32..64), and measured +6..22 us on the depthwise kernels.
// Results land in s_a / s_b [CB]; the caller synchronises before reading them.
__device__ __forceinline__ void chunk_sums(int CB, int R, int tx, int ty, const float* pa, const float* pb,
                                           float* tmp, float* s_a, float* s_b) {
  float* ta = tmp;
  float* tb = tmp + 256 * 8;
  if (ty < R) {
    const int o = ty * CB + tx * 8;
    *reinterpret_cast<float4*>(ta + o) = make_float4(pa[0], pa[1], pa[2], pa[3]);
    *reinterpret_cast<float4*>(ta + o + 4) = make_float4(pa[4], pa[5], pa[6], pa[7]);
    *reinterpret_cast<float4*>(tb + o) = make_float4(pb[0], pb[1], pb[2], pb[3]);
    *reinterpret_cast<float4*>(tb + o + 4) = make_float4(pb[4], pb[5], pb[6], pb[7]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < CB; c += blockDim.x) {
    float sa = 0.f, sb = 0.f;
    for (int r = 0; r < R; ++r) {
      sa += ta[r * CB + c];
      sb += tb[r * CB + c];
    }
    s_a[c] = sa;
    s_b[c] = sb;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a linear block id: consecutive "logical" tiles land on the same
// XCD (blocks b and b+8 share an XCD under round-robin dispatch), improving L2 reuse of shared
// operand panels.  Placement only affects speed, never correctness (guide §5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  if (nblocks < 2 * nx) return bid;
  int xcd = bid % nx;
  int q = nblocks / nx, r = nblocks % nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / nx;
}

// Kernel arguments reach the waves through the scalar cache, one 64-B line per miss, and the
// compiler loads each field where it is first used (then waits for it).  The conv / wgrad / pool
// descriptors are 300-650 B and are read in several phases (prologue tables, K loop, epilogue,
// statistics), so each phase paid a dependent miss on the kernarg segment: with kernargs moved to
// host memory (HIP_FORCE_DEV_KERNARG=0) a small backward conv took +6 us, i.e. several serial
// misses per launch.  Touching every line once at entry, all loads in flight together, turns
// those into one round trip that overlaps the first tile loads.
template <int BYTES>
__device__ __forceinline__ void prefetch_kernargs() {
  const unsigned* p = (const unsigned*)__builtin_amdgcn_kernarg_segment_ptr();
  constexpr int L = (BYTES + 63) / 64;
  unsigned v[L];
#pragma unroll
  for (int i = 0; i < L; ++i) v[i] = p[i * 16];
#pragma unroll
  for (int i = 0; i < L; ++i) asm volatile("" ::"s"(v[i]));
}

// ---------------------------------------------------------------------------------------------
// Grouped execution (client-batched federated training; runtime/grouped.py).
// A grouped program keeps K copies of ALL its buffers at one fixed byte stride: copy g of any
// buffer lives at (address of copy 0) + g * stride.  One grouped launch runs all K copies: the
// launcher multiplies its grid's z extent by K (ggrid), and a workgroup's copy is
// g = blockIdx.z / zn, zn being the kernel's own z extent (1 unless it splits over z itself).
// Every pointer the workgroup dereferences -- its argument struct's and the ones it reads from
// device descriptor tables -- is shifted by g * stride (gshift / gsh); null pointers stay null
// (they select modes).  The host side checks that every pointer of a grouped plan lies inside
// copy 0, so a shift never leaves the program's own memory.  Ungrouped launches: stride 0.
struct GroupArg {
  long long stride;  // bytes between copies (0: ungrouped)
  int zn;            // the kernel's own z extent
  int pad;
};
struct LaunchGroups {
  int k = 1;
  long long stride = 0;
};
LaunchGroups& launch_groups();  // per host thread; the plan executor sets it around grouped ops
inline GroupArg garg(int zn = 1) {
  const LaunchGroups& l = launch_groups();
  return GroupArg{l.k > 1 ? l.stride : 0, zn, 0};
}
inline dim3 ggrid(dim3 g) {
  g.z *= (unsigned)launch_groups().k;
  return g;
}
inline dim3 ggrid(int gx) { return ggrid(dim3((unsigned)gx)); }
__device__ __forceinline__ long long goff(const GroupArg& ga) {
  return ga.stride ? (long long)(blockIdx.z / (unsigned)ga.zn) * ga.stride : 0;
}
__device__ __forceinline__ int gz(const GroupArg& ga) { return (int)(blockIdx.z % (unsigned)ga.zn); }
// Every pointer a kernel dereferences is device global memory (hipMalloc / torch allocations),
// but pointers read from argument structs and device tables are generic ("flat") to the
// compiler, and an integer round trip hides their provenance for good: hipcc then emits FLAT
// loads/stores, which count in both vmcnt and lgkmcnt, so every LDS wait (lgkmcnt) of a K loop
// also waited for the global prefetch in flight, and flat accesses are invalid for the sc1
// hand-off protocol (MI355X_MICROARCH.md "Valid forms").  gsh therefore routes every pointer
// through the global address space (addrspace(1)); LLVM's address-space inference then turns
// every access derived from it into global_* / buffer-free vector memory instructions.
template <typename T>
using gptr_t = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ T* as_global(T* p) {
  return (T*)(gptr_t<T>)p;
}
template <typename T>
__device__ __forceinline__ T* gsh(T* p, long long off) {
  typedef __attribute__((address_space(1))) char gchar;
  gchar* q = (gchar*)(gptr_t<T>)p;
  return (T*)(gptr_t<T>)(q ? q + off : q);  // null pointers stay null (they select modes)
}

// BatchNorm descriptor shared by every kernel that applies a BN affine (+activation) to an
// operand on the fly ("pending BN").  mode 1: batch statistics from `stats` ([sum|sumsq] over
// `count` samples); mode 2: inference (moving statistics).  mode 0: identity (act only).
struct BnArgs {
  const float* stats;     // [2*C] sum, sumsq (mode 1)
  const float* gamma;     // [C]
  const float* beta;      // [C]
  const float* mmean;     // [C] (mode 2)
  const float* mvar;      // [C] (mode 2)
  float inv_count;        // 1/count for mode 1
  float eps;
  int mode;
  int act;
  int C;                  // channels covered by stats/gamma (stats row length)
  int slots;              // mode 1: `stats` holds this many [sum|sumsq] copies (0/1: one), see below
  const float* shift;     // mode 1 (nullable): per-channel shift K, stats hold sum(y-K), sum((y-K)^2)
};

__device__ __forceinline__ void gshift(BnArgs& b, long long o) {
  b.stats = gsh(b.stats, o); b.gamma = gsh(b.gamma, o); b.beta = gsh(b.beta, o);
  b.mmean = gsh(b.mmean, o); b.mvar = gsh(b.mvar, o); b.shift = gsh(b.shift, o);
}

// Shifted statistics.  Producers accumulate sum(y - K) and sum((y - K)^2) with a per-channel
// shift K (the previous step's batch mean, updated after every backward by stats_shift_kernel),
// so the variance sum((y-K)^2)/n - (sum(y-K)/n)^2 cancels only (mean - K)^2 instead of mean^2:
// a channel with mean 50 and std 0.1 loses ~all of its fp32 variance in E[y^2] - E[y]^2 (the
// 2500-sized sums round at ~1e-4 per add) but keeps it with K ~ 50.  K = 0 on the first step.
__device__ __forceinline__ float bn_shift(const BnArgs& b, int c) { return b.shift ? b.shift[c] : 0.f; }
__device__ __forceinline__ void shifted_mean_var(float k, float s0, float s1, float inv_n, float& mean,
                                                 float& var) {
  const float d = s0 * inv_n;
  mean = k + d;
  var = fmaxf(s1 * inv_n - d * d, 0.f);
}

// Statistics slots.  Per-channel sums are accumulated with global float atomics, which execute
// at the memory side and serialise per ADDRESS (measured ~24 ns per add, tools/micro/
// atomic_flush.hip: 676 workgroups adding into one array cost +14 us, 2500 cost +58 us, the same
// adds spread over 32 copies cost nothing).  Producers with many row blocks therefore add into
// copy (row block % slots) of a [slots][2][C] array, and every consumer sums the copies while it
// builds its coefficient table (slots x 2C L2-resident floats per workgroup).
__device__ __forceinline__ int stat_slots(int s) { return s > 1 ? s : 1; }

// Slot-summed [sum, sumsq] of channel cc, every one of the 2*MAX_STAT_SLOTS loads issued before the
// first add (slots past S re-read copy S-1 and are masked out: unconditional loads keep hipcc from
// branching around each one and waiting per element), so a table costs one memory round trip.
constexpr int MAX_STAT_SLOTS = 16;
__device__ __forceinline__ void slot_sums_1(const float* p0, const float* p1, int S, size_t stride, int cc,
                                            float& v0, float& v1) {
  if (S == 1) {  // single copy (small maps): two loads, not 2*MAX_STAT_SLOTS
    v0 = p0[cc];
    v1 = p1[cc];
    return;
  }
  if (S <= 4) {
    float t0[4], t1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const size_t o = (size_t)(s < S ? s : S - 1) * stride + cc;
      t0[s] = p0[o];
      t1[s] = p1[o];
    }
    v0 = 0.f;
    v1 = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v0 += s < S ? t0[s] : 0.f;
      v1 += s < S ? t1[s] : 0.f;
    }
    return;
  }
  float t0[MAX_STAT_SLOTS], t1[MAX_STAT_SLOTS];
#pragma unroll
  for (int s = 0; s < MAX_STAT_SLOTS; ++s) {
    const size_t o = (size_t)(s < S ? s : S - 1) * stride + cc;
    t0[s] = p0[o];
    t1[s] = p1[o];
  }
  v0 = 0.f;
  v1 = 0.f;
#pragma unroll
  for (int s = 0; s < MAX_STAT_SLOTS; ++s) {
    v0 += s < S ? t0[s] : 0.f;
    v1 += s < S ? t1[s] : 0.f;
  }
}

// [sum, sumsq] of channel c over all slot copies (mode 1)
__device__ __forceinline__ void bn_slot_sums(const BnArgs& b, int c, float& s0, float& s1) {
  const int S = min(stat_slots(b.slots), MAX_STAT_SLOTS);
  if (S == 1) {
    s0 = b.stats[c];
    s1 = b.stats[b.C + c];
    return;
  }
  slot_sums_1(b.stats, b.stats + b.C, S, 2 * (size_t)b.C, c, s0, s1);
}

__device__ __forceinline__ void bn_coeffs(const BnArgs& b, int c, float& scale, float& shift) {
  if (b.mode == 0) {
    scale = 1.f;
    shift = 0.f;
    return;
  }
  float mean, var;
  if (b.mode == 1) {
    float s0, s1;
    bn_slot_sums(b, c, s0, s1);
    shifted_mean_var(bn_shift(b, c), s0, s1, b.inv_count, mean, var);
  } else {
    mean = b.mmean[c];
    var = b.mvar[c];
  }
  float r = rsqrtf(var + b.eps);
  float g = b.gamma ? b.gamma[c] : 1.f;
  float be = b.beta ? b.beta[c] : 0.f;
  scale = g * r;
  shift = be - mean * scale;
}

// BN scale/shift table for channels [0, C) into LDS, NT threads.  All global loads of a thread
// (up to 4 channels per batch) are issued before any arithmetic so the table costs ONE memory
// latency, not one per channel slot (loads retire in order: a per-channel loop would wait for
// each slot's loads in turn).
template <int NT>
__device__ __forceinline__ void bn_coeff_table(const BnArgs& b, int C, float* s_scale, float* s_shift) {
  const int tid = threadIdx.x;
  if (b.mode == 0) {
    for (int c = tid; c < C; c += NT) { s_scale[c] = 1.f; s_shift[c] = 0.f; }
    return;
  }
  const float* p0 = b.mode == 1 ? b.stats : b.mmean;
  const float* p1 = b.mode == 1 ? b.stats + b.C : b.mvar;
  const float mul = b.mode == 1 ? b.inv_count : 1.f;
  const int S = b.mode == 1 ? min(stat_slots(b.slots), MAX_STAT_SLOTS) : 1;
  const size_t stride = 2 * (size_t)b.C;
  // slotted statistics: one channel per thread per pass, all slot copies in flight at once
  for (int c = tid; S > 1 && c < C; c += NT) {
    float v0, v1;
    slot_sums_1(p0, p1, S, stride, c, v0, v1);
    const float g = b.gamma ? b.gamma[c] : 1.f;
    const float be = b.beta ? b.beta[c] : 0.f;
    float mean, var;
    shifted_mean_var(bn_shift(b, c), v0, v1, mul, mean, var);
    const float rs = rsqrtf(var + b.eps);
    s_scale[c] = g * rs;
    s_shift[c] = be - mean * g * rs;
  }
  for (int base = 0; S == 1 && base < C; base += 4 * NT) {
    float v0[4], v1[4], g[4], be[4], k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int c = base + u * NT + tid;
      int cc = c < C ? c : 0;
      v0[u] = p0[cc];
      v1[u] = p1[cc];
      g[u] = b.gamma ? b.gamma[cc] : 1.f;
      be[u] = b.beta ? b.beta[cc] : 0.f;
      k[u] = b.mode == 1 ? bn_shift(b, cc) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int c = base + u * NT + tid;
      if (c >= C) break;
      float mean = v0[u], var = v1[u];
      if (b.mode == 1) shifted_mean_var(k[u], v0[u], v1[u], mul, mean, var);
      float sc = g[u] * rsqrtf(var + b.eps);
      s_scale[c] = sc;
      s_shift[c] = be[u] - mean * sc;
    }
  }
}

// Backward tables for channels [0, C): BN scale/shift (to recompute z = bn(x)) and mean/rstd
// (for x-hat), all global loads of a batch of 4 channels per thread issued before any arithmetic.
// mode 0 gives the identity (1, 0, 0, 1).
template <int NT>
__device__ __forceinline__ void bn_full_table(const BnArgs& b, int C, float* s_sc, float* s_sh, float* s_mu,
                                              float* s_rs) {
  const int tid = threadIdx.x;
  if (b.mode == 0) {
    for (int c = tid; c < C; c += NT) { s_sc[c] = 1.f; s_sh[c] = 0.f; s_mu[c] = 0.f; s_rs[c] = 1.f; }
    return;
  }
  const float* p0 = b.mode == 1 ? b.stats : b.mmean;
  const float* p1 = b.mode == 1 ? b.stats + b.C : b.mvar;
  const float mul = b.mode == 1 ? b.inv_count : 1.f;
  const int S = b.mode == 1 ? min(stat_slots(b.slots), MAX_STAT_SLOTS) : 1;
  const size_t stride = 2 * (size_t)b.C;
  // slotted statistics: one channel per thread per pass, all slot copies in flight at once
  for (int c = tid; S > 1 && c < C; c += NT) {
    float v0, v1;
    slot_sums_1(p0, p1, S, stride, c, v0, v1);
    const float g = b.gamma ? b.gamma[c] : 1.f;
    const float be = b.beta ? b.beta[c] : 0.f;
    float mean, var;
    shifted_mean_var(bn_shift(b, c), v0, v1, mul, mean, var);
    const float rs = rsqrtf(var + b.eps);
    s_sc[c] = g * rs;
    s_sh[c] = be - mean * g * rs;
    s_mu[c] = mean;
    s_rs[c] = rs;
  }
  for (int base = 0; S == 1 && base < C; base += 4 * NT) {
    float v0[4], v1[4], g[4], be[4], k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int c = base + u * NT + tid;
      int cc = c < C ? c : 0;
      v0[u] = p0[cc];
      v1[u] = p1[cc];
      g[u] = b.gamma ? b.gamma[cc] : 1.f;
      be[u] = b.beta ? b.beta[cc] : 0.f;
      k[u] = b.mode == 1 ? bn_shift(b, cc) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int c = base + u * NT + tid;
      if (c >= C) break;
      float mean = v0[u], var = v1[u];
      if (b.mode == 1) shifted_mean_var(k[u], v0[u], v1[u], mul, mean, var);
      float rs = rsqrtf(var + b.eps);
      float sc = g[u] * rs;
      s_sc[c] = sc;
      s_sh[c] = be[u] - mean * sc;
      s_mu[c] = mean;
      s_rs[c] = rs;
    }
  }
}

// Pending BatchNorm BACKWARD ("backward pending affine").  The input gradient of a training-mode
// BatchNorm is  dX = A*dZ + B*X + C  per channel, with
//   A = gamma*rstd,  B = -gamma*rstd^2 * mean(dZ*xhat),  C = -gamma*rstd*mean(dZ) - B*mean
// where the two means are reductions over the whole batch that the PRODUCER of dZ accumulated.
// Instead of materialising dX with a separate pass (one launch + a full write and re-read per BN),
// every CONSUMER of dX stages  v' = A*v + B*x + C  while loading its operand v (= dZ), with x the
// BN's raw forward input at the same pixel and channel.  With `unit_alpha` the operand already
// holds the A*dZ terms (DenseNet's fp32 concat-gradient buffer, into which each BatchNorm's
// producer accumulated A*dZ in its epilogue) and only the B*x + C part of ONE BatchNorm is
// still pending.  mode 0 = off; inference-mode BatchNorms (mode 2) give A = gamma*rstd, B = C = 0.
// All pointers are pre-offset to the operand's first channel.  Optionally one workgroup of the
// consumer folds the statistics-slot copies of the reductions into the BatchNorm's d beta / d gamma
// (fold_*: channels [0, fold_C) from gsum/gsumx bases fgsum/fgsumx).
// mode 1: pending BatchNorm BACKWARD (v' = A*dZ + B*x + C, A/B/C from the BN's statistics and
// gradient sums; unit_alpha: A = 1).  mode 2: a BatchNorm FORWARD applied while a consumer stages
// its operand, plus an optional residual tensor x (unit_alpha = 1: v' = sc*v + sh + x) -- the
// MobileNetV2 block output BN_project(p) [+ h_in] built inside the next expand conv.
struct BwdAff {
  const bf16_t* x; int ldx;
  BnArgs bn;
  const float* gsum; const float* gsumx;
  int gsum_slots, gsum_ld;
  float inv_n;
  int unit_alpha;
  int mode;
  int fold_C;
  const float* fgsum; const float* fgsumx;
  float* fold_sum; float* fold_sumx;
};

__device__ __forceinline__ void gshift(BwdAff& b, long long o) {
  b.x = gsh(b.x, o); gshift(b.bn, o); b.gsum = gsh(b.gsum, o); b.gsumx = gsh(b.gsumx, o);
  b.fgsum = gsh(b.fgsum, o); b.fgsumx = gsh(b.fgsumx, o);
  b.fold_sum = gsh(b.fold_sum, o); b.fold_sumx = gsh(b.fold_sumx, o);
}

// A/B/C table for channels c0 + [0, n) into sA/sB/sC[0, n) (LDS); channels at or past `lim` get
// the identity; all loads of a channel are issued before its arithmetic.
template <int NT>
__device__ __forceinline__ void bwd_aff_table(const BwdAff& b, int c0, int n, int lim, float* sA, float* sB,
                                              float* sC) {
  const int tid = threadIdx.x;
  const int SS = b.bn.mode == 1 ? min(stat_slots(b.bn.slots), MAX_STAT_SLOTS) : 1;
  const int SG = b.bn.mode == 1 ? min(stat_slots(b.gsum_slots), MAX_STAT_SLOTS) : 1;
  for (int i = tid; i < n; i += NT) {
    const int c = c0 + i;
    if (b.mode == 0 || c >= lim) {
      sA[i] = 1.f;
      sB[i] = 0.f;
      sC[i] = 0.f;
      continue;
    }
    float m0, m1, q0 = 0.f, q1 = 0.f;
    const float g = b.bn.gamma ? b.bn.gamma[c] : 1.f;
    if (b.bn.mode == 1) {
      slot_sums_1(b.bn.stats, b.bn.stats + b.bn.C, SS, 2 * (size_t)b.bn.C, c, m0, m1);
      if (b.mode == 1) slot_sums_1(b.gsum, b.gsumx, SG, (size_t)b.gsum_ld, c, q0, q1);
    } else {
      m0 = b.bn.mmean[c];
      m1 = b.bn.mvar[c];
    }
    float mean = m0, var = m1;
    if (b.bn.mode == 1) shifted_mean_var(bn_shift(b.bn, c), m0, m1, b.bn.inv_count, mean, var);
    const float rstd = rsqrtf(var + b.bn.eps);
    if (b.mode == 2) {  // forward BatchNorm (+ residual x): v' = g*rstd*v + [x] + beta - mean*g*rstd
      sA[i] = g * rstd;
      sB[i] = b.unit_alpha ? 1.f : 0.f;
      sC[i] = (b.bn.beta ? b.bn.beta[c] : 0.f) - mean * g * rstd;
      continue;
    }
    const float sd = q0 * b.inv_n, sdx = q1 * b.inv_n;
    const float Bc = -g * rstd * rstd * sdx;
    sA[i] = b.unit_alpha ? 1.f : g * rstd;
    sB[i] = Bc;
    sC[i] = -g * rstd * sd - Bc * mean;
  }
}

// Batched table inputs for launches whose statistics have at most 4 slot copies (every layer with
// <= 16K rows: DenseNet stages 2-4).  The general table builders above branch on the runtime slot
// count and wait for each array's loads before the next array's are issued, so a backward conv
// with a pending-affine prologue and an epilogue BatchNorm paid three to four dependent memory
// round trips before its K loop (tools/micro/conv_phases.hip: ~6k shader cycles for the prologue
// table alone).  Here every load of every table a thread builds is issued first (4 clamped slot
// loads per array, unconditional), then everything is combined: one round trip.
#ifndef IDC_BATCH_SLOTS
#define IDC_BATCH_SLOTS 4
#endif
// slot copies the batched loads take: 8 (-DIDC_BATCH_SLOTS=8) costs 20-40 registers in the
// backward conv tiles and one occupancy step on 32 of them (tools/kernel_resources.py, round 5)
constexpr int BATCH_SLOTS = IDC_BATCH_SLOTS;
struct Raw4 {
  float a0[BATCH_SLOTS], a1[BATCH_SLOTS];
};
__device__ __forceinline__ void load4(const float* p0, const float* p1, int S, size_t stride, int c, Raw4& r) {
#pragma unroll
  for (int s = 0; s < BATCH_SLOTS; ++s) {
    const size_t o = (size_t)(s < S ? s : S - 1) * stride + c;
    r.a0[s] = p0[o];
    r.a1[s] = p1[o];
  }
}
__device__ __forceinline__ void sum4(const Raw4& r, int S, float& v0, float& v1) {
  v0 = r.a0[0];
  v1 = r.a1[0];
#pragma unroll
  for (int s = 1; s < BATCH_SLOTS; ++s) {
    v0 += s < S ? r.a0[s] : 0.f;
    v1 += s < S ? r.a1[s] : 0.f;
  }
}
__device__ __forceinline__ bool bn_slots4(const BnArgs& b) { return b.mode != 1 || stat_slots(b.slots) <= BATCH_SLOTS; }
__device__ __forceinline__ bool bwd_aff_slots4(const BwdAff& b) {
  return b.mode == 0 || b.bn.mode != 1 ||
         (stat_slots(b.bn.slots) <= BATCH_SLOTS && stat_slots(b.gsum_slots) <= BATCH_SLOTS);
}

// raw inputs of one channel of a BwdAff table (training-mode BatchNorm, <= 4 slots)
struct BwdAffRaw {
  Raw4 st, gs;
  float g, k, be;
};
__device__ __forceinline__ void bwd_aff_load(const BwdAff& b, int c, BwdAffRaw& r) {
  load4(b.bn.stats, b.bn.stats + b.bn.C, stat_slots(b.bn.slots), 2 * (size_t)b.bn.C, c, r.st);
  if (b.mode == 1) load4(b.gsum, b.gsumx, stat_slots(b.gsum_slots), (size_t)b.gsum_ld, c, r.gs);
  r.g = b.bn.gamma ? b.bn.gamma[c] : 1.f;
  r.k = bn_shift(b.bn, c);
  r.be = (b.mode == 2 && b.bn.beta) ? b.bn.beta[c] : 0.f;
}
__device__ __forceinline__ void bwd_aff_finish(const BwdAff& b, const BwdAffRaw& r, float& A, float& B, float& C) {
  float m0, m1, q0, q1;
  sum4(r.st, stat_slots(b.bn.slots), m0, m1);
  float mean, var;
  shifted_mean_var(r.k, m0, m1, b.bn.inv_count, mean, var);
  const float rstd = rsqrtf(var + b.bn.eps);
  if (b.mode == 2) {  // forward BatchNorm (+ residual), see bwd_aff_table
    A = r.g * rstd;
    B = b.unit_alpha ? 1.f : 0.f;
    C = r.be - mean * A;
    return;
  }
  sum4(r.gs, stat_slots(b.gsum_slots), q0, q1);
  const float Bc = -r.g * rstd * rstd * (q1 * b.inv_n);
  A = b.unit_alpha ? 1.f : r.g * rstd;
  B = Bc;
  C = -r.g * rstd * (q0 * b.inv_n) - Bc * mean;
}

// d beta / d gamma of the BatchNorm: sum of the slot copies, once per step, spread over the
// launch's workgroups (a 64-channel-aligned share each) so no single workgroup's prologue carries
// the whole fold
template <int NT>
__device__ __forceinline__ void bwd_aff_fold(const BwdAff& b) {
  if (b.fold_sum == nullptr) return;
  // (x, y only: a grouped launch's z is the program copy, each copy folds its own sums)
  const int nb = gridDim.x * gridDim.y;
  const int bid = blockIdx.x + gridDim.x * blockIdx.y;
  int share = (b.fold_C + nb - 1) / nb;
  share = (share + 63) / 64 * 64;
  const int c0 = bid * share, c1 = min(b.fold_C, c0 + share);
  const int SG = min(stat_slots(b.gsum_slots), MAX_STAT_SLOTS);
  for (int c = c0 + (int)threadIdx.x; c < c1; c += NT) {
    float q0, q1;
    slot_sums_1(b.fgsum, b.fgsumx, SG, (size_t)b.gsum_ld, c, q0, q1);
    b.fold_sum[c] += q0;
    b.fold_sumx[c] += q1;
  }
}

// v[j] = A[j]*v[j] + B[j]*x[j] + C[j] for 8 channels (tables 32-B aligned in LDS)
__device__ __forceinline__ void bwd_aff8(float* v, const float* x, const float* sA, const float* sB,
                                         const float* sC) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = fmaf(sA[j], v[j], fmaf(sB[j], x[j], sC[j]));
}

// mean and 1/sigma of a channel (for x-hat in backward)
__device__ __forceinline__ void bn_mean_rstd(const BnArgs& b, int c, float& mean, float& rstd) {
  float var;
  if (b.mode == 1) {
    float s0, s1;
    bn_slot_sums(b, c, s0, s1);
    shifted_mean_var(bn_shift(b, c), s0, s1, b.inv_count, mean, var);
  } else {
    mean = b.mmean[c];
    var = b.mvar[c];
  }
  rstd = rsqrtf(var + b.eps);
}

}  // namespace idc
