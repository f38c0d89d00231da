// Memory-bound kernels of the idc_models_amd runtime (gfx950).
//
// Every kernel here streams NHWC bf16 (or fp32 gradient) rows with 16-byte vectors: a thread owns
// one 8-channel chunk of a row (guide Guideline 13), a block covers R = 256/(C/8) rows per sweep
// and per-channel reductions go lane -> LDS float atomics -> ONE global atomic per channel per
// block.  Per-channel BN coefficients are computed once per block into LDS.
//
//   bn_bwd_apply   dst (=|+=) A*dZ + B*x + C      BatchNorm backward (DenseNet concat grads += )
//   bn_bwd_reduce  dZ = dy*act'(bn(x)), sum dZ, sum dZ*xhat   (BN backward pass 1)
//   maxpool_fwd    pending BN+act -> max pool (+argmax, +output stats)   (DenseNet stem, VGG)
//   avgpool_fwd    pending BN+act -> avg pool (DenseNet transition: pool BEFORE the 1x1 conv,
//                  exact because a 1x1 conv commutes with 2x2 average pooling; 4x fewer FLOPs)
//   pool_bwd       max/avg pool backward as a GATHER (no atomics) + BN-backward epilogue
//   bn_update_moving  all BN layers' moving mean/var in ONE launch per step
//   head_fwd/bwd   fused [BN+act ->] GAP -> Dense -> BCE / softmax-CE (+ grads)
//   rmsprop        fused Keras RMSprop over the flat fp32 arena (1/world folded in)
//   cast_weights   fp32 Keras HWIO master -> bf16 kernel layouts (fwd + flipped dgrad), one launch
//   input_stage    uint8/fp32 NHWC images -> bf16 NHWC padded to 8 channels
#include "common.h"
#include <cstdlib>

#include "nn_kernels.h"
#include "persist.h"

namespace idc {

LaunchGroups& launch_groups() {
  static thread_local LaunchGroups lg;
  return lg;
}


namespace {

struct ChunkMap {
  int C8, R, tx, ty;
  __device__ ChunkMap(int C) {
    C8 = C / 8;
    R = 256 / C8;
    if (R < 1) R = 1;
    tx = threadIdx.x % C8;
    ty = threadIdx.x / C8;
  }
  __device__ bool active() const { return ty < R; }
};

__device__ __forceinline__ void load8(const void* base, int f32, size_t off, float* v) {
  if (f32) {
    const float* p = reinterpret_cast<const float*>(base) + off;
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(base) + off);
    unpack8(u, v);
  }
}

__device__ __forceinline__ void store8(void* base, int f32, size_t off, const float* v, int acc) {
  if (f32) {
    float* p = reinterpret_cast<float*>(base) + off;
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = v[j];
    if (acc) {
      float4 a = *reinterpret_cast<const float4*>(p);
      float4 b = *reinterpret_cast<const float4*>(p + 4);
      w[0] += a.x; w[1] += a.y; w[2] += a.z; w[3] += a.w;
      w[4] += b.x; w[5] += b.y; w[6] += b.z; w[7] += b.w;
    }
    *reinterpret_cast<float4*>(p) = make_float4(w[0], w[1], w[2], w[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(w[4], w[5], w[6], w[7]);
  } else {
    bf16_t* p = reinterpret_cast<bf16_t*>(base) + off;
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = v[j];
    if (acc) {
      float o[8];
      unpack8(*reinterpret_cast<const uint4*>(p), o);
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] += o[j];
    }
    *reinterpret_cast<uint4*>(p) = pack8(w);
  }
}

inline int grid_rows(int M, int C, int per_thread_rows = 4, int div = 8) {
  int C8 = C / 8;
  int R = 256 / C8;
  if (R < 1) R = 1;
  const long long full = ((long long)M + (long long)R * per_thread_rows - 1) / ((long long)R * per_thread_rows);
  // every workgroup first builds its BatchNorm tables (slot-summed statistics: dependent memory
  // round trips of a few us) and then grid-strides over rows: a grid sized for one pass of
  // per_thread_rows rows ran the prologue per ~64 rows (the stem max-pool backward: 2500
  // workgroups, 151 us).  Keep at most max(512, full/8) workgroups (>= 2 per CU).
  long long blocks = full < 512 ? full : (full + div - 1) / div > 512 ? (full + div - 1) / div : 512;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

// block-level: s_a/s_b partial sums -> global atomics
// this block's statistics slot copy of p (null stays null); stride between copies in floats
__device__ __forceinline__ float* slot_ptr(float* p, int slots, size_t stride) {
  return p ? p + (size_t)(blockIdx.x % stat_slots(slots)) * stride : nullptr;
}

__device__ __forceinline__ void flush_sums(float* s_a, float* s_b, int C, float* ga, float* gb) {
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    if (ga) atomicAdd(&ga[c], s_a[c]);
    if (gb) atomicAdd(&gb[c], s_b[c]);
  }
}

// per-channel block totals of ChunkMap-laid partials (common.h chunk_sums)
__device__ __forceinline__ void chunk_reduce(const ChunkMap& cm, int C, const float* pa, const float* pb,
                                             float* tmp, float* s_a, float* s_b) {
  chunk_sums(C, cm.R, cm.tx, cm.ty, pa, pb, tmp, s_a, s_b);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Bandwidth kernel: every thread owns one 8-channel chunk of RU rows per iteration and issues
// all of its loads before any arithmetic (RU independent 16-B loads in flight per operand), with
// the destination type / accumulate mode as template parameters so the loop is branch-free.
template <bool F32, bool ACC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdApplyArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(BnBwdApplyArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  constexpr int RU = 4;
  extern __shared__ float sh[];
  float* sA = sh;
  float* sB = sh + a.C;
  float* sC = sh + 2 * a.C;
  // one grid-stride pass of RU rows per thread is the common case (grid sized for it): issue that
  // pass's loads first so the coefficient loads below overlap them
  ChunkMap cm(a.C);
  const int c = cm.tx * 8;
  const int step = gridDim.x * cm.R;
  const int row0 = blockIdx.x * cm.R + cm.ty;
  uint4 dz[RU], xx[RU];
  float4 o0[RU], o1[RU];
  int rows[RU];
  auto load_pass = [&](int r0) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      int r = r0 + u * step;
      rows[u] = r < a.M ? r : a.M - 1;  // clamped: loads stay unconditional
      dz[u] = *reinterpret_cast<const uint4*>(a.dz + (size_t)rows[u] * a.lddz + c);
      xx[u] = *reinterpret_cast<const uint4*>(a.x + (size_t)rows[u] * a.ldx + c);
      if constexpr (F32 && ACC) {
        const float* q = reinterpret_cast<const float*>(a.dst) + (size_t)rows[u] * a.lddst + c;
        o0[u] = *reinterpret_cast<const float4*>(q);
        o1[u] = *reinterpret_cast<const float4*>(q + 4);
      }
    }
  };
  const bool active = cm.active();
  if (active && row0 < a.M) load_pass(row0);
  // coefficient table, up to 4 channels per thread per batch with every load of the batch issued
  // before any arithmetic (gamma is required: no per-element "pointer or 1" select, which makes
  // hipcc branch around each load and wait for it)
  const bool batch_mode = a.bn.mode == 1;
  const int SG = min(stat_slots(a.gsum_slots), MAX_STAT_SLOTS);
  const int SS = min(stat_slots(a.bn.slots), MAX_STAT_SLOTS);
  // single-copy statistics (small maps, many channels): 4 channels per thread per batch; slotted
  // ones (large maps, <= 512 channels): one channel per batch, its 2*(SS+SG) loads in flight
  const int per = (SG == 1 && SS == 1) ? 4 : 1;
  for (int base = 0; base < a.C; base += per * 256) {
    float m0[4], m1[4], g[4], q0[4], q1[4], k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= per) break;
      const int c = base + u * 256 + threadIdx.x;
      const int cc = c < a.C ? c : 0;
      g[u] = a.bn.gamma[cc];
      k[u] = batch_mode ? bn_shift(a.bn, cc) : 0.f;
      if (batch_mode) {
        if (SS == 1) {
          m0[u] = a.bn.stats[cc];
          m1[u] = a.bn.stats[a.bn.C + cc];
        } else {
          slot_sums_1(a.bn.stats, a.bn.stats + a.bn.C, SS, 2 * (size_t)a.bn.C, cc, m0[u], m1[u]);
        }
        if (SG == 1) {
          q0[u] = a.gsum[cc];
          q1[u] = a.gsumx[cc];
        } else {
          slot_sums_1(a.gsum, a.gsumx, SG, a.gsum_ld, cc, q0[u], q1[u]);
        }
      } else {
        m0[u] = a.bn.mmean[cc];
        m1[u] = a.bn.mvar[cc];
        q0[u] = q1[u] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = base + u * 256 + threadIdx.x;
      if (u >= per || c >= a.C) break;
      float mean = m0[u], var = m1[u];
      if (batch_mode) shifted_mean_var(k[u], m0[u], m1[u], a.bn.inv_count, mean, var);
      const float rstd = rsqrtf(var + a.bn.eps);
      if (blockIdx.x == 0 && a.fold_sum) {  // d beta / d gamma into the gradient arena
        a.fold_sum[c] += q0[u];
        a.fold_sumx[c] += q1[u];
      }
      const float sd = q0[u] * a.inv_n, sdx = q1[u] * a.inv_n;
      sA[c] = g[u] * rstd;
      sB[c] = -g[u] * rstd * rstd * sdx;
      sC[c] = -g[u] * rstd * sd + g[u] * rstd * rstd * mean * sdx;
    }
  }
  __syncthreads();
  if (!active) return;
  float ka[8], kb[8], kc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { ka[j] = sA[c + j]; kb[j] = sB[c + j]; kc[j] = sC[c + j]; }
  for (int row0_ = row0; row0_ < a.M; row0_ += step * RU) {
    if (row0_ != row0) load_pass(row0_);
    const int row0 = row0_;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (row0 + u * step >= a.M) break;
      float d[8], x[8], o[8];
      unpack8(dz[u], d);
      unpack8(xx[u], x);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = ka[j] * d[j] + kb[j] * x[j] + kc[j];
      if constexpr (F32) {
        float* q = reinterpret_cast<float*>(a.dst) + (size_t)rows[u] * a.lddst + c;
        if constexpr (ACC) {
          o[0] += o0[u].x; o[1] += o0[u].y; o[2] += o0[u].z; o[3] += o0[u].w;
          o[4] += o1[u].x; o[5] += o1[u].y; o[6] += o1[u].z; o[7] += o1[u].w;
        }
        *reinterpret_cast<float4*>(q) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(q + 4) = make_float4(o[4], o[5], o[6], o[7]);
      } else {
        bf16_t* q = reinterpret_cast<bf16_t*>(a.dst) + (size_t)rows[u] * a.lddst + c;
        if constexpr (ACC) {
          float p[8];
          unpack8(*reinterpret_cast<const uint4*>(q), p);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += p[j];
        }
        *reinterpret_cast<uint4*>(q) = pack8(o);
      }
    }
  }
}

hipError_t bn_bwd_apply(const BnBwdApplyArgs& a, hipStream_t st) {
  if (a.M == 0) return hipSuccess;
  if (a.bn.gamma == nullptr || (a.bn.mode == 1 && (a.gsum == nullptr || a.gsumx == nullptr)) ||
      (a.bn.mode == 2 && (a.bn.mmean == nullptr || a.bn.mvar == nullptr)) || (a.bn.mode != 1 && a.bn.mode != 2))
    return hipErrorInvalidValue;
  // ~1 iteration of RU rows per thread: enough blocks to fill all 256 CUs several times over
  dim3 grid(grid_rows(a.M, a.C, 4)), block(256);
  size_t shm = 3 * a.C * 4;
  if (a.dst_f32) {
    if (a.accumulate) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true>), ggrid(grid), block, shm, st, a, garg());
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false>), ggrid(grid), block, shm, st, a, garg());
  } else {
    if (a.accumulate) hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true>), ggrid(grid), block, shm, st, a, garg());
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false>), ggrid(grid), block, shm, st, a, garg());
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdReduceArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(BnBwdReduceArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sh = sh + a.C;
  float* s_mu = sh + 2 * a.C;
  float* s_rs = sh + 3 * a.C;
  float* s_a = sh + 4 * a.C;
  float* s_b = sh + 5 * a.C;
  float* s_tmp = sh + 6 * a.C;
  bn_full_table<256>(a.bn, a.C, s_sc, s_sh, s_mu, s_rs);
  __syncthreads();
  ChunkMap cm(a.C);
  float ps[8] = {0}, px[8] = {0};
  if (cm.active()) {
    const int c = cm.tx * 8;
    for (int row = blockIdx.x * cm.R + cm.ty; row < a.M; row += gridDim.x * cm.R) {
      float dy[8], x[8], d[8];
      load8(a.dy, a.dy_f32, (size_t)row * a.lddy + c, dy);
      unpack8(*reinterpret_cast<const uint4*>(a.x + (size_t)row * a.ldx + c), x);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = dy[j] * act_mask(x[j] * s_sc[c + j] + s_sh[c + j], a.bn.act);
      if (a.dz && a.dz_f32) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = s_sc[c + j] * d[j];
        float* q = reinterpret_cast<float*>(a.dz) + (size_t)row * a.lddz + c;
        *reinterpret_cast<float4*>(q) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(q + 4) = make_float4(o[4], o[5], o[6], o[7]);
      } else if (a.dz) {
        uint4 p = pack8(d);
        *reinterpret_cast<uint4*>(a.dz + (size_t)row * a.lddz + c) = p;
        unpack8(p, d);  // reduce exactly what was stored
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ps[j] += d[j];
        px[j] += d[j] * (x[j] - s_mu[c + j]) * s_rs[c + j];
      }
    }
  }
  chunk_reduce(cm, a.C, ps, px, s_tmp, s_a, s_b);
  flush_sums(s_a, s_b, a.C, slot_ptr(a.gsum, a.gsum_slots, a.gsum_ld), slot_ptr(a.gsumx, a.gsum_slots, a.gsum_ld));
}

hipError_t bn_bwd_reduce(const BnBwdReduceArgs& a, hipStream_t st) {
  if (a.M == 0) return hipSuccess;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, ggrid(dim3(grid_rows(a.M, a.C, 4))), dim3(256),
                     (6 * a.C + 2 * 256 * 8) * 4, st, a, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
template <bool IS_MAX, int K>
__global__ __launch_bounds__(256) void pool_fwd_kernel(PoolArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(PoolArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sh = sh + a.C;
  float* s_a = sh + 2 * a.C;
  float* s_b = sh + 3 * a.C;
  float* s_tmp = sh + 4 * a.C;
  bn_coeff_table<256>(a.pro, a.C, s_sc, s_sh);
  __syncthreads();
  ChunkMap cm(a.C);
  const int Mo = a.N * a.Ho * a.Wo;
  float ps[8] = {0}, pq[8] = {0};
  const bool ident = (a.pro.mode == 0 && a.pro.act == ACT_NONE);
  if (cm.active()) {
    const int c = cm.tx * 8;
    float kk[8];  // statistics shift of this thread's chunk
#pragma unroll
    for (int j = 0; j < 8; ++j) kk[j] = a.stats_shift ? a.stats_shift[c + j] : 0.f;
    for (int o = blockIdx.x * cm.R + cm.ty; o < Mo; o += gridDim.x * cm.R) {
      int wo = o % a.Wo, t = o / a.Wo, ho = t % a.Ho, n = t / a.Ho;
      float best[8], sum[8];
      uint8_t arg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -3.4e38f; sum[j] = 0.f; arg[j] = 0; }
      const int k = K > 0 ? K : a.k;
      // K > 0 (the model shapes: 3x3 stem max pool, 2x2 pools): every tap's load is issued before
      // any arithmetic — out-of-image taps load a clamped in-image pixel and are replaced by the
      // zero padding afterwards — instead of k*k dependent round trips; K == 0: runtime k
      constexpr int KK = K > 0 ? K * K : 1;
      uint4 raw[KK];
      if constexpr (K > 0) {
#pragma unroll
        for (int q = 0; q < KK; ++q) {
          const int h = min(max(ho * a.s - a.pt + q / K, 0), a.H - 1);
          const int w = min(max(wo * a.s - a.pl + q % K, 0), a.W - 1);
          raw[q] = *reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.ldx + c);
        }
      }
#pragma unroll
      for (int q = 0; q < (K > 0 ? KK : 1); ++q)
        for (int qq = (K > 0 ? q : 0); qq < (K > 0 ? q + 1 : k * k); ++qq) {
          const int r = qq / k, s2 = qq - r * k;
          const int h = ho * a.s - a.pt + r, w = wo * a.s - a.pl + s2;
          float v[8];
          if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
            if constexpr (K > 0) {
              unpack8(raw[q], v);
            } else {
              unpack8(*reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h) * a.W + w) * a.ldx + c), v);
            }
            if (!ident) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j] * s_sc[c + j] + s_sh[c + j], a.pro.act);
            }
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;  // Keras ZeroPadding before the pool
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (IS_MAX) {
              if (v[j] > best[j]) { best[j] = v[j]; arg[j] = (uint8_t)qq; }
            } else {
              sum[j] += v[j];
            }
          }
        }
      float out[8];
      const float inv = 1.f / (float)(k * k);
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = IS_MAX ? best[j] : sum[j] * inv;
      uint4 p = pack8(out);
      *reinterpret_cast<uint4*>(a.y + (size_t)o * a.ldy + c) = p;
      if (IS_MAX && a.argmax) {
        uint2 ar;
        ar.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
        ar.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
        *reinterpret_cast<uint2*>(a.argmax + (size_t)o * a.C + c) = ar;
      }
      if (a.stats) {
        unpack8(p, out);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dj = out[j] - kk[j];
          ps[j] += dj;
          pq[j] += dj * dj;
        }
      }
    }
  }
  if (a.stats) chunk_reduce(cm, a.C, ps, pq, s_tmp, s_a, s_b);
  if (a.stats)
    flush_sums(s_a, s_b, a.C, slot_ptr(a.stats, a.stats_slots, 2 * (size_t)a.stats_ld) + a.stats_off,
               slot_ptr(a.stats, a.stats_slots, 2 * (size_t)a.stats_ld) + a.stats_ld + a.stats_off);
}

// grid divisor of the pool kernels (grid_rows): IDC_POOL_GRID_DIV, default 8
static int pool_grid_div() {
  static const int d = [] {
    const char* e = std::getenv("IDC_POOL_GRID_DIV");
    const int v = e ? std::atoi(e) : 8;
    return v >= 1 ? v : 8;
  }();
  return d;
}

template <bool IS_MAX>
static hipError_t pool_fwd(const PoolArgs& a, hipStream_t st) {
  // one output row per thread per pass: the k*k taps already give k*k loads in flight
  const dim3 grid(grid_rows(a.N * a.Ho * a.Wo, a.C, 1, pool_grid_div())), block(256);
  const size_t shm = (4 * a.C + 2 * 256 * 8) * 4;
  if (a.k == 3) hipLaunchKernelGGL((pool_fwd_kernel<IS_MAX, 3>), ggrid(grid), block, shm, st, a, garg());
  else if (a.k == 2) hipLaunchKernelGGL((pool_fwd_kernel<IS_MAX, 2>), ggrid(grid), block, shm, st, a, garg());
  else hipLaunchKernelGGL((pool_fwd_kernel<IS_MAX, 0>), ggrid(grid), block, shm, st, a, garg());
  return hipGetLastError();
}

hipError_t maxpool_fwd(const PoolArgs& a, hipStream_t st) {
  if (maxpool_img_fwd_ok(a)) return maxpool_img_fwd(a, st);
  return pool_fwd<true>(a, st);
}

hipError_t avgpool_fwd(const PoolArgs& a, hipStream_t st) { return pool_fwd<false>(a, st); }

// Gather-form pool backward: each input element collects from the windows that contain it, then
// (optionally) the backward of the pending BN+act that fed the pool: dZ = g * act'(bn(x)) and the
// BN-backward sums.  WIN = windows covering an input pixel per spatial dim (1 when k <= s, 2 when
// k <= 2s): the window loop is unrolled and predicated, and each thread issues the loads of RU
// rows (every window's dy / argmax, and x) before any arithmetic.
template <int WIN, int RU>
__global__ __launch_bounds__(256) void pool_bwd_kernel(PoolBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(PoolBwdArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sh = sh + a.C;
  float* s_mu = sh + 2 * a.C;
  float* s_rs = sh + 3 * a.C;
  float* s_a = sh + 4 * a.C;
  float* s_b = sh + 5 * a.C;
  float* s_da = sh + 6 * a.C;  // dyaff coefficients
  float* s_db = sh + 7 * a.C;
  float* s_dc = sh + 8 * a.C;
  float* s_tmp = sh + 9 * a.C;
  const bool epi = (a.bn.mode != 0 || a.bn.act != ACT_NONE);
  const bool sums = epi && (a.gsum || a.gsumx);
  const bool dyaff = a.dyaff.mode != 0;
  if (epi) bn_full_table<256>(a.bn, a.C, s_sc, s_sh, s_mu, s_rs);
  if (dyaff) {
    bwd_aff_table<256>(a.dyaff, 0, a.C, a.C, s_da, s_db, s_dc);
    bwd_aff_fold<256>(a.dyaff);
  }
  __syncthreads();
  ChunkMap cm(a.C);
  const int Mi = a.N * a.H * a.W;
  float ps[8] = {0, 0, 0, 0, 0, 0, 0, 0}, px[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const float lo = act_lo(a.bn.act), hi = act_hi(a.bn.act);
  if (cm.active()) {
    const int c = cm.tx * 8;
    const float inv = 1.f / (float)(a.k * a.k);
    const int step = gridDim.x * cm.R;
    for (int i0 = blockIdx.x * cm.R + cm.ty; i0 < Mi; i0 += step * RU) {
      float d[RU][WIN * WIN][8];
      uint2 am[RU][WIN * WIN];
      bool ok[RU][WIN * WIN];
      uint8_t mine[RU][WIN * WIN];
      uint4 xr[RU];
      int rows[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int i = i0 + u * step;
        rows[u] = i < Mi ? i : Mi - 1;
        const int ii = rows[u];
        const int w = ii % a.W, t = ii / a.W, h = t % a.H, n = t / a.H;
        // windows oh with oh*s - pt <= h <= oh*s - pt + k - 1
        int oh_lo = h + a.pt - a.k + 1 + a.s - 1;
        oh_lo = oh_lo < 0 ? 0 : oh_lo / a.s;
        int oh_hi = (h + a.pt) / a.s;
        int ow_lo = w + a.pl - a.k + 1 + a.s - 1;
        ow_lo = ow_lo < 0 ? 0 : ow_lo / a.s;
        int ow_hi = (w + a.pl) / a.s;
        oh_hi = oh_hi < a.Ho - 1 ? oh_hi : a.Ho - 1;
        ow_hi = ow_hi < a.Wo - 1 ? ow_hi : a.Wo - 1;
#pragma unroll
        for (int dh = 0; dh < WIN; ++dh)
#pragma unroll
          for (int dw = 0; dw < WIN; ++dw) {
            const int q = dh * WIN + dw;
            const int oh = oh_lo + dh, ow = ow_lo + dw;
            const bool v = (i < Mi) && oh <= oh_hi && ow <= ow_hi;
            ok[u][q] = v;
            const size_t o = v ? (size_t)(n * a.Ho + oh) * a.Wo + ow : 0;
            load8(a.dy, a.dy_f32, o * a.lddy + c, d[u][q]);
            if (dyaff) {
              float xo[8];
              unpack8(*reinterpret_cast<const uint4*>(a.dyaff.x + o * a.dyaff.ldx + c), xo);
              bwd_aff8(d[u][q], xo, s_da + c, s_db + c, s_dc + c);
            }
            if (!a.is_avg) {
              am[u][q] = *reinterpret_cast<const uint2*>(a.argmax + o * a.C + c);
              mine[u][q] = (uint8_t)((h - (oh * a.s - a.pt)) * a.k + (w - (ow * a.s - a.pl)));
            }
          }
        if (epi) xr[u] = *reinterpret_cast<const uint4*>(a.x + (size_t)rows[u] * a.ldx + c);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        if (i0 + u * step >= Mi) break;
        float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < WIN * WIN; ++q) {
          if (!ok[u][q]) continue;
          if (a.is_avg) {
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] += d[u][q][j] * inv;
          } else {
            const uint2 ar = am[u][q];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t word = j < 4 ? ar.x : ar.y;
              const uint8_t b = (uint8_t)(word >> (8 * (j & 3)));
              g[j] += (b == mine[u][q]) ? d[u][q][j] : 0.f;
            }
          }
        }
        bf16_t* dst = a.dx + (size_t)rows[u] * a.lddx + c;
        if (epi && a.dx_f32) {
          float x[8], o[8];
          unpack8(xr[u], x);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = x[j] * s_sc[c + j] + s_sh[c + j];
            g[j] = (z > lo && z < hi) ? g[j] : 0.f;
            o[j] = s_sc[c + j] * g[j];
            ps[j] += g[j];
            px[j] += g[j] * (x[j] - s_mu[c + j]) * s_rs[c + j];
          }
          float* q = reinterpret_cast<float*>(a.dx) + (size_t)rows[u] * a.lddx + c;
          *reinterpret_cast<float4*>(q) = make_float4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<float4*>(q + 4) = make_float4(o[4], o[5], o[6], o[7]);
        } else if (epi) {
          float x[8];
          unpack8(xr[u], x);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float z = x[j] * s_sc[c + j] + s_sh[c + j];
            g[j] = (z > lo && z < hi) ? g[j] : 0.f;
          }
          const uint4 p = pack8(g);
          *reinterpret_cast<uint4*>(dst) = p;
          if (sums) {
            unpack8(p, g);  // reduce exactly what was stored
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              ps[j] += g[j];
              px[j] += g[j] * (x[j] - s_mu[c + j]) * s_rs[c + j];
            }
          }
        } else {
          *reinterpret_cast<uint4*>(dst) = pack8(g);
        }
      }
    }
  }
  if (sums) {
    chunk_reduce(cm, a.C, ps, px, s_tmp, s_a, s_b);
    flush_sums(s_a, s_b, a.C, slot_ptr(a.gsum, a.gsum_slots, a.gsum_ld),
               slot_ptr(a.gsumx, a.gsum_slots, a.gsum_ld));
  }
}

// Scatter-form backward of a NON-overlapping pool (k == s, no padding): one thread per (pooled
// pixel, 8-channel chunk) reads dy (and the argmax bytes) ONCE and writes the k x k window's
// chunks; the gather form re-reads them for every input pixel (k^2 times).  Input rows / columns
// past the last window (floor pooling, 25 -> 12) are written as zero gradients by the threads of
// the last window row / column.  EPI: the backward of the pending BN+act that fed the pool, per
// input pixel (dZ = g * act'(bn(x)), sums of dZ and dZ*xhat, fp32 gamma*rstd*dZ or bf16 dZ),
// exactly as the gather form.  Used for the VGG16 max pools (no epilogue) and the DenseNet
// transition average pools (BN epilogue, fp32 concat-gradient output).
template <bool AVG, bool EPI, int K>
__global__ __launch_bounds__(256) void pool_bwd_scatter_kernel(PoolBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(PoolBwdArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sh = sh + a.C;
  float* s_mu = sh + 2 * a.C;
  float* s_rs = sh + 3 * a.C;
  float* s_a = sh + 4 * a.C;
  float* s_b = sh + 5 * a.C;
  float* s_tmp = sh + 9 * a.C;
  if constexpr (EPI) {
    bn_full_table<256>(a.bn, a.C, s_sc, s_sh, s_mu, s_rs);
    __syncthreads();
  }
  const bool sums = EPI && (a.gsum || a.gsumx);
  ChunkMap cm(a.C);
  const int k = K > 0 ? K : a.k;
  const float inv = 1.f / (float)(k * k);
  const float lo = act_lo(a.bn.act), hi = act_hi(a.bn.act);
  const long long Np = (long long)a.N * a.Ho * a.Wo;
  float ps[8] = {0, 0, 0, 0, 0, 0, 0, 0}, px[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // K > 0: the window is unrolled and every load of it (dy, argmax, the k*k x chunks) is issued
  // before any arithmetic -- one memory round trip per window instead of k*k dependent ones (the
  // runtime-bounded loop waited for each x load in turn: the DenseNet transition pools ran at
  // ~1.5 TB/s, 30 us each)
  constexpr int KK = K > 0 ? K * K : 1;
  if (cm.active()) {
    const int c = cm.tx * 8;
    for (long long pp = (long long)blockIdx.x * cm.R + cm.ty; pp < Np; pp += (long long)gridDim.x * cm.R) {
      const int wo = (int)(pp % a.Wo);
      const long long t = pp / a.Wo;
      const int ho = (int)(t % a.Ho);
      const int n = (int)(t / a.Ho);
      const int h0 = ho * k, w0 = wo * k;
      float d[8];
      load8(a.dy, a.dy_f32, (size_t)pp * a.lddy + c, d);
      uint2 am = make_uint2(0, 0);
      if constexpr (!AVG) am = *reinterpret_cast<const uint2*>(a.argmax + (size_t)pp * a.C + c);
      uint4 xr[KK];
      if constexpr (EPI && K > 0) {
#pragma unroll
        for (int q = 0; q < KK; ++q)
          xr[q] = *reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + h0 + q / K) * a.W + w0 + q % K) * a.ldx + c);
      }
      // the window's k x k pixels
#pragma unroll
      for (int q = 0; q < (K > 0 ? KK : 1); ++q)
        for (int qq = (K > 0 ? q : 0); qq < (K > 0 ? q + 1 : k * k); ++qq) {
          const int dh = qq / k, dw = qq - dh * k;
          const size_t pix = (size_t)(n * a.H + h0 + dh) * a.W + w0 + dw;
          float g[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if constexpr (AVG) {
              g[j] = d[j] * inv;
            } else {
              const uint32_t word = j < 4 ? am.x : am.y;
              g[j] = (uint8_t)(word >> (8 * (j & 3))) == (uint8_t)qq ? d[j] : 0.f;
            }
          }
          if constexpr (EPI) {
            float x[8];
            if constexpr (K > 0) unpack8(xr[q], x);
            else unpack8(*reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c), x);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float z = x[j] * s_sc[c + j] + s_sh[c + j];
              g[j] = (z > lo && z < hi) ? g[j] : 0.f;
            }
            if (a.dx_f32) {
              float o[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                o[j] = s_sc[c + j] * g[j];
                ps[j] += g[j];
                px[j] += g[j] * (x[j] - s_mu[c + j]) * s_rs[c + j];
              }
              float* o4 = reinterpret_cast<float*>(a.dx) + pix * a.lddx + c;
              *reinterpret_cast<float4*>(o4) = make_float4(o[0], o[1], o[2], o[3]);
              *reinterpret_cast<float4*>(o4 + 4) = make_float4(o[4], o[5], o[6], o[7]);
            } else {
              const uint4 pk = pack8(g);
              *reinterpret_cast<uint4*>(a.dx + pix * a.lddx + c) = pk;
              unpack8(pk, g);  // reduce exactly what was stored
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                ps[j] += g[j];
                px[j] += g[j] * (x[j] - s_mu[c + j]) * s_rs[c + j];
              }
            }
          } else {
            *reinterpret_cast<uint4*>(a.dx + pix * a.lddx + c) = pack8(g);
          }
        }
      // input rows / columns past the last window (floor pooling, 13 -> 6) get zero gradients
      // from the threads of the last window row / column: no loads (a zero gradient adds nothing
      // to the BatchNorm sums, and gamma*rstd*0 = 0 in the fp32 form)
      if (ho == a.Ho - 1 || wo == a.Wo - 1) {
        const int h1 = ho == a.Ho - 1 ? a.H : h0 + k;
        const int w1 = wo == a.Wo - 1 ? a.W : w0 + k;
        for (int h = h0; h < h1; ++h)
          for (int w = w0; w < w1; ++w) {
            if (h < h0 + k && w < w0 + k) continue;
            const size_t pix = (size_t)(n * a.H + h) * a.W + w;
            if (EPI && a.dx_f32) {
              float* o4 = reinterpret_cast<float*>(a.dx) + pix * a.lddx + c;
              *reinterpret_cast<float4*>(o4) = make_float4(0.f, 0.f, 0.f, 0.f);
              *reinterpret_cast<float4*>(o4 + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
              *reinterpret_cast<uint4*>(a.dx + pix * a.lddx + c) = make_uint4(0u, 0u, 0u, 0u);
            }
          }
      }
    }
  }
  if (sums) {
    chunk_reduce(cm, a.C, ps, px, s_tmp, s_a, s_b);
    flush_sums(s_a, s_b, a.C, slot_ptr(a.gsum, a.gsum_slots, a.gsum_ld),
               slot_ptr(a.gsumx, a.gsum_slots, a.gsum_ld));
  }
}

// the scatter form applies: k == s without padding, no dy affine, whole windows inside the image,
// a channel count whose 8-chunks tile the 256-thread block (ChunkMap), and — with BN sums — the
// normal statistics slots (the deterministic mode sizes one private slot per gather workgroup)
static bool pool_bwd_scatter_ok(const PoolBwdArgs& a) {
  static const bool on = [] {
    const char* e = std::getenv("IDC_POOL_SCATTER");
    return !(e && e[0] == '0');
  }();
  const bool epi = a.bn.mode != 0 || a.bn.act != ACT_NONE;
  const int C8 = a.C / 8;
  return on && a.k == a.s && a.pt == 0 && a.pl == 0 && a.dyaff.mode == 0 && (a.C % 8) == 0 && C8 <= 256 &&
         (256 % C8) == 0 && (a.lddx % 8) == 0 && (a.lddy % 8) == 0 && (!epi || (a.ldx % 8) == 0) &&
         a.Ho * a.k <= a.H && a.Wo * a.k <= a.W && a.k * a.k <= 255 && (a.dx_f32 ? epi : true) &&
         (!epi || !(a.gsum || a.gsumx) || a.gsum_slots <= MAX_STAT_SLOTS);
}

hipError_t pool_bwd(const PoolBwdArgs& a, hipStream_t st) {
  if (a.dx_f32 && !(a.bn.mode != 0 || a.bn.act != ACT_NONE)) return hipErrorInvalidValue;
  if (pool_bwd_scatter_ok(a)) {
    const long long Np = (long long)a.N * a.Ho * a.Wo;
    const int R = 256 / (a.C / 8);
    long long blocks = (Np + R - 1) / R;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) return hipSuccess;
    const bool epi = a.bn.mode != 0 || a.bn.act != ACT_NONE;
    const size_t shm_s = epi ? (9 * (size_t)a.C + 2 * 256 * 8) * 4 : 0;
#define IDC_PS(AV, EP)                                                                                      \
  if (a.k == 2)                                                                                             \
    hipLaunchKernelGGL((pool_bwd_scatter_kernel<AV, EP, 2>), ggrid((int)blocks), dim3(256), shm_s, st, a, garg()); \
  else                                                                                                      \
    hipLaunchKernelGGL((pool_bwd_scatter_kernel<AV, EP, 0>), ggrid((int)blocks), dim3(256), shm_s, st, a, garg());
    if (a.is_avg) {
      if (epi) { IDC_PS(true, true) } else { IDC_PS(true, false) }
    } else {
      if (epi) { IDC_PS(false, true) } else { IDC_PS(false, false) }
    }
#undef IDC_PS
    return hipGetLastError();
  }
  if (a.dyaff.mode != 0 && (a.dyaff.x == nullptr || (a.dyaff.ldx % 8))) return hipErrorInvalidValue;
  if (maxpool_img_bwd_ok(a)) return maxpool_img_bwd(a, st);
  const size_t shm = (9 * a.C + 2 * 256 * 8) * 4;
  const int M = a.N * a.H * a.W;
  if (a.k <= a.s) {
    hipLaunchKernelGGL((pool_bwd_kernel<1, 4>), ggrid(dim3(grid_rows(M, a.C, 4, pool_grid_div()))), dim3(256), shm, st, a, garg());
  } else if (a.k <= 2 * a.s) {
    hipLaunchKernelGGL((pool_bwd_kernel<2, 2>), ggrid(dim3(grid_rows(M, a.C, 2, pool_grid_div()))), dim3(256), shm, st, a, garg());
  } else {
    return hipErrorInvalidValue;  // windows overlapping more than 2 per dim: not used by any model
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ void bn_update_moving_kernel(const BnMovingDesc* d, int n, GroupArg ga) {
  const long long go = goff(ga);
  BnMovingDesc b = gsh(d, go)[blockIdx.y];
  gshift(b, go);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < b.C; c += gridDim.x * blockDim.x) {
    float s0 = 0.f, s1 = 0.f;
    for (int s = 0; s < stat_slots(b.slots); ++s) {
      s0 += b.stats[(size_t)s * 2 * b.ld + c];
      s1 += b.stats[(size_t)s * 2 * b.ld + b.ld + c];
    }
    float mean, var;
    shifted_mean_var(b.shift ? b.shift[c] : 0.f, s0, s1, b.inv_count, mean, var);
    var *= b.unbias;
    b.mmean[c] = b.momentum * b.mmean[c] + (1.f - b.momentum) * mean;
    b.mvar[c] = b.momentum * b.mvar[c] + (1.f - b.momentum) * var;
  }
}

// after the backward: every statistics array's shift becomes this step's batch mean (the next
// step's producers accumulate around it, common.h "Shifted statistics")
__global__ void stats_shift_kernel(const ShiftDesc* d, int n, GroupArg ga) {
  const long long go = goff(ga);
  ShiftDesc b = gsh(d, go)[blockIdx.y];
  gshift(b, go);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < b.ld; c += gridDim.x * blockDim.x) {
    float s0 = 0.f;
    for (int s = 0; s < stat_slots(b.slots); ++s) s0 += b.stats[(size_t)s * 2 * b.ld + c];
    // a non-finite batch (a step the non-finite guard skips) keeps the old shift
    const float k = b.shift[c] + s0 * b.inv_count;
    if (isfinite(k)) b.shift[c] = k;
  }
}

hipError_t stats_shift(const ShiftDesc* d, int n, int maxC, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(stats_shift_kernel, ggrid(dim3((maxC + 255) / 256, n)), dim3(256), 0, st, d, n, garg());
  return hipGetLastError();
}

hipError_t bn_update_moving(const BnMovingDesc* d, int n, int maxC, hipStream_t st) {
  if (n == 0) return hipSuccess;
  dim3 grid((maxC + 255) / 256, n);
  hipLaunchKernelGGL(bn_update_moving_kernel, ggrid(grid), dim3(256), 0, st, d, n, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// head forward: one block per sample
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(HeadArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ float sh[];
  float* s_feat = sh;            // [C]
  float* s_red = sh + a.C;       // [U][4 waves]
  const int n = blockIdx.x;
  const bool ident = (a.pro.mode == 0 && a.pro.act == ACT_NONE);
  const float inv_hw = 1.f / (float)a.HW;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float sc = 1.f, sf = 0.f;
    if (!ident) bn_coeffs(a.pro, c, sc, sf);
    float acc = 0.f;
    for (int p = 0; p < a.HW; ++p) {
      float v = bf2f(a.x[((size_t)n * a.HW + p) * a.ldx + c]);
      if (!ident) v = apply_act(v * sc + sf, a.pro.act);
      acc += v;
    }
    acc *= inv_hw;
    s_feat[c] = acc;
    a.feats[(size_t)n * a.C + c] = acc;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int u = 0; u < a.U; ++u) {
    float p = 0.f;
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) p += s_feat[c] * a.w[(size_t)c * a.U + u];
    p = wave_sum(p);
    if (lane == 0) s_red[u * 4 + wid] = p;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float lg[32];
    for (int u = 0; u < a.U; ++u) {
      lg[u] = s_red[u * 4] + s_red[u * 4 + 1] + s_red[u * 4 + 2] + s_red[u * 4 + 3] + (a.b ? a.b[u] : 0.f);
      a.logits[n * a.U + u] = lg[u];
    }
    if (a.training || a.loss) {
      float loss = 0.f;
      if (a.U == 1) {
        float x = lg[0], z = a.labels[n];
        loss = fmaxf(x, 0.f) - x * z + log1pf(expf(-fabsf(x)));
        float sig = 1.f / (1.f + expf(-x));
        if (a.dlogits) a.dlogits[n] = (sig - z) * a.dl_scale;
      } else {
        float mx = lg[0];
        for (int u = 1; u < a.U; ++u) mx = fmaxf(mx, lg[u]);
        float se = 0.f;
        for (int u = 0; u < a.U; ++u) se += expf(lg[u] - mx);
        float lse = mx + logf(se);
        float tsum = 0.f;
        for (int u = 0; u < a.U; ++u) tsum += a.labels[n * a.U + u];
        for (int u = 0; u < a.U; ++u) {
          float y = a.labels[n * a.U + u];
          loss += -y * (lg[u] - lse);
          if (a.dlogits) a.dlogits[n * a.U + u] = (expf(lg[u] - lse) * tsum - y) * a.dl_scale;
        }
      }
      if (a.loss && a.loss_vec) {
        // agent-scope store of this sample's loss, then one arrival; the block that completes the
        // step's N arrivals sums them (agent-scope loads: other XCDs' L2s) in a fixed order
        idc::persist::st_coh(a.loss_vec + n, loss);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = (t + 1u) % (unsigned)a.N == 0u;
        // the last arrival re-arms the ticket for the next launch (every arrival of this one is
        // in), so the count never depends on N dividing 2^32 or on earlier launches completing
        if (last) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_red[4 * a.U] = last ? 1.f : 0.f;
      } else if (a.loss) {
        atomicAdd(a.loss, loss * a.loss_scale);
      }
    }
  }
  if (!(a.loss && a.loss_vec && (a.training || a.loss))) return;
  __syncthreads();
  float* s_fin = s_red + 4 * a.U;  // [flag, 4 wave partials] (launch reserves 8 floats)
  if (s_fin[0] == 0.f) return;     // block-uniform: not the last arrival
  float v = 0.f;
  for (int i = threadIdx.x; i < a.N; i += blockDim.x) v += idc::persist::ld_coh(a.loss_vec + i);
  v = wave_sum(v);
  if (lane == 0) s_fin[1 + wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) *a.loss = (s_fin[1] + s_fin[2] + s_fin[3] + s_fin[4]) * a.loss_scale;
}

hipError_t head_fwd(const HeadArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(head_fwd_kernel, ggrid(a.N), dim3(256), (a.C + 4 * a.U + 8) * 4, st, a, garg());
  return hipGetLastError();
}

// head backward on a 2-D grid: blockIdx.x = 64-channel slice, blockIdx.y = chunk of HB samples.
// Each of the 4 waves owns HB/4 samples of the chunk; dW partials are reduced over the waves in
// LDS and added once per (channel, unit) per chunk; dA = (dlogits . W^T) / HW is broadcast over
// the pixels with 4 loads/stores in flight per lane.  (One block per channel slice — the old
// form — left 16 blocks looping over all 256 samples: ~50 us for a 1 us job.)
template <int HB>
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(HeadBwdArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  __shared__ float s_dw[4][64][17];
  __shared__ float s_dl[HB][16];
  const int c0 = blockIdx.x * 64;
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = c0 + cl;
  const bool cok = c < a.C;
  float wc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) wc[u] = (cok && u < a.U) ? a.w[(size_t)c * a.U + u] : 0.f;
  float acc[16], accb = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = 0.f;
  const float inv_hw = 1.f / (float)a.HW;
  constexpr int PER = HB / 4;
  // chunks of HB samples, strided over gridDim.y (gridDim.y == 1 in the deterministic mode: every
  // dW / db element then receives exactly one add)
  for (int n0 = blockIdx.y * HB; n0 < a.N; n0 += gridDim.y * HB) {
    __syncthreads();  // s_dl of the previous chunk fully consumed
    for (int i = threadIdx.x; i < HB * a.U; i += blockDim.x) {
      const int n = n0 + i / a.U;
      s_dl[i / a.U][i % a.U] = n < a.N ? a.dlogits[n * a.U + i % a.U] : 0.f;
    }
    __syncthreads();
    float f[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int n = n0 + grp * PER + k;
      f[k] = (cok && n < a.N) ? a.feats[(size_t)n * a.C + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int nl = grp * PER + k, n = n0 + nl;
      float df = 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float dl = u < a.U ? s_dl[nl][u] : 0.f;
        acc[u] += f[k] * dl;
        df += dl * wc[u];
      }
      if (a.dA && cok && n < a.N) {
        const float v = df * inv_hw;
        float* dst = a.dA + (size_t)n * a.HW * a.ldda + c;
        for (int p = 0; p < a.HW; ++p) dst[(size_t)p * a.ldda] = v;
      }
    }
    if (blockIdx.x == 0 && threadIdx.x < a.U)
      for (int k = 0; k < HB; ++k) accb += s_dl[k][threadIdx.x];
  }
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (u < a.U) s_dw[grp][cl][u] = acc[u];
  __syncthreads();
  if (grp == 0 && cok)
    for (int u = 0; u < a.U; ++u)
      atomicAdd(&a.dw[(size_t)c * a.U + u], s_dw[0][cl][u] + s_dw[1][cl][u] + s_dw[2][cl][u] + s_dw[3][cl][u]);
  if (blockIdx.x == 0 && threadIdx.x < a.U && a.db) atomicAdd(&a.db[threadIdx.x], accb);
}

hipError_t head_bwd(const HeadBwdArgs& a, hipStream_t st) {
  if (a.U > 16) return hipErrorInvalidValue;
  constexpr int HB = 16;
  dim3 grid((a.C + 63) / 64, a.det ? 1 : (a.N + HB - 1) / HB);
  hipLaunchKernelGGL(head_bwd_kernel<HB>, ggrid(grid), dim3(256), 0, st, a, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rmsprop_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                      float* __restrict__ ms, long long n4, float lr,
                                                      float rho, float eps, float gs,
                                                      const int* __restrict__ skip, int* hostflag,
                                                      GroupArg ga) {
  {
    const long long go = goff(ga);
    w = gsh(w, go); g = gsh(g, go); ms = gsh(ms, go); skip = gsh(skip, go);
  }
  if (skip && *skip) {  // non-finite gradients / a persistent give-up: weights and slots unchanged
    // a give-up on ANY rank (bits above bit 0 of the all-reduced guard word) also raises this
    // rank's pinned host flag, so every replica's runtime applies the same IDC_DS_ON_FAIL policy
    // at the same step (program.py check_persistent), not only the rank whose launch gave up
    if (hostflag && (*skip & ~1) && blockIdx.x == 0 && threadIdx.x == 0)
      __hip_atomic_store(hostflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(ms)[i];
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float gg[4] = {gv.x * gs, gv.y * gs, gv.z * gs, gv.w * gs};
    float mm[4] = {mv.x, mv.y, mv.z, mv.w};
    float ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mm[j] = rho * mm[j] + (1.f - rho) * gg[j] * gg[j];
      ww[j] -= lr * gg[j] / (sqrtf(mm[j]) + eps);
    }
    reinterpret_cast<float4*>(ms)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    reinterpret_cast<float4*>(w)[i] = make_float4(ww[0], ww[1], ww[2], ww[3]);
  }
}

// zero fill as a plain kernel: keeps graph segments free of memset nodes and lets the fill
// overlap with nothing but its own stream order (16-B stores for the aligned body)
__global__ __launch_bounds__(256) void zero_fill_kernel(unsigned char* __restrict__ p, long long nbytes, GroupArg ga) {
  p = gsh(p, goff(ga));
  const long long n16 = nbytes >> 4;
  uint4* q = reinterpret_cast<uint4*>(p);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    q[i] = make_uint4(0u, 0u, 0u, 0u);
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (nbytes & 15)) p[(n16 << 4) + t] = 0;
}

hipError_t zero_fill(void* p, long long nbytes, hipStream_t st) {
  if (nbytes <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(p) & 15) return hipErrorInvalidValue;
  long long blocks = ((nbytes >> 4) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(zero_fill_kernel, ggrid((int)blocks), dim3(256), 0, st,
                     reinterpret_cast<unsigned char*>(p), nbytes, garg());
  return hipGetLastError();
}

// any non-finite value in g[0:n) -> *flag = 1 (the flag is cleared at the start of backward)
__global__ __launch_bounds__(256) void finite_check_kernel(const float* __restrict__ g, long long n4,
                                                           int* __restrict__ flag, GroupArg ga) {
  g = gsh(g, goff(ga));
  flag = gsh(flag, goff(ga));
  int bad = 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(g)[i];
    bad |= !isfinite(v.x) | !isfinite(v.y) | !isfinite(v.z) | !isfinite(v.w);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

hipError_t finite_check(const float* g, long long n, int* flag, hipStream_t st) {
  long long n4 = n / 4;
  long long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(finite_check_kernel, ggrid((int)blocks), dim3(256), 0, st, g, n4, flag, garg());
  return hipGetLastError();
}

__global__ void finite_flag_reset_kernel(int* flag, int* status, GroupArg ga) {
  flag = gsh(flag, goff(ga));
  status = gsh(status, goff(ga));
  // flag bit 0: non-finite gradients; bit 1: a persistent launch gave up (persist.h note_fail);
  // summed over data-parallel ranks by the step-guard all-reduce, so any non-zero value skips
  status[0] = flag[0];
  status[1] += flag[0] != 0;  // running count of skipped steps
  flag[0] = 0;
}

hipError_t finite_flag_reset(int* flag, int* status, hipStream_t st) {
  hipLaunchKernelGGL(finite_flag_reset_kernel, ggrid(1), dim3(1), 0, st, flag, status, garg());
  return hipGetLastError();
}

hipError_t rmsprop(float* w, const float* g, float* ms, long long n, float lr, float rho, float eps,
                   float grad_scale, const int* skip, int* hostflag, hipStream_t st) {
  long long n4 = n / 4;  // arena sizes are multiples of 64 elements
  long long blocks = (n4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(rmsprop_kernel, ggrid((int)blocks), dim3(256), 0, st, w, g, ms, n4, lr, rho, eps,
                     grad_scale, skip, hostflag, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// fp32 Keras HWIO masters -> bf16 kernel layouts, as a tiled transpose.  A kernel is the
// row-major matrix src[R = KH*KW*Cin][Cout]; one block moves one 64x64 tile of it:
//   dgrad [Cin][KH][KW][Cout] (spatially flipped): rows stay rows -> written straight from the
//         coalesced loads (Cout contiguous on both sides);
//   fwd   [Cout][KH][KW][Cpad]: the transpose -> staged through LDS, written K-contiguous.
// Blocks map to (entry, tile) through a host-built tile -> entry table (`begin` = the entry's
// first tile), so there is no per-element search and every global access is coalesced.
__global__ __launch_bounds__(256) void cast_weights_kernel(const CastEntry* __restrict__ es,
                                                           const int* __restrict__ tile_entry,
                                                           long long ntiles, GroupArg ga) {
  __shared__ float tile[64][65];
  const long long go = goff(ga);
  es = gsh(es, go);
  tile_entry = gsh(tile_entry, go);
  for (long long b = blockIdx.x; b < ntiles; b += gridDim.x) {
    CastEntry e = es[tile_entry[b]];
    gshift(e, go);
    const int R = e.KH * e.KW * e.Cin;
    const int tiles_c = (e.Cout + 63) / 64;
    const long long lt = b - e.begin;
    const int r0 = (int)(lt / tiles_c) * 64, c0 = (int)(lt % tiles_c) * 64;
    const int col = c0 + (threadIdx.x & 15) * 4;
    const bool vec = (e.Cout & 3) == 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rl = (threadIdx.x >> 4) + 16 * k, r = r0 + rl;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        const float* src = e.src + (size_t)r * e.Cout;
        if (vec && col + 3 < e.Cout) {
          const float4 q = *reinterpret_cast<const float4*>(src + col);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = col + j < e.Cout ? src[col + j] : 0.f;
        }
        if (e.dgrad) {
          // src row r = (ri, si, ci) -> dgrad row (ci, KH-1-ri, KW-1-si)
          const int ci = r % e.Cin, rs = r / e.Cin, si = rs % e.KW, ri = rs / e.KW;
          bf16_t* dst = e.dgrad + (((size_t)ci * e.KH + (e.KH - 1 - ri)) * e.KW + (e.KW - 1 - si)) * e.Cout;
          if (vec && col + 3 < e.Cout) {
            *reinterpret_cast<uint2*>(dst + col) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
          } else {
            for (int j = 0; j < 4; ++j)
              if (col + j < e.Cout) dst[col + j] = f2bf(v[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[rl][(threadIdx.x & 15) * 4 + j] = v[j];
    }
    __syncthreads();
    // fwd: 64 output channels x 64 K rows; consecutive lanes write consecutive K positions
    const int ldd = e.KH * e.KW * e.Cpad;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int cl = idx >> 6, rl = idx & 63;
      const int co = c0 + cl, r = r0 + rl;
      if (co < e.Cout && r < R) {
        const int ci = r % e.Cin, rs = r / e.Cin;
        e.fwd[(size_t)co * ldd + (size_t)rs * e.Cpad + ci] = f2bf(tile[rl][cl]);
      }
    }
    __syncthreads();
  }
}

hipError_t cast_weights(const CastEntry* d_entries, const int* tile_entry, long long ntiles, hipStream_t st) {
  if (d_entries == nullptr || ntiles == 0) return hipSuccess;
  long long blocks = ntiles < 8192 ? ntiles : 8192;
  hipLaunchKernelGGL(cast_weights_kernel, ggrid((int)blocks), dim3(256), 0, st, d_entries, tile_entry, ntiles, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Input staging, the first op of every training / inference step: uint8 (x/255) or fp32 NHWC
// pixels -> bf16 [.., Cpad] operand, and (lab_code != 0) the labels -> fp32 head labels in the same
// launch (the caller's own tensors are read directly: no staging copies before the step).
// lab_code: 1 fp32, 2 int64, 3 int32, 4 uint8; U == 1: out[i] = y[i]; U > 1: integer class ids
// become one-hot rows, fp32 input is an [N, U] matrix copied as is.
__device__ __forceinline__ float load_label(const void* y, int code, long long i) {
  switch (code) {
    case 1: return reinterpret_cast<const float*>(y)[i];
    case 2: return (float)reinterpret_cast<const long long*>(y)[i];
    case 3: return (float)reinterpret_cast<const int*>(y)[i];
    default: return (float)reinterpret_cast<const uint8_t*>(y)[i];
  }
}

__global__ __launch_bounds__(256) void input_stage_kernel(const void* x, int u8, long long npix, int C,
                                                          bf16_t* y, int Cpad, const void* lab, int lab_code,
                                                          int N, int U, float* lab_out, GroupArg ga) {
  x = gsh(x, goff(ga));
  y = gsh(y, goff(ga));
  // labels read in place: in a grouped program they live in the region like x (client batching
  // stages each client's epoch in its own copy); goff is 0 otherwise
  lab = gsh(lab, goff(ga));
  const long long tid0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long nthr = (long long)gridDim.x * blockDim.x;
  for (long long p = tid0; p < npix; p += nthr) {
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < C && c < 8; ++c) {
      v[c] = u8 ? (float)reinterpret_cast<const uint8_t*>(x)[p * C + c] * (1.f / 255.f)
                : reinterpret_cast<const float*>(x)[p * C + c];
    }
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      uint4 q = c0 == 0 ? pack8(v) : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(y + p * Cpad + c0) = q;
    }
  }
  if (lab_code) {
    lab_out = gsh(lab_out, goff(ga));
    const long long nl = (long long)N * U;
    for (long long q = tid0; q < nl; q += nthr) {
      float o;
      if (U == 1 || lab_code == 1) {
        o = load_label(lab, lab_code, q);
      } else {
        const long long i = q / U;
        o = (long long)load_label(lab, lab_code, i) == q - i * U ? 1.f : 0.f;
      }
      lab_out[q] = o;
    }
  }
}

hipError_t input_stage(const void* x, int x_u8, int N, int H, int W, int C, bf16_t* y, int Cpad,
                       const void* lab, int lab_code, int U, float* lab_out, hipStream_t st) {
  if (lab_code && (lab == nullptr || lab_out == nullptr || U < 1 || lab_code > 4)) return hipErrorInvalidValue;
  long long npix = (long long)N * H * W;
  long long blocks = (npix + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(input_stage_kernel, ggrid((int)blocks), dim3(256), 0, st, x, x_u8, npix, C, y, Cpad, lab,
                     lab_code, N, U, lab_out, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Per-copy training metrics of a grouped (client-batched) step: workgroup g reads copy g of the
// program's loss [1], logits [B] and labels [B] (copy 0 + g * stride bytes) and adds the loss and
// the number of correct predictions (logit > thr vs label > 0.5) into acc[2g], acc[2g + 1].  One
// launch per step instead of torch ops over [K]-views of the region, which TensorIterator splits
// per copy (the views span more than 2^31 bytes).
__global__ __launch_bounds__(64) void group_metrics_kernel(const float* loss, const float* logits,
                                                           const float* labels, long long stride, int B,
                                                           float thr, double* acc) {
  const int g = blockIdx.x;
  const long long off = (long long)g * stride;
  const float* lg = reinterpret_cast<const float*>(reinterpret_cast<const char*>(logits) + off);
  const float* lb = reinterpret_cast<const float*>(reinterpret_cast<const char*>(labels) + off);
  int c = 0;
  for (int i = threadIdx.x; i < B; i += 64) c += ((lg[i] > thr) == (lb[i] > 0.5f)) ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (threadIdx.x == 0) {
    const float l = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(loss) + off);
    acc[2 * g] += (double)l;
    acc[2 * g + 1] += (double)c;
  }
}

hipError_t group_metrics(const float* loss, const float* logits, const float* labels, long long stride, int K,
                         int B, float thr, double* acc, hipStream_t st) {
  if (K < 1 || B < 1 || !loss || !logits || !labels || !acc) return hipErrorInvalidValue;
  hipLaunchKernelGGL(group_metrics_kernel, dim3(K), dim3(64), 0, st, loss, logits, labels, stride, B, thr, acc);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* x, int ldx, int M, int C,
                                                       float* stats, int stats_ld, int stats_off,
                                                       int stats_slots, GroupArg ga) {
  x = gsh(x, goff(ga));
  stats = gsh(stats, goff(ga));
  extern __shared__ float sh[];
  float* s_a = sh;
  float* s_b = sh + C;
  float* s_tmp = sh + 2 * C;
  ChunkMap cm(C);
  float ps[8] = {0}, pq[8] = {0};
  if (cm.active()) {
    const int c = cm.tx * 8;
    for (int row = blockIdx.x * cm.R + cm.ty; row < M; row += gridDim.x * cm.R) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)row * ldx + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { ps[j] += v[j]; pq[j] += v[j] * v[j]; }
    }
  }
  chunk_reduce(cm, C, ps, pq, s_tmp, s_a, s_b);
  float* so = slot_ptr(stats, stats_slots, 2 * (size_t)stats_ld);
  flush_sums(s_a, s_b, C, so + stats_off, so + stats_ld + stats_off);
}

hipError_t bn_stats(const bf16_t* x, int ldx, int M, int C, float* stats, int stats_ld, int stats_off,
                    int stats_slots, hipStream_t st) {
  hipLaunchKernelGGL(bn_stats_kernel, ggrid(dim3(grid_rows(M, C, 16))), dim3(256), (2 * C + 2 * 256 * 8) * 4, st, x, ldx, M, C,
                     stats, stats_ld, stats_off, stats_slots, garg());
  return hipGetLastError();
}

// y = act(bn(x)) [+ res]; optional stats of y  (MobileNetV2 block outputs, eval paths)
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* x, int ldx, BnArgs bn, const bf16_t* res,
                                                       int ldres, bf16_t* y, int ldy, int M, int C,
                                                       float* stats, int stats_ld, int stats_slots, GroupArg ga) {
  {
    const long long go = goff(ga);
    x = gsh(x, go); gshift(bn, go); res = gsh(res, go); y = gsh(y, go); stats = gsh(stats, go);
  }
  extern __shared__ float sh[];
  float* s_sc = sh;
  float* s_sh = sh + C;
  float* s_a = sh + 2 * C;
  float* s_b = sh + 3 * C;
  float* s_tmp = sh + 4 * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) bn_coeffs(bn, c, s_sc[c], s_sh[c]);
  __syncthreads();
  ChunkMap cm(C);
  float ps[8] = {0}, pq[8] = {0};
  if (cm.active()) {
    const int c = cm.tx * 8;
    for (int row = blockIdx.x * cm.R + cm.ty; row < M; row += gridDim.x * cm.R) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)row * ldx + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j] * s_sc[c + j] + s_sh[c + j], bn.act);
      if (res) {
        float r[8];
        unpack8(*reinterpret_cast<const uint4*>(res + (size_t)row * ldres + c), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += r[j];
      }
      uint4 p = pack8(v);
      *reinterpret_cast<uint4*>(y + (size_t)row * ldy + c) = p;
      if (stats) {
        unpack8(p, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) { ps[j] += v[j]; pq[j] += v[j] * v[j]; }
      }
    }
  }
  if (stats) {
    chunk_reduce(cm, C, ps, pq, s_tmp, s_a, s_b);
    float* so = slot_ptr(stats, stats_slots, 2 * (size_t)stats_ld);
    flush_sums(s_a, s_b, C, so, so + stats_ld);
  }
}

hipError_t bn_apply(const bf16_t* x, int ldx, BnArgs bn, const bf16_t* res, int ldres, bf16_t* y, int ldy,
                    int M, int C, float* stats, int stats_ld, int stats_slots, hipStream_t st) {
  hipLaunchKernelGGL(bn_apply_kernel, ggrid(dim3(grid_rows(M, C))), dim3(256), (4 * C + 2 * 256 * 8) * 4, st, x, ldx, bn, res, ldres,
                     y, ldy, M, C, stats, stats_ld, stats_slots, garg());
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Fixed-order slot reduction: a block owns 32 channels; thread (ty, tx) sums slots ty, ty+8, ...
// of channel tx, then the 8 partials are added in ty order — the same bits every run (the
// deterministic mode folds every producer's per-workgroup slots through here).
__global__ __launch_bounds__(256) void slot_collapse_kernel(const float* src, float* dst, const float* src2,
                                                            float* dst2, int slots, int ld, int C, GroupArg ga) {
  {
    const long long go = goff(ga);
    src = gsh(src, go); dst = gsh(dst, go); src2 = gsh(src2, go); dst2 = gsh(dst2, go);
  }
  __shared__ float sa[8][33], sb[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  float a = 0.f, b = 0.f;
  if (c < C) {
    for (int s = ty; s < slots; s += 8) {
      a += src[(size_t)s * ld + c];
      if (src2) b += src2[(size_t)s * ld + c];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
    float ta = 0.f, tb = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ta += sa[k][tx];
      tb += sb[k][tx];
    }
    dst[c] += ta;
    if (dst2) dst2[c] += tb;
  }
}

hipError_t slot_collapse(const float* src, float* dst, const float* src2, float* dst2, int slots, int ld,
                         int C, hipStream_t st) {
  if (C <= 0) return hipSuccess;
  if (src == nullptr || dst == nullptr || (src2 == nullptr) != (dst2 == nullptr) || slots < 1 || ld < C)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(slot_collapse_kernel, ggrid(dim3((C + 31) / 32)), dim3(256), 0, st, src, dst, src2, dst2, slots,
                     ld, C, garg());
  return hipGetLastError();
}

int rows_grid(int M, int C, int per_thread_rows) { return grid_rows(M, C, per_thread_rows); }
int pool_rows_grid(int M, int C, int per_thread_rows) { return grid_rows(M, C, per_thread_rows, pool_grid_div()); }

}  // namespace idc
