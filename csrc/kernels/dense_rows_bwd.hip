// Row-resident dense-stage BACKWARD for DenseNet (gfx950): the data gradients of every dense layer
// of a late stage in ONE launch in which each workgroup OWNS whole images for the whole stage --
// the backward counterpart of dense_rows.hip, same interface as dense_stage_bwd.hip (DenseBwdArgs).
//
// Reference: the DenseNet fits of /root/reference/dist_model_tf_dense.py:147-150,168-172 (Keras
// DenseNet201; the north-star benchmark trains DenseNet-121).  With the notation of
// dense_stage_bwd.hip (layer l: x = buf[:, :cin_l], t = W1 relu(bn1_l(x)), y = W2 * relu(bn2_l(t))):
//
//   workgroup g keeps, for ITS rows only and for the whole launch, the forward stage rows x (bf16)
//   and the fp32 concat gradient dX (entering as A_f dZ_f of the consumer BatchNorm) in LDS, and
//   the per-channel summed pending affines Btot / Ctot (identical in every workgroup).  For
//   l = L-1 .. 0:
//     dy   = dX[:, slice l] + Btot x + Ctot      (slice l is final: every later layer is done)
//     dA2  = W2^T * dy  (3x3, image-local)        -> dZ2 = dA2 relu'(bn2(t)), bn2 reductions
//     ---- barrier A (bn2 reductions summed over every workgroup) ----
//     dT   = A2 dZ2 + B2 t + C2                   -> dT  (the cv1 weight-gradient operand)
//     dA1  = dT W1^T  (1x1, cin_l channels)       -> dX[:, :cin_l] += A1 relu'(bn1(x)) dA1,
//                                                    bn1 reductions
//     ---- barrier B (bn1 reductions) ----         -> Btot / Ctot += B1 / C1, d gamma / d beta
//   then dx16 = bf16(dX[:, :c0] + Btot x + Ctot) for the transition / stem.
// Only the BatchNorm reductions cross workgroups (statistics slots + sharded arrival counters,
// persist.h); the data never leaves the workgroup (dy -> dO16 and dT -> dt are stored for the
// side-lane weight gradients only).  All workgroups must be co-resident (the launcher checks).
#include "dense_stage.h"
#include "persist.h"

namespace idc {
namespace {

using namespace persist;

constexpr int NTB = 512;      // 8 waves
constexpr int RR = 16;        // rows per workgroup (one 16-row MFMA block)
constexpr int TPB = 128 + 8;  // t / dT row pitch (bf16)
constexpr int DYP = 32 + 8;   // dy row pitch (bf16)
constexpr int S = DS_SLOTS;
constexpr int MAXCB = 8;      // 1x1 dgrad column blocks per wave (cin <= 8 x 8 x 16 = 1024)

struct BwdLayout {
  int xs, dx, tb, dy, dt, mean, var, bt, ct, p0, p1, tab2, lay, total;
};

__host__ __device__ inline BwdLayout bwd_layout(int ld, int nlayers) {
  BwdLayout L{};
  int o = 0;
  L.xs = o;
  o += RR * (ld + 8) * 2;
  L.dx = o;
  o += RR * (ld + 4) * 4;
  L.tb = o;
  o += RR * TPB * 2;
  L.dy = o;
  o += (RR + 1) * DYP * 2;
  o = (o + 15) & ~15;
  L.dt = o;
  o += RR * TPB * 2;
  L.mean = o;
  o += ld * 4;
  L.var = o;
  o += ld * 4;
  L.bt = o;
  o += ld * 4;
  L.ct = o;
  o += ld * 4;
  L.p0 = o;  // this workgroup's not-yet-reduced bn1 backward terms per channel (C part, B part)
  o += ld * 4;
  L.p1 = o;
  o += ld * 4;
  L.tab2 = o;  // sc2, sh2, mean2, rstd2, A2, B2, C2 of the current layer [7][128]
  o += 7 * 128 * 4;
  L.lay = o;
  o += nlayers * (int)sizeof(DenseBwdLayerDesc);
  L.total = o;
  return L;
}

constexpr int LDS_MAX_B = 160 * 1024;

// (B, C) of a training-mode BatchNorm from its reductions (q0 = sum dZ, q1 = sum dZ xhat)
__device__ __forceinline__ void bc_of(float g, float mean, float rstd, float q0, float q1, float inv_n, float& B,
                                      float& C) {
  B = -g * rstd * rstd * (q1 * inv_n);
  C = -g * rstd * (q0 * inv_n) - B * mean;
}

// (B, C) of the stage's consumer BatchNorm for channel c (its reductions precede the launch)
__device__ __forceinline__ void pend_bc_of(const BwdAff& pend, int c, float& B, float& C) {
  B = 0.f;
  C = 0.f;
  if (pend.mode == 0 || pend.bn.mode != 1) return;
  const int SS = min(stat_slots(pend.bn.slots), MAX_STAT_SLOTS);
  const int SG = min(stat_slots(pend.gsum_slots), MAX_STAT_SLOTS);
  float m0, m1, q0, q1, mean, var;
  slot_sums_1(pend.bn.stats, pend.bn.stats + pend.bn.C, SS, 2 * (size_t)pend.bn.C, c, m0, m1);
  slot_sums_1(pend.gsum, pend.gsumx, SG, (size_t)pend.gsum_ld, c, q0, q1);
  shifted_mean_var(bn_shift(pend.bn, c), m0, m1, pend.bn.inv_count, mean, var);
  bc_of(pend.bn.gamma ? pend.bn.gamma[c] : 1.f, mean, rsqrtf(var + pend.bn.eps), q0, q1, pend.inv_n, B, C);
}

// sum over the 4 lane groups of a wave (rows (lane >> 4) * 4 + q of an MFMA output block)
__device__ __forceinline__ float colsum16(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

}  // namespace

__global__ __launch_bounds__(NTB) void dense_rows_bwd_kernel(DenseBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(DenseBwdArgs) + sizeof(GroupArg)>();
  const long long go = goff(ga);
  const bf16_t* __restrict__ buf = gsh(a.buf, go);
  const float* __restrict__ sstats = gsh(a.sstats, go);
  const float* __restrict__ sshift = gsh(a.sshift, go);
  const float* __restrict__ dbuf = gsh(a.dbuf, go);
  bf16_t* __restrict__ dx16 = gsh(a.dx16, go);
  const DenseBwdLayerDesc* __restrict__ layers = gsh(a.layers, go);
  unsigned* sync = gsh(a.sync, go);
  int* err = gsh(a.err, go);
  const persist::FailSink fsink{err, gsh(a.stepflag, go), a.hostflag};
  unsigned long long* stamps = gsh(a.stamps, go);  // [layer][group][NSTAMP] (diagnostics)
  const unsigned max_polls = a.max_polls ? a.max_polls : DEFAULT_POLLS;
  BwdAff pend = a.pend;
  gshift(pend, go);
  const int L = a.nlayers, ld = a.ld;
  // sync words (dense_stage.h dsb_sync_words): layer l's barrier A / B counters at lsync(l) and
  // lsync(l) + 8 (8 shards each), the fail flag last
  auto cntA = [&](int l) { return sync + 1 + DSB_SYNC_PER_LAYER * l; };
  auto cntB = [&](int l) { return sync + 9 + DSB_SYNC_PER_LAYER * l; };
  unsigned* fail = sync + dsb_sync_words(L) - 1;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const BwdLayout LY = bwd_layout(ld, L);
  const int ldp = ld + 8, ldf = ld + 4;
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem + LY.xs);
  float* dX = reinterpret_cast<float*>(smem + LY.dx);
  bf16_t* tb = reinterpret_cast<bf16_t*>(smem + LY.tb);
  bf16_t* dyb = reinterpret_cast<bf16_t*>(smem + LY.dy);
  bf16_t* dtb = reinterpret_cast<bf16_t*>(smem + LY.dt);
  float* s_mean = reinterpret_cast<float*>(smem + LY.mean);
  float* s_var = reinterpret_cast<float*>(smem + LY.var);
  float* s_bt = reinterpret_cast<float*>(smem + LY.bt);
  float* s_ct = reinterpret_cast<float*>(smem + LY.ct);
  float* s_p0 = reinterpret_cast<float*>(smem + LY.p0);
  float* s_p1 = reinterpret_cast<float*>(smem + LY.p1);
  float* t2 = reinterpret_cast<float*>(smem + LY.tab2);
  float *s_sc2 = t2, *s_sh2 = t2 + 128, *s_m2 = t2 + 256, *s_r2 = t2 + 384;
  float *s_A2 = t2 + 512, *s_B2 = t2 + 640, *s_C2 = t2 + 768;
  DenseBwdLayerDesc* s_lay = reinterpret_cast<DenseBwdLayerDesc*>(smem + LY.lay);
  __shared__ int s_bad;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = (lane >> 4) * 8, rq = (lane >> 4) * 4;
  const int HW = a.H * a.W, M = a.N * HW;
  const int G = (int)gridDim.x, gi = (int)blockIdx.x;
  const int row0 = gi * a.rows_ipg * HW;
  const int Rg = min(a.rows_ipg * HW, M - row0);
  const int c0 = a.c0;
  const float inv_n = a.inv_count;
  const float lo = act_lo(a.act), hi = act_hi(a.act);
  const int taps = a.k2 * a.k2, pad = a.k2 >> 1;

  // ---- the group's forward rows, entering concat gradient, moments, pending affines, layers
  {
    const int nw = L * (int)sizeof(DenseBwdLayerDesc) / 4;
    for (int i = tid; i < nw; i += NTB) reinterpret_cast<unsigned*>(s_lay)[i] = reinterpret_cast<const unsigned*>(layers)[i];
  }
  for (int idx = tid; idx < RR * (ld / 8); idx += NTB) {
    const int r = idx / (ld / 8), c = (idx - r * (ld / 8)) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    float4 d0 = make_float4(0.f, 0.f, 0.f, 0.f), d1 = d0;
    if (r < Rg) {
      v = *reinterpret_cast<const uint4*>(buf + (size_t)(row0 + r) * ld + c);
      d0 = *reinterpret_cast<const float4*>(dbuf + (size_t)(row0 + r) * ld + c);
      d1 = *reinterpret_cast<const float4*>(dbuf + (size_t)(row0 + r) * ld + c + 4);
    }
    *reinterpret_cast<uint4*>(xs + r * ldp + c) = v;
    *reinterpret_cast<float4*>(dX + r * ldf + c) = d0;
    *reinterpret_cast<float4*>(dX + r * ldf + c + 4) = d1;
  }
  for (int c = tid; c < ld; c += NTB) {
    float mean, var, B, C;
    shifted_mean_var(sshift ? sshift[c] : 0.f, sstats[c], sstats[ld + c], inv_n, mean, var);
    s_mean[c] = mean;
    s_var[c] = var;
    pend_bc_of(pend, c, B, C);
    s_bt[c] = B;
    s_ct[c] = C;
    s_p0[c] = 0.f;
    s_p1[c] = 0.f;
  }
  // per-workgroup bn1 reductions of every layer (for d beta / d gamma, summed by the finishing
  // kernel): [layer][group][2][cin_layer], layer l at G * 2 * (l c0 + 32 l (l - 1) / 2)
  float* rpart = gsh(a.rpart, go);
  if (tid < DYP / 2) reinterpret_cast<uint32_t*>(dyb + RR * DYP)[tid] = 0u;  // the zero row
  // image-local position of the lane's 3x3 A-fragment row
  int img_base = 0, ph = 0, pw = 0;
  {
    const int mm = fr < Rg ? fr : 0;
    const int img = mm / HW, rem = mm - img * HW;
    img_base = img * HW;
    ph = rem / a.W;
    pw = rem - ph * a.W;
  }

  for (int l = L - 1; l >= 0; --l) {
    __syncthreads();
    const int sti = l * G + gi;
    stamp(stamps, sti, 0);
    const DenseBwdLayerDesc d = s_lay[l];
    const int cin = d.cin;
    // ---- 3x3 weight fragments (this wave: dA2 channels 16 wid + fr), t rows, bn2 tables
    v8bf bq[9];
    {
      const bf16_t* w2d = gsh(d.w2d, go);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        bq[tap] = tap < taps ? *reinterpret_cast<const v8bf*>(w2d + ((size_t)(16 * wid + fr) * taps + tap) * 32 + fk)
                             : v8bf{};
    }
    if (tid < RR * 16) {
      const int r = tid >> 4, c = (tid & 15) * 8;
      const bf16_t* tg = gsh(d.t, go);
      *reinterpret_cast<uint4*>(tb + r * TPB + c) =
          r < Rg ? *reinterpret_cast<const uint4*>(tg + (size_t)(row0 + r) * 128 + c) : make_uint4(0, 0, 0, 0);
    } else if (tid < RR * 16 + 128) {
      const int c = tid - RR * 16;
      const float* ts = gsh(d.tstats, go);
      const float* tsh = gsh(d.tshift, go);
      float mean, var;
      shifted_mean_var(tsh ? tsh[c] : 0.f, ts[c], ts[128 + c], inv_n, mean, var);
      const float rstd = rsqrtf(var + d.eps2);
      const float sc = gsh(d.g2, go)[c] * rstd;
      s_sc2[c] = sc;
      s_sh2[c] = gsh(d.b2, go)[c] - mean * sc;
      s_m2[c] = mean;
      s_r2[c] = rstd;
    }
    // ---- dy = dX[:, slice l] + Btot x + Ctot (bf16): LDS and dO16
    if (tid < RR * 4) {
      const int r = tid >> 2, c8 = (tid & 3) * 8, c = cin + c8;
      float x[8], v[8];
      unpack8(*reinterpret_cast<const uint4*>(xs + r * ldp + c), x);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = r < Rg ? dX[r * ldf + c + q] + s_bt[c + q] * x[q] + s_ct[c + q] : 0.f;
      const uint4 pk = pack8(v);
      *reinterpret_cast<uint4*>(dyb + r * DYP + c8) = pk;
      if (r < Rg) *reinterpret_cast<uint4*>(gsh(d.dO16, go) + (size_t)(row0 + r) * 32 + c8) = pk;
    }
    __syncthreads();
    stamp(stamps, sti, 1);
    // ---- dA2 (3x3 dgrad) -> dZ2 and the bn2 reductions
    float dz2[4];
    const int c2 = 16 * wid + fr;
    {
      v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        if (tap < taps) {
          const int kr = tap / a.k2, kc = tap - kr * a.k2;
          const int hh = ph + kr - pad, ww = pw + kc - pad;
          const bool ok = fr < Rg && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
          const int lrow = ok ? img_base + hh * a.W + ww : RR;
          const v8bf af = *reinterpret_cast<const v8bf*>(dyb + lrow * DYP + fk);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[tap], acc, 0, 0, 0);
        }
      const float sc = s_sc2[c2], sh = s_sh2[c2], mu = s_m2[c2], rs = s_r2[c2];
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rq + q;
        const float t = bf2f(tb[r * TPB + c2]);
        const float z = sc * t + sh;
        dz2[q] = (r < Rg && z > lo && z < hi) ? acc[q] : 0.f;
        s0 += dz2[q];
        s1 += dz2[q] * (t - mu) * rs;
      }
      s0 = colsum16(s0);
      s1 = colsum16(s1);
      if (lane < 16) {
        float* r2 = gsh(d.r2, go) + (gi % S) * 256;
        atomicAdd(r2 + c2, s0);
        atomicAdd(r2 + 128 + c2, s1);
      }
    }
    stamp(stamps, sti, 2);
    publish_shard(cntA(l), gi);
    // 1x1 dgrad weight fragments (column blocks wid + 8 j) and bn1 parameters of those columns:
    // in flight while the barrier waits
    // (the first half of the column blocks; the second half is issued as the first is consumed)
    const int ncb = cin >> 4;
    const bf16_t* w1d = gsh(d.w1d, go);
    constexpr int HCB = MAXCB / 2;
    v8bf wq[HCB][4];
    float g1c[MAXCB], b1c[MAXCB];
    auto load_wq = [&](int j, v8bf (&q)[4]) {
      const int cb = wid + 8 * j;
      const bool ok = cb < ncb;
      const int c = ok ? 16 * cb + fr : 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = ok ? *reinterpret_cast<const v8bf*>(w1d + (size_t)c * 128 + k * 32 + fk) : v8bf{};
    };
    {
      const float* g1 = gsh(d.g1, go);
      const float* b1 = gsh(d.b1, go);
#pragma unroll
      for (int j = 0; j < HCB; ++j) load_wq(j, wq[j]);
#pragma unroll
      for (int j = 0; j < MAXCB; ++j) {
        const int cb = wid + 8 * j;
        const bool ok = cb < ncb;
        const int c = ok ? 16 * cb + fr : 0;
        g1c[j] = ok ? g1[c] : 0.f;
        b1c[j] = ok ? b1[c] : 0.f;
      }
    }
    if (wid == 0) {
      const bool ok = wait_sum8(cntA(l), (unsigned)G, fail, fsink, max_polls);
      if (lane == 0) s_bad = !ok;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(s_bad)) return;
    stamp(stamps, sti, 3);
    // ---- bn2 backward affine, dT
    if (tid < 128) {
      float q0, q1, B2, C2;
      slot_sum<S>(gsh(d.r2, go), 128, tid, q0, q1);
      const float g2 = gsh(d.g2, go)[tid];
      bc_of(g2, s_m2[tid], s_r2[tid], q0, q1, inv_n, B2, C2);
      s_A2[tid] = g2 * s_r2[tid];
      s_B2[tid] = B2;
      s_C2[tid] = C2;
      if (gi == 0) {
        gsh(d.dbeta2, go)[tid] = q0;
        gsh(d.dgamma2, go)[tid] = q1;
      }
    }
    __syncthreads();
    {
      const float A2 = s_A2[c2], B2 = s_B2[c2], C2 = s_C2[c2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rq + q;
        const float t = bf2f(tb[r * TPB + c2]);
        const float v = r < Rg ? A2 * dz2[q] + B2 * t + C2 : 0.f;
        dtb[r * TPB + c2] = (bf16_t)(pack2bf(v, 0.f) & 0xffffu);
      }
    }
    __syncthreads();
    if (tid < RR * 16) {  // dT for the cv1 weight gradient
      const int r = tid >> 4, c = (tid & 15) * 8;
      if (r < Rg)
        *reinterpret_cast<uint4*>(gsh(d.dt, go) + (size_t)(row0 + r) * 128 + c) =
            *reinterpret_cast<const uint4*>(dtb + r * TPB + c);
    }
    stamp(stamps, sti, 4);
    // ---- dA1 = dT W1^T over cin channels: dX += A1 dZ1, bn1 reductions
    {
      v8bf af[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) af[k] = *reinterpret_cast<const v8bf*>(dtb + fr * TPB + k * 32 + fk);
      float* rp = rpart + (size_t)G * 2 * (l * c0 + 16 * l * (l - 1)) + (size_t)gi * 2 * cin;
      const float kn = -inv_n;
#pragma unroll
      for (int j = 0; j < MAXCB; ++j) {
        const int cb = wid + 8 * j;
        if (cb < ncb) {
          v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], wq[j % HCB][k], acc, 0, 0, 0);
          if (j < HCB && wid + 8 * (j + HCB) < ncb) load_wq(j + HCB, wq[j % HCB]);
          const int c = 16 * cb + fr;
          const float mean = s_mean[c], rstd = rsqrtf(s_var[c] + d.eps1);
          const float sc = g1c[j] * rstd, sh = b1c[j] - mean * sc;
          float s0 = 0.f, s1 = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = rq + q;
            const float x = bf2f(xs[r * ldp + c]);
            const float z = sc * x + sh;
            const float dz = (r < Rg && z > lo && z < hi) ? acc[q] : 0.f;
            dX[r * ldf + c] += sc * dz;
            s0 += dz;
            s1 += dz * (x - mean) * rstd;
          }
          s0 = colsum16(s0);
          s1 = colsum16(s1);
          if (lane < 16) {
            // the channel's bn1 backward terms B = -g rstd^2 mean(dZ xhat), C = -g rstd mean(dZ)
            // - B mean are linear in the sums: accumulate this workgroup's share per channel and
            // reduce across workgroups only when the channel's slice is needed (deferred)
            s_p1[c] += kn * g1c[j] * rstd * rstd * s1;
            s_p0[c] += kn * g1c[j] * rstd * s0;
            rp[c] = s0;
            rp[cin + c] = s1;
          }
        }
      }
    }
    stamp(stamps, sti, 5);
    if (l > 0) {
      // ---- slice l-1 (channels [cin - 32, cin)) is the next dy: reduce its pending terms
      __syncthreads();  // s_p0 / s_p1 of the slice complete
      float* r1 = gsh(d.r1, go);  // [S][2][32]
      if (tid < 64) {
        const int c = cin - 32 + (tid & 31), which = tid >> 5;
        atomicAdd(r1 + (gi % S) * 64 + which * 32 + (tid & 31), which ? s_p1[c] : s_p0[c]);
      }
      publish_shard(cntB(l), gi);
      if (wid == 0) {
        const bool ok = wait_sum8(cntB(l), (unsigned)G, fail, fsink, max_polls);
        if (lane == 0) s_bad = !ok;
      }
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s_bad)) return;
      stamp(stamps, sti, 6);
      if (tid < 32) {
        const int c = cin - 32 + tid;
        float q0, q1;
        slot_sum<S>(r1, 32, tid, q0, q1);
        s_bt[c] += q1;
        s_ct[c] += q0 - s_mean[c] * q1;
      }
    }
    stamp(stamps, sti, 7);
  }
  __syncthreads();
  // ---- the stage input channels [0, c0): their pending terms reduced once (layer 0's slots)
  {
    float* r1 = gsh(s_lay[0].r1, go);  // [S][2][c0]
    for (int c = tid; c < c0; c += NTB) {
      atomicAdd(r1 + (gi % S) * 2 * c0 + c, s_p0[c]);
      atomicAdd(r1 + (gi % S) * 2 * c0 + c0 + c, s_p1[c]);
    }
    publish_shard(cntB(0), gi);
    if (wid == 0) {
      const bool ok = wait_sum8(cntB(0), (unsigned)G, fail, fsink, max_polls);
      if (lane == 0) s_bad = !ok;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(s_bad)) return;
    for (int c = tid; c < c0; c += NTB) {
      float q0, q1;
      slot_sum<S>(r1, c0, c, q0, q1);
      s_bt[c] += q1;
      s_ct[c] += q0 - s_mean[c] * q1;
    }
    __syncthreads();
  }
  // ---- the stage input's final gradient (bf16) for the transition / stem
  for (int idx = tid; idx < Rg * (c0 / 8); idx += NTB) {
    const int r = idx / (c0 / 8), c = (idx - r * (c0 / 8)) * 8;
    float x[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(xs + r * ldp + c), x);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = dX[r * ldf + c + q] + s_bt[c + q] * x[q] + s_ct[c + q];
    *reinterpret_cast<uint4*>(dx16 + (size_t)(row0 + r) * c0 + c) = pack8(v);
  }
}

// d beta / d gamma of every layer's bn1: the per-workgroup sums of dZ1 / dZ1 xhat over the groups
__global__ __launch_bounds__(256) void dense_rows_bwd_fin_kernel(DenseBwdArgs a, int G, GroupArg ga) {
  const long long go = goff(ga);
  const int l = blockIdx.y;
  const DenseBwdLayerDesc* layers = gsh(a.layers, go);
  const int cin = layers[l].cin;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cin) return;
  const float* rp = gsh(a.rpart, go) + (size_t)G * 2 * (l * a.c0 + 16 * l * (l - 1));
  float q0 = 0.f, q1 = 0.f;
  for (int g = 0; g < G; ++g) {
    q0 += rp[(size_t)g * 2 * cin + c];
    q1 += rp[(size_t)g * 2 * cin + cin + c];
  }
  gsh(layers[l].dbeta1, go)[c] = q0;
  gsh(layers[l].dgamma1, go)[c] = q1;
}

long long dense_rows_bwd_part_floats(int c0, int nlayers, int grid) {
  const long long L = nlayers;
  return (long long)grid * 2 * (L * c0 + 16 * L * (L - 1));
}

bool dense_rows_bwd_geometry(int N, int H, int W, int ld, int nlayers, int& ipg, int& grid) {
  const int HW = H * W;
  if (ld % 32 || ld - 32 > MAXCB * 8 * 16 || nlayers > 64) return false;
  const int ip = RR / HW;
  if (ip < 1 || bwd_layout(ld, nlayers).total > LDS_MAX_B) return false;
  const int g = (N + ip - 1) / ip;
  if (g > 256) return false;
  ipg = ip;
  grid = g;
  return true;
}

hipError_t dense_rows_bwd(const DenseBwdArgs& a, hipStream_t st) {
  int ipg = 0, grid = 0;
  if (!dense_rows_bwd_geometry(a.N, a.H, a.W, a.ld, a.nlayers, ipg, grid) || launch_groups().k > 1 ||
      (a.k2 != 1 && a.k2 != 3) || a.c0 % 32 || a.rpart == nullptr ||
      a.rpart_floats < dense_rows_bwd_part_floats(a.c0, a.nlayers, grid))
    return hipErrorInvalidValue;
  DenseBwdArgs b = a;
  b.rows_ipg = ipg;
  hipLaunchKernelGGL(dense_rows_bwd_kernel, ggrid(grid), dim3(NTB), bwd_layout(a.ld, a.nlayers).total, st, b,
                     garg());
  const int maxc = a.c0 + 32 * (a.nlayers - 1);
  hipLaunchKernelGGL(dense_rows_bwd_fin_kernel, ggrid(dim3((maxc + 255) / 256, a.nlayers)), dim3(256), 0, st, b,
                     grid, garg());
  return hipGetLastError();
}

}  // namespace idc
