// Persistent dense-stage BACKWARD for DenseNet (gfx950): the data gradients of every dense layer of
// one stage, their BatchNorm reductions and d gamma / d beta, in ONE launch.
//
// Forward of layer l (dense_stage.hip):  x = buf[:, :cin_l],  t = W1 . relu(bn1_l(x)),
// y = W2 * relu(bn2_l(t)) -> buf[:, cin_l : cin_l + 32) ("slice l").  Reference: the DenseNet fits of
// /root/reference/dist_model_tf_dense.py:147-150,168-172 (Keras Applications DenseNet201; the
// north-star benchmark trains DenseNet-121).
//
// The gradient of a stage-buffer channel c is the sum over every BatchNorm that normalises it (the
// bn1 of each later layer k, and the stage's consumer -- transition or final -- BatchNorm) of
//     A_k dZ_k + B_k x_c + C_k,    A_k = g_k rstd,  B_k = -g_k rstd^2 mean(dZ_k xhat),
//     C_k = -g_k rstd mean(dZ_k) - B_k mean        (common.h BwdAff)
// with dZ_k = relu'_k . (W1_k^T dT_k) restricted to c.  The B x + C parts are per-channel AFFINE
// terms of the same x, so they add up to ONE affine term per channel (btot).  Every term of slice s
// is only needed when the chain reaches P_s, so the older terms are GATHERED per slice instead of
// being scattered into the fp32 buffer layer after layer:
//
//   P_l   3x3 dgrad: dY = dbuf[:, slice l] + dnew_{l+1} + Btot x + Ctot (+ layer l+1's B, C), staged
//         bf16 (also stored as dO16 for the cv2 weight gradient); dA2 = W2^T * dY;
//         dZ2 = dA2 * relu'(bn2(t)) -> z2 and the bn2 reductions (slots).
//   QN_l  dT_l = A2 z2 + B2 t + C2 (stored as dt_l: weight-gradient and gather operand), then the
//         1x1 dgrad of ONLY the newest slice l-1 (the one P_{l-1} reads next) into dnew[l & 1], with
//         its bn1_l reductions.
//   G_s   the terms of layers k = s+2 .. L-1 for slice s (in chunks of DSB_KG layers per tile):
//         sum_k A_k relu'_k (dT_k W1_k[s]^T) added to dbuf[:, slice s] (float atomics), bn1_k
//         reductions for slice s; the last G_s tile turns all of slice s's reductions (and the
//         consumer BatchNorm's) into btot and writes d beta / d gamma of those bn1_k channels.
//   GIN / FIN1  the same for the stage input channels [0, c0): layers k >= 1 once QN_1 is done,
//         layer 0 once QN_0 is done (its last tile per 32-channel group finalises btot).
//   FIN2  dx16 = bf16(dbuf + Btot x + Ctot): the transition's / stem's operand.
// The dependent chain is P_l -> QN_l -> P_{l-1}; G_{l-2} starts after QN_l and has P_{l-1} and
// QN_{l-1} to finish before P_{l-2} needs it.
//
// Work queue (ticket order; every wait is on an EARLIER ticket, so no deadlock at any residency):
//   for l = L-1 .. 0: P_l, QN_l, G_{l-2} (l >= 2), GIN (l == 1);  then FIN1, FIN2.
// Hand-off primitives and memory model: persist.h.
#include "dense_stage.h"
#include "persist.h"

namespace idc {
namespace {

using namespace persist;

constexpr int NT = 256;
// a lane's 16 channels of a 128-channel row are two 8-channel pieces 64 apart: each wave-level
// access then covers 128 contiguous bytes of the 8-lane row group (16 consecutive channels per
// lane put the pieces at a 32-B stride: half-line accesses, 2-way LDS bank conflicts)
constexpr int ESEG2 = 64;
constexpr int S = DS_SLOTS;
constexpr int DPITCH = 32 + 8;  // staged dY rows (bf16)
constexpr int TP = 128 + 8;     // staged dT rows (bf16)
constexpr int RP = 129;         // fp32 [32][128] epilogue tile pitch
constexpr int OP = 65;          // fp32 [32][64] epilogue tile pitch

struct Smem {
  float tab[4][128];  // per-channel tables of the tile
  union {
    struct {
      bf16_t dy[(DS_MAX_STAGE_ROWS + 1) * DPITCH];  // + one all-zero row (3x3 padding taps)
      float r0[32 * RP];
      float r1[32 * RP];
    } p;
    struct {
      bf16_t dt[32 * TP];
      float r0[32 * OP];
      float part[2][4][64];
    } q;
    float fin[2][8][32];
  } u;
  float sB[64], sC[64];
  int task, bad, last, kind, layer, tile;
};

// forward BatchNorm moments of channel c from single-copy shifted statistics (pre-launch data)
__device__ __forceinline__ void fwd_moments(const float* st, int ld, const float* shift, int c, float inv_n,
                                            float eps, float& mean, float& rstd) {
  float var;
  shifted_mean_var(shift ? shift[c] : 0.f, st[c], st[ld + c], inv_n, mean, var);
  rstd = rsqrtf(var + eps);
}

// (B, C) of a training-mode BatchNorm from its reductions (q0 = sum dZ, q1 = sum dZ xhat)
__device__ __forceinline__ void bwd_bc(float g, float mean, float rstd, float q0, float q1, float inv_n, float& B,
                                       float& C) {
  B = -g * rstd * rstd * (q1 * inv_n);
  C = -g * rstd * (q0 * inv_n) - B * mean;
}

// (B, C) of the stage's consumer BatchNorm for channel c (its reductions precede the launch)
__device__ __forceinline__ void pend_bc(const BwdAff& pend, int c, float& B, float& C) {
  B = 0.f;
  C = 0.f;
  if (pend.mode == 0 || pend.bn.mode != 1) return;
  const int SS = min(stat_slots(pend.bn.slots), MAX_STAT_SLOTS);
  const int SG = min(stat_slots(pend.gsum_slots), MAX_STAT_SLOTS);
  float m0, m1, q0, q1, mean, var;
  slot_sums_1(pend.bn.stats, pend.bn.stats + pend.bn.C, SS, 2 * (size_t)pend.bn.C, c, m0, m1);
  slot_sums_1(pend.gsum, pend.gsumx, SG, (size_t)pend.gsum_ld, c, q0, q1);
  shifted_mean_var(bn_shift(pend.bn, c), m0, m1, pend.bn.inv_count, mean, var);
  bwd_bc(pend.bn.gamma ? pend.bn.gamma[c] : 1.f, mean, rsqrtf(var + pend.bn.eps), q0, q1, pend.inv_n, B, C);
}

__device__ __forceinline__ void unpack16(const uint4& a, const uint4& b, float* f) {
  unpack8(a, f);
  unpack8(b, f + 8);
}

}  // namespace

__global__ __launch_bounds__(NT) void dense_stage_bwd_kernel(DenseBwdArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(DenseBwdArgs) + sizeof(GroupArg)>();
  const long long go = goff(ga);
  const bf16_t* __restrict__ buf = gsh(a.buf, go);
  const float* __restrict__ sstats = gsh(a.sstats, go);
  const float* __restrict__ sshift = gsh(a.sshift, go);
  float* __restrict__ dbuf = gsh(a.dbuf, go);
  float* __restrict__ dnew = gsh(a.dnew, go);
  bf16_t* __restrict__ dx16 = gsh(a.dx16, go);
  bf16_t* __restrict__ z2 = gsh(a.z2, go);
  const DenseBwdLayerDesc* __restrict__ layers = gsh(a.layers, go);
  const DenseBwdPhase* __restrict__ phases = gsh(a.phases, go);
  unsigned* sync = gsh(a.sync, go);
  float* btot = gsh(a.btot, go);
  int* err = gsh(a.err, go);
  const persist::FailSink fsink{err, gsh(a.stepflag, go), a.hostflag};
  unsigned long long* stamps = gsh(a.stamps, go);
  const unsigned max_polls = a.max_polls ? a.max_polls : DEFAULT_POLLS;
  BwdAff pend = a.pend;
  gshift(pend, go);

  const int L = a.nlayers, ld = a.ld;
  // sync words (dense_stage.h dsb_sync_words)
  auto lsync = [&](int l) { return sync + 1 + DSB_SYNC_PER_LAYER * l; };  // P 8, QN 8, G arrivals, G done
  unsigned* gin_cnt = sync + 1 + DSB_SYNC_PER_LAYER * L;
  unsigned* f1_cnt = gin_cnt + 8;
  unsigned* f1_done = f1_cnt + DSB_MAX_CG;
  unsigned* f2_cnt = f1_done + 1;
  unsigned* fail = f2_cnt + 1;

  __shared__ __attribute__((aligned(16))) Smem s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int HW = a.H * a.W, M = a.N * HW;
  const int nmt = (M + 31) / 32;
  const int taps = a.k2 * a.k2, pad = a.k2 >> 1;
  const float lo = act_lo(a.act), hi = act_hi(a.act);
  const float inv_n = a.inv_count;
  const int ncg = a.c0 / 32;
  const int nkc_in = (L - 1 + DSB_KG - 1) / DSB_KG;  // GIN's layer chunks (layers 1 .. L-1)

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      const int task = (int)__hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s.task = task;
      if (task < a.ntickets) {  // the phase holding this ticket (binary search on first tickets)
        int lo_i = 0, hi_i = a.nphases - 1;
        while (lo_i < hi_i) {
          const int mid = (lo_i + hi_i + 1) >> 1;
          if (phases[mid].first <= task) lo_i = mid;
          else hi_i = mid - 1;
        }
        const DenseBwdPhase ph = phases[lo_i];
        s.kind = ph.kind;
        s.layer = ph.layer;
        s.tile = task - ph.first;
      }
    }
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(s.task);
    if (task >= a.ntickets) return;
    stamp(stamps, task, 0);
    const int kind = __builtin_amdgcn_readfirstlane(s.kind);
    const int l = __builtin_amdgcn_readfirstlane(s.layer);
    const int tile = __builtin_amdgcn_readfirstlane(s.tile);

    // one wait of thread 0 (plain counter) or of wave 0 (8-shard counter), broadcast; a failed
    // wait ends the workgroup
#define DSB_WAIT(cnt, need)                                                                   \
  do {                                                                                        \
    if (tid == 0) s.bad = !wait_count((cnt), (unsigned)(need), fail, fsink, max_polls);         \
    __syncthreads();                                                                          \
    if (__builtin_amdgcn_readfirstlane(s.bad)) return;                                       \
  } while (0)
#define DSB_WAIT8(cnt, need)                                                                  \
  do {                                                                                        \
    if (wid == 0) {                                                                           \
      const bool ok_ = wait_sum8((cnt), (unsigned)(need), fail, fsink, max_polls);              \
      if (lane == 0) s.bad = !ok_;                                                            \
    }                                                                                         \
    __syncthreads();                                                                          \
    if (__builtin_amdgcn_readfirstlane(s.bad)) return;                                       \
  } while (0)

    if (kind == DSB_P) {
      // ================================================================ P_l: 3x3 dgrad of cv2
      const DenseBwdLayerDesc d = layers[l];
      const int cin = d.cin;
      const int j = tile, m0 = j * 32;
      const bf16_t* __restrict__ w2d = gsh(d.w2d, go);
      const bf16_t* __restrict__ tb = gsh(d.t, go);
      // weight fragments: wave w owns input channels [32w, 32w + 32) of cv2
      v8bf bq[9][2];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int ci = wid * 32 + jj * 16 + fr;
          bq[tap][jj] = tap < taps ? *reinterpret_cast<const v8bf*>(w2d + ((size_t)ci * taps + tap) * 32 + fk) : v8bf{};
        }
      // bn2 forward tables (pre-launch data) and the epilogue's t rows
      if (tid < 128) {
        float mean, rstd;
        fwd_moments(gsh(d.tstats, go), 128, gsh(d.tshift, go), tid, inv_n, d.eps2, mean, rstd);
        const float sc = gsh(d.g2, go)[tid] * rstd;
        s.tab[0][tid] = sc;
        s.tab[1][tid] = gsh(d.b2, go)[tid] - mean * sc;
        s.tab[2][tid] = mean;
        s.tab[3][tid] = rstd;
      }
      const int er = tid >> 3, eseg = (tid & 7) * 8, em = m0 + er;  // pieces eseg, eseg + 64 (ESEG2)
      uint4 tv0 = make_uint4(0, 0, 0, 0), tv1 = tv0;
      if (em < M) {
        tv0 = *reinterpret_cast<const uint4*>(tb + (size_t)em * 128 + eseg);
        tv1 = *reinterpret_cast<const uint4*>(tb + (size_t)em * 128 + eseg + ESEG2);
      }
      const int mend = min(m0 + 32, M);
      const int img_lo = m0 / HW, img_hi = (mend - 1) / HW;
      const int row_lo = img_lo * HW, R = (img_hi - img_lo + 1) * HW;
      int aoff[2][9];  // LDS offsets of this lane's A fragments per tap (padding: the zero row)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = m0 + h * 16 + fr;
        const int mm = m < M ? m : M - 1;
        const int img = mm / HW, rem = mm - img * HW;
        const int ph = rem / a.W, pw = rem - ph * a.W;
        const int ibase = img * HW - row_lo;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int kr = tap / a.k2, kc = tap - kr * a.k2;
          const int hh = ph + kr - pad, ww = pw + kc - pad;
          const bool ok = tap < taps && m < M && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
          aoff[h][tap] = (ok ? ibase + hh * a.W + ww : DS_MAX_STAGE_ROWS) * DPITCH + fk;
        }
      }
      // slice l is final once QN_{l+1} (its newest-slice term) and G_l (the terms of layers >= l+2,
      // gathered and summed into btot by G_l's last tile) are complete
      if (l < L - 1) DSB_WAIT8(lsync(l + 1) + 8, nmt);
      if (l <= L - 3) DSB_WAIT(lsync(l) + 17, 1);
      stamp(stamps, task, 1);
      const float* dn = dnew + (size_t)((l + 1) & 1) * M * 32;
      // staged rows: R x 32 channels, 8 channels per chunk, <= 2 chunks per thread
      constexpr int CU = DS_MAX_STAGE_ROWS * 4 / NT;
      float4 dv[CU][2], nv[CU][2];
      uint4 xv[CU];
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int idx = tid + u * NT;
        const int row = row_lo + (idx >> 2), c8 = (idx & 3) * 8;
        const bool ok = idx < R * 4;
        const float* dp = dbuf + (size_t)row * ld + cin + c8;
        dv[u][0] = ok ? ld_coh_f4(dp) : make_float4(0.f, 0.f, 0.f, 0.f);
        dv[u][1] = ok ? ld_coh_f4(dp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool okn = ok && l < L - 1;
        nv[u][0] = okn ? ld_coh_f4(dn + (size_t)row * 32 + c8) : make_float4(0.f, 0.f, 0.f, 0.f);
        nv[u][1] = okn ? ld_coh_f4(dn + (size_t)row * 32 + c8 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        xv[u] = ok ? *reinterpret_cast<const uint4*>(buf + (size_t)row * ld + cin + c8) : make_uint4(0, 0, 0, 0);
      }
      if (tid < 32) {
        // slice channel c: btot + the newest contribution (bn1 of layer l+1, from its slots)
        const int c = cin + tid;
        float B, C;
        if (l <= L - 3) {
          B = ld_coh(btot + c);
          C = ld_coh(btot + ld + c);
        } else {
          pend_bc(pend, c, B, C);
        }
        if (l < L - 1) {
          const DenseBwdLayerDesc dn1 = layers[l + 1];
          float q0, q1, mean, rstd, Bn, Cn;
          slot_sum<S>(gsh(dn1.r1, go), dn1.cin, c, q0, q1);
          fwd_moments(sstats, ld, sshift, c, inv_n, dn1.eps1, mean, rstd);
          bwd_bc(gsh(dn1.g1, go)[c], mean, rstd, q0, q1, inv_n, Bn, Cn);
          B += Bn;
          C += Cn;
          if (j == 0) {
            gsh(dn1.dbeta1, go)[c] = q0;
            gsh(dn1.dgamma1, go)[c] = q1;
          }
        }
        s.sB[tid] = B;
        s.sC[tid] = C;
      }
      __syncthreads();
      bf16_t* __restrict__ dO16 = gsh(d.dO16, go);
      if (tid < DPITCH / 2) reinterpret_cast<uint32_t*>(s.u.p.dy + DS_MAX_STAGE_ROWS * DPITCH)[tid] = 0u;
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int idx = tid + u * NT;
        if (idx < R * 4) {
          const int lrow = idx >> 2, c8 = (idx & 3) * 8, row = row_lo + lrow;
          float x[8], v[8];
          unpack8(xv[u], x);
          const float dd[8] = {dv[u][0].x + nv[u][0].x, dv[u][0].y + nv[u][0].y, dv[u][0].z + nv[u][0].z,
                               dv[u][0].w + nv[u][0].w, dv[u][1].x + nv[u][1].x, dv[u][1].y + nv[u][1].y,
                               dv[u][1].z + nv[u][1].z, dv[u][1].w + nv[u][1].w};
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = dd[q] + s.sB[c8 + q] * x[q] + s.sC[c8 + q];
          const uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(s.u.p.dy + lrow * DPITCH + c8) = pk;
          if (row >= m0 && row < mend) *reinterpret_cast<uint4*>(dO16 + (size_t)row * 32 + c8) = pk;
        }
      }
      __syncthreads();
      stamp(stamps, task, 2);
      // every LDS read of the tile first (offsets computed before the wait), then the MFMAs
      v8bf af[2][9];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
          if (tap < taps) af[h][tap] = *reinterpret_cast<const v8bf*>(s.u.p.dy + aoff[h][tap]);
      v4f acc[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[h][jj] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        if (tap < taps) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              acc[h][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[h][tap], bq[tap][jj], acc[h][jj], 0, 0, 0);
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            s.u.p.r0[(h * 16 + (lane >> 4) * 4 + q) * RP + wid * 32 + jj * 16 + fr] = acc[h][jj][q];
      __syncthreads();
      {
        float tvf[16], dz[16];
        unpack16(tv0, tv1, tvf);
        const bool okm = em < M;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int c = eseg + q + (q >= 8 ? ESEG2 - 8 : 0);
          const float dA = s.u.p.r0[er * RP + c];
          const float z = s.tab[0][c] * tvf[q] + s.tab[1][c];
          dz[q] = (okm && z > lo && z < hi) ? dA : 0.f;
          const float xh = (tvf[q] - s.tab[2][c]) * s.tab[3][c];
          s.u.p.r0[er * RP + c] = dz[q];
          s.u.p.r1[er * RP + c] = dz[q] * xh;
        }
        if (okm) {
          st_coh16(z2 + (size_t)em * 128 + eseg, pack8(dz));
          st_coh16(z2 + (size_t)em * 128 + eseg + ESEG2, pack8(dz + 8));
        }
      }
      __syncthreads();
      {
        const int c = tid & 127, which = tid >> 7;
        const float* src = which ? s.u.p.r1 : s.u.p.r0;
        float sum = 0.f;
#pragma unroll 8
        for (int row = 0; row < 32; ++row) sum += src[row * RP + c];
        atomicAdd(gsh(d.r2, go) + (j % S) * 256 + which * 128 + c, sum);
      }
      stamp(stamps, task, 3);
      publish_shard(lsync(l), j);
    } else if (kind == DSB_QN) {
      // ========================================= QN_l: dT, then the newest slice's 1x1 dgrad
      const DenseBwdLayerDesc d = layers[l];
      const int cin = d.cin;
      const int j = tile, m0 = j * 32, cn = cin - 32;
      const bf16_t* __restrict__ w1d = gsh(d.w1d, go);
      const bf16_t* __restrict__ tb = gsh(d.t, go);
      const int hq = wid >> 1, jq = wid & 1;  // this wave's 16x16 output block
      v8bf bq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        bq[i] = *reinterpret_cast<const v8bf*>(w1d + (size_t)(cn + jq * 16 + fr) * 128 + i * 32 + fk);
      float g2c = 0.f, mean2 = 0.f, rstd2 = 1.f;
      if (tid < 128) {
        fwd_moments(gsh(d.tstats, go), 128, gsh(d.tshift, go), tid, inv_n, d.eps2, mean2, rstd2);
        g2c = gsh(d.g2, go)[tid];
      }
      if (tid >= 128 && tid < 160) {  // bn1 of the newest slice
        const int i = tid - 128, c = cn + i;
        float mean, rstd;
        fwd_moments(sstats, ld, sshift, c, inv_n, d.eps1, mean, rstd);
        const float sc = gsh(d.g1, go)[c] * rstd;
        s.tab[0][i] = sc;
        s.tab[1][i] = gsh(d.b1, go)[c] - mean * sc;
        s.tab[2][i] = mean;
        s.tab[3][i] = rstd;
      }
      const int er = tid >> 3, eseg = (tid & 7) * 8, em = m0 + er;  // pieces eseg, eseg + 64 (ESEG2)
      uint4 tv0 = make_uint4(0, 0, 0, 0), tv1 = tv0;
      if (em < M) {
        tv0 = *reinterpret_cast<const uint4*>(tb + (size_t)em * 128 + eseg);
        tv1 = *reinterpret_cast<const uint4*>(tb + (size_t)em * 128 + eseg + ESEG2);
      }
      // epilogue rows of this lane: 2 rows per wave instruction, 32 channels each
      const int ech = lane & 31;
      float xq[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = m0 + wid * 2 + (lane >> 5) + 8 * k;
        xq[k] = m < M ? bf2f(buf[(size_t)m * ld + cn + ech]) : 0.f;
      }
      DSB_WAIT8(lsync(l), nmt);
      stamp(stamps, task, 1);
      uint4 zv0 = make_uint4(0, 0, 0, 0), zv1 = zv0;
      if (em < M) {
        zv0 = ld_coh16(z2 + (size_t)em * 128 + eseg);
        zv1 = ld_coh16(z2 + (size_t)em * 128 + eseg + ESEG2);
      }
      if (tid < 128) {
        float q0, q1, B2, C2;
        slot_sum<S>(gsh(d.r2, go), 128, tid, q0, q1);
        bwd_bc(g2c, mean2, rstd2, q0, q1, inv_n, B2, C2);
        s.u.q.r0[tid] = g2c * rstd2;  // A2 / B2 / C2 tables (r0 is free until the MFMAs)
        s.u.q.r0[128 + tid] = B2;
        s.u.q.r0[256 + tid] = C2;
        if (j == 0) {
          gsh(d.dbeta2, go)[tid] = q0;
          gsh(d.dgamma2, go)[tid] = q1;
        }
      }
      __syncthreads();
      {
        float zf[16], tf[16], v[16];
        unpack16(zv0, zv1, zf);
        unpack16(tv0, tv1, tf);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int c = eseg + q + (q >= 8 ? ESEG2 - 8 : 0);
          v[q] = s.u.q.r0[c] * zf[q] + s.u.q.r0[128 + c] * tf[q] + s.u.q.r0[256 + c];
        }
        const uint4 p0 = pack8(v), p1 = pack8(v + 8);
        *reinterpret_cast<uint4*>(s.u.q.dt + er * TP + eseg) = p0;
        *reinterpret_cast<uint4*>(s.u.q.dt + er * TP + eseg + ESEG2) = p1;
        if (em < M) {
          bf16_t* dtg = gsh(d.dt, go) + (size_t)em * 128 + eseg;
          st_coh16(dtg, p0);
          st_coh16(dtg + ESEG2, p1);
        }
      }
      __syncthreads();
      stamp(stamps, task, 2);
      if (l == 0) {  // layer 0's 1x1 dgrad covers the stage input channels: FIN1 does it
        stamp(stamps, task, 3);
        publish_shard(lsync(l) + 8, j);
        continue;
      }
      v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const v8bf af = *reinterpret_cast<const v8bf*>(s.u.q.dt + (hq * 16 + fr) * TP + i * 32 + fk);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[i], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) s.u.q.r0[(hq * 16 + (lane >> 4) * 4 + q) * OP + jq * 16 + fr] = acc[q];
      __syncthreads();
      float* dnw = dnew + (size_t)(l & 1) * M * 32;
      float sdz = 0.f, sdx = 0.f;
      const float sc1 = s.tab[0][ech], sh1 = s.tab[1][ech], mu1 = s.tab[2][ech], rs1 = s.tab[3][ech];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = wid * 2 + (lane >> 5) + 8 * k, m = m0 + row;
        const float dA = s.u.q.r0[row * OP + ech];
        const float z = sc1 * xq[k] + sh1;
        const float dz = (m < M && z > lo && z < hi) ? dA : 0.f;
        if (m < M) st_coh(dnw + (size_t)m * 32 + ech, sc1 * dz);
        sdz += dz;
        sdx += dz * (xq[k] - mu1) * rs1;
      }
      sdz += __shfl_xor(sdz, 32, 64);
      sdx += __shfl_xor(sdx, 32, 64);
      if (lane < 32) {
        s.u.q.part[0][wid][lane] = sdz;
        s.u.q.part[1][wid][lane] = sdx;
      }
      __syncthreads();
      if (tid < 64) {
        const int which = tid >> 5, c = tid & 31;
        const float sum = s.u.q.part[which][0][c] + s.u.q.part[which][1][c] + s.u.q.part[which][2][c] +
                          s.u.q.part[which][3][c];
        atomicAdd(gsh(d.r1, go) + (size_t)(j % S) * 2 * cin + which * cin + cn + c, sum);
      }
      stamp(stamps, task, 3);
      publish_shard(lsync(l) + 8, j);
    } else if (kind == DSB_G || kind == DSB_GIN || kind == DSB_FIN1) {
      // ============ gathered 1x1 dgrad terms of layers [k0, k1) for 32 channels [cs, cs + 32)
      int j, cs, k0, k1, cg = 0;
      if (kind == DSB_G) {  // slice l, layers l+2 .. L-1
        const int kc = tile / nmt;
        j = tile - kc * nmt;
        cs = layers[l].cin;
        k0 = l + 2 + kc * DSB_KG;
        k1 = min(L, k0 + DSB_KG);
      } else if (kind == DSB_GIN) {  // stage input group cg, layers 1 .. L-1
        j = tile % nmt;
        const int r = tile / nmt;
        cg = r % ncg;
        const int kc = r / ncg;
        cs = cg * 32;
        k0 = 1 + kc * DSB_KG;
        k1 = min(L, k0 + DSB_KG);
      } else {  // FIN1: stage input group cg, layer 0
        j = tile % nmt;
        cg = tile / nmt;
        cs = cg * 32;
        k0 = 0;
        k1 = 1;
      }
      const int m0 = j * 32;
      const int hq = wid >> 1, jq = wid & 1;        // this wave's 16 x 16 block of the 32 x 32 tile
      const int c = cs + jq * 16 + fr;              // this lane's channel (MFMA B column = D column)
      const int arow = m0 + hq * 16 + fr;           // this lane's A-operand row
      float xq[4], mean, var;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + hq * 16 + (lane >> 4) * 4 + q;
        xq[q] = m < M ? bf2f(buf[(size_t)m * ld + c]) : 0.f;
      }
      {
        const float kk = sshift ? sshift[c] : 0.f;
        shifted_mean_var(kk, sstats[c], sstats[ld + c], inv_n, mean, var);
      }
      if (kind == DSB_G) DSB_WAIT8(lsync(l + 2) + 8, nmt);        // dT of every layer >= l+2
      else if (kind == DSB_GIN) DSB_WAIT8(lsync(1) + 8, nmt);    // dT of every layer >= 1
      else {
        DSB_WAIT8(lsync(0) + 8, nmt);                            // dT_0
        if (L > 1) DSB_WAIT8(gin_cnt, nmt * ncg * nkc_in);     // GIN's reductions (finalise)
      }
      stamp(stamps, task, 1);
      v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
      // one layer's operands: 4 k-steps of dT_k rows and of W1_k's row for the lane's channel, and
      // the channel's gamma / beta of bn1_k -- everything a layer's term reads from memory, so the
      // loop keeps two layers of loads in flight under the current layer's MFMAs
      struct Ops {
        v8bf a[4], b[4];
        float g, bt;
      };
      auto load = [&](int k, Ops& o) {
        const DenseBwdLayerDesc dk = layers[k];
        const bf16_t* dtk = gsh(dk.dt, go) + (size_t)arow * 128 + fk;
        const bf16_t* wk = gsh(dk.w1d, go) + (size_t)c * 128 + fk;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o.a[i] = arow < M ? __builtin_bit_cast(v8bf, ld_coh16(dtk + i * 32)) : v8bf{};
          o.b[i] = *reinterpret_cast<const v8bf*>(wk + i * 32);
        }
        o.g = gsh(dk.g1, go)[c];
        o.bt = gsh(dk.b1, go)[c];
      };
      // per-layer reductions stay in registers until every load of the tile has been issued: a
      // float atomic issued between the prefetches would make the next operand wait (vmcnt counts
      // loads and atomics in issue order) for the atomic's round trip
      float rdz[DSB_KG], rdx[DSB_KG];
      auto layer_term = [&](int kk, const Ops& o) {
        v4f dA = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) dA = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o.a[i], o.b[i], dA, 0, 0, 0);
        const float rstd = rsqrtf(var + layers[k0 + kk].eps1);
        float sdz = 0.f, sdx = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = m0 + hq * 16 + (lane >> 4) * 4 + q;
          const float xh = (xq[q] - mean) * rstd;
          const float z = o.g * xh + o.bt;
          const float dz = (m < M && z > lo && z < hi) ? dA[q] : 0.f;
          acc[q] += o.g * rstd * dz;
          sdz += dz;
          sdx += dz * xh;
        }
        sdz += __shfl_xor(sdz, 16, 64);
        sdx += __shfl_xor(sdx, 16, 64);
        sdz += __shfl_xor(sdz, 32, 64);
        sdx += __shfl_xor(sdx, 32, 64);
        rdz[kk] = sdz;
        rdx[kk] = sdx;
      };
      static_assert(DSB_KG == 6, "the gather loop below is unrolled for 6 layers, 3 operand buffers");
      Ops o0, o1, o2;
      load(k0, o0);
      if (k0 + 1 < k1) load(k0 + 1, o1);
      stamp(stamps, task, 2);
      if (k0 + 2 < k1) load(k0 + 2, o2);
      layer_term(0, o0);
      if (k0 + 1 < k1) {
        if (k0 + 3 < k1) load(k0 + 3, o0);
        layer_term(1, o1);
      }
      if (k0 + 2 < k1) {
        if (k0 + 4 < k1) load(k0 + 4, o1);
        layer_term(2, o2);
      }
      if (k0 + 3 < k1) {
        if (k0 + 5 < k1) load(k0 + 5, o2);
        layer_term(3, o0);
      }
      if (k0 + 4 < k1) layer_term(4, o1);
      if (k0 + 5 < k1) layer_term(5, o2);
      if (lane < 16) {
#pragma unroll
        for (int kk = 0; kk < DSB_KG; ++kk) {
          if (k0 + kk < k1) {
            const DenseBwdLayerDesc dk = layers[k0 + kk];
            float* r1 = gsh(dk.r1, go) + (size_t)(j % S) * 2 * dk.cin;
            atomicAdd(r1 + c, rdz[kk]);
            atomicAdd(r1 + dk.cin + c, rdx[kk]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + hq * 16 + (lane >> 4) * 4 + q;
        if (m < M) atomicAdd(dbuf + (size_t)m * ld + c, acc[q]);
      }
      stamp(stamps, task, 3);
      // arrival; the last tile of G_l (of FIN1's group cg) turns the channels' reductions of every
      // layer k that normalises them (and the consumer BatchNorm's) into btot, and writes their
      // d beta / d gamma
      unsigned* arrive = kind == DSB_G ? lsync(l) + 16 : kind == DSB_GIN ? gin_cnt + (tile & 7) : f1_cnt + cg;
      const int ntiles = kind == DSB_G ? nmt * ((L - 2 - l + DSB_KG - 1) / DSB_KG) : nmt;
      const unsigned old = publish(arrive);
      if (kind == DSB_GIN) continue;
      if (tid == 0) s.last = old == (unsigned)(ntiles - 1);
      __syncthreads();
      if (!__builtin_amdgcn_readfirstlane(s.last)) continue;
      {
        // thread (channel ch, layer group kg): layers kf .. L-1 with k = kf + kg (mod 8)
        const int ch = tid & 31, kg = tid >> 5, cc = cs + ch;
        const int kf = kind == DSB_G ? l + 2 : 0;
        float mu, vv;
        shifted_mean_var(sshift ? sshift[cc] : 0.f, sstats[cc], sstats[ld + cc], inv_n, mu, vv);
        float B = 0.f, C = 0.f;
        for (int k = kf + kg; k < L; k += 8) {
          const DenseBwdLayerDesc dk = layers[k];
          float q0, q1, Bk, Ck;
          slot_sum<S>(gsh(dk.r1, go), dk.cin, cc, q0, q1);
          bwd_bc(gsh(dk.g1, go)[cc], mu, rsqrtf(vv + dk.eps1), q0, q1, inv_n, Bk, Ck);
          B += Bk;
          C += Ck;
          gsh(dk.dbeta1, go)[cc] = q0;
          gsh(dk.dgamma1, go)[cc] = q1;
        }
        if (kg == 0) {
          float Bp, Cp;
          pend_bc(pend, cc, Bp, Cp);
          B += Bp;
          C += Cp;
        }
        s.u.fin[0][kg][ch] = B;
        s.u.fin[1][kg][ch] = C;
        __syncthreads();
        if (tid < 64) {
          const int which = tid >> 5, c2 = tid & 31;
          float v = 0.f;
#pragma unroll
          for (int g = 0; g < 8; ++g) v += s.u.fin[which][g][c2];
          st_coh(btot + (size_t)which * ld + cs + c2, v);
        }
      }
      publish(kind == DSB_G ? lsync(l) + 17 : f1_done);
    } else {
      // ================================= FIN2: the stage input channels' final gradient (bf16)
      const int cb = tile / nmt, j = tile - cb * nmt, m0 = j * 32;
      DSB_WAIT(f1_done, ncg);
      stamp(stamps, task, 1);
      const int c = cb * 64 + lane;
      const bool okc = c < a.c0;
      float B = 0.f, C = 0.f;
      if (okc) {
        B = ld_coh(btot + c);
        C = ld_coh(btot + ld + c);
      }
      stamp(stamps, task, 2);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int m = m0 + wid + 4 * k;
        if (okc && m < M) {
          const float v = ld_coh(dbuf + (size_t)m * ld + c) + B * bf2f(buf[(size_t)m * ld + c]) + C;
          dx16[(size_t)m * a.c0 + c] = f2bf(v);
        }
      }
      stamp(stamps, task, 3);
      publish(f2_cnt);
    }
#undef DSB_WAIT
#undef DSB_WAIT8
  }
}

hipError_t dense_stage_bwd(const DenseBwdArgs& a, int grid, hipStream_t st) {
  if (a.nlayers < 1 || (a.k2 != 1 && a.k2 != 3) || a.ld % 8 != 0 || a.c0 % 32 != 0 || a.c0 <= 32 ||
      a.c0 > a.ld || a.c0 / 32 > DSB_MAX_CG || a.N < 1 || a.H < 1 || a.W < 1 || a.buf == nullptr ||
      a.sstats == nullptr || a.dbuf == nullptr || a.dnew == nullptr || a.dx16 == nullptr || a.z2 == nullptr ||
      a.layers == nullptr || a.phases == nullptr || a.sync == nullptr || a.btot == nullptr || a.nphases < 1 ||
      a.ntickets < 1 || !dense_stage_shape_ok(a.N, a.H, a.W, 0))
    return hipErrorInvalidValue;
  if (a.rows && dense_rows_bwd(a, st) == hipSuccess) return hipSuccess;
  if (grid <= 0) grid = 256;
  const int k = launch_groups().k;
  if (k > 1) grid = grid / k > 8 ? grid / k : 8;
  if (grid > a.ntickets) grid = a.ntickets;
  hipLaunchKernelGGL(dense_stage_bwd_kernel, ggrid(grid), dim3(NT), 0, st, a, garg());
  return hipGetLastError();
}

}  // namespace idc
