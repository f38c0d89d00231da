// Persistent dense-stage forward for DenseNet (gfx950): all dense layers of one stage in ONE launch.
//
// A dense layer is  y = conv3x3(ReLU(BN2(conv1x1(ReLU(BN1(x[:, :cin]))))))  written into channels
// [cin, cin+32) of the stage buffer (reference: /root/reference/dist_model_tf_dense.py:131-133
// builds DenseNet-121 / -201 through Keras Applications).  In the late stages (bs
// 256: 3x3 and 1x1 maps, M = 2,304 / 256 pixels) every conv is a few hundred MFLOP, so the stage is
// a chain of 2 x layers dependent phases whose cost is the hand-off between them, not arithmetic.
//
// One launch walks the stage as a WORK QUEUE of tiles:
//     [layer 0: 1x1 tiles (A_0)][layer 0: 3x3 tiles (B_0)][layer 1: 1x1 tiles (A_1)] ...
// or, when more than one A phase's worth of workgroups is resident (lookahead order),
//     [A_0][A_1][B_0][A_2][B_1] ... [A_{L-1}][B_{L-2}][B_{L-1}]
// A workgroup takes the next ticket (one agent-scope atomic) and waits, where it must, until a
// phase's completion counter is full.  In layer order every tile a waiting workgroup depends on
// was taken earlier by a workgroup that is already running (or done): that queue cannot deadlock
// whatever number of workgroups is resident.  In lookahead order only A_{l+1}'s last k-step waits
// on a later ticket (B_l, queued right after it), so the queue progresses whenever more than nA
// workgroups are resident -- the launcher uses it only then.  Every wait is
// poll-bounded; a workgroup that gives up sets the launch's fail flag (all others then leave) and
// the first one to set it counts the launch in the persistent error counter.
//
// What is on the dependent chain, and what is not (the DenseNet structure):
//   * A_l's 1x1 input is the concatenation of every earlier slice, and a slice's batch statistics
//     are final once its producer phase is.  Only the NEWEST slice (32 channels, from B_{l-1}) is
//     on the chain: an A_l tile first accumulates the channels [0, cin-32) -- final since A_{l-1}
//     -- into registers, then waits for B_{l-1} and adds one 32-deep k-step.  Workgroups that run
//     ahead of the chain do that accumulation while B_{l-1} is still computing.
//   * BatchNorm statistics produced in the launch go into DS_SLOTS slot copies (float atomics
//     serialise per address at ~24 ns, common.h "Statistics slots": 144 tiles adding into one
//     row cost ~3.5 us per phase); a consumer sums the copies of the channels it needs (<= 8 KB).
//     Tile 0 of the consuming phase writes the summed statistics into the program's single-copy
//     rows (tstats, sstats) that the backward and the moving averages read after the launch.
//   * Completion counters are polled with agent-coherent (sc1) loads from ONE lane (an atomic
//     read-modify-write poll by ~200 workgroups contends with the producers' increments).
//
// Hand-off memory model: every byte produced inside the launch (t, the stage-buffer slices, the
// statistics) is stored and loaded with agent-scope atomic accesses (sc1), the producer drains
// them (s_waitcnt vmcnt(0)) before its counter increment, the consumer loads after its poll
// matched and a workgroup barrier (MI355X_MICROARCH.md, "Valid forms", first table row).
//
// Tile shapes (64-wide waves, v_mfma_f32_16x16x32_bf16):
//   A (1x1): 32 rows x 64 output channels; each wave owns 16 channels over the whole K (no
//            cross-wave reduction); the 32-row A operand is staged once per workgroup in LDS,
//            BN1+ReLU applied while staging, in 256-channel chunks, one chunk's loads in flight
//            under the previous chunk's MFMAs.
//   B (3x3): 32 rows x all 32 output channels; the rows of t under the tile's 3x3 windows (whole
//            images: 45 rows on 3x3 maps) are staged in LDS with BN2+ReLU applied, the 9 taps x 128
//            channels are split over the 4 waves and reduced in LDS.
// Diagnostics: with `stamps` set, thread 0 writes s_memrealtime (100 MHz) at ticket / dependency
// cleared / operands staged / before publish for every work item (tools/dense_stamps.py).
#include "dense_stage.h"
#include "persist.h"

#include <cstdlib>

namespace idc {
namespace {

constexpr int NT = 256;
constexpr int S = DS_SLOTS;
constexpr int ACH = 256;            // A-phase staging chunk (channels)
constexpr int APITCH = ACH + 8;     // LDS row pitch (bf16): 528 B rows, conflict-free b128 reads
constexpr int TPITCH = 128 + 8;     // B-phase staged t row pitch (bf16)
constexpr int RLD = 33;             // B-phase partial-tile row stride (floats)
constexpr int RLDA = 65;            // A-phase epilogue tile row stride (floats)

struct Smem {
  float sc[DS_MAX_CIN];
  float sh[DS_MAX_CIN];
  union {
    bf16_t a[2][32 * APITCH];
    bf16_t t[(DS_MAX_STAGE_ROWS + 1) * TPITCH];  // + one all-zero row (3x3 padding taps)
  } u;
  float red[4][32 * RLD];
  int task;
  int bad;
};
static_assert(sizeof(float) * 32 * RLDA <= sizeof(float) * 4 * 32 * RLD, "A epilogue tile fits red");

using namespace persist;

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

// BN scale/shift for channels [0, C) (C <= DS_MAX_CIN) from the single-copy shifted statistics
// (row length ld), read agent-coherently (some of them were written in this launch); each thread's
// loads of a batch of 4 channels are all issued before the arithmetic
__device__ __forceinline__ void bn_table(const float* st, int ld, const float* shift, const float* g,
                                         const float* b, float inv_n, float eps, int C0, int C, float* sc,
                                         float* sh) {
  const int tid = threadIdx.x;
  for (int base = C0; base < C; base += 4 * NT) {
    float s0[4], s1[4], k[4], gg[4], bb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = base + tid + u * NT;
      const int cc = c < C ? c : 0;
      s0[u] = ld_coh(st + cc);
      s1[u] = ld_coh(st + ld + cc);
      k[u] = shift ? shift[cc] : 0.f;
      gg[u] = g[cc];
      bb[u] = b[cc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = base + tid + u * NT;
      if (c < C) {
        float mean, var;
        shifted_mean_var(k[u], s0[u], s1[u], inv_n, mean, var);
        const float r = gg[u] * rsqrtf(var + eps);
        sc[c] = r;
        sh[c] = bb[u] - mean * r;
      }
    }
  }
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
  // counters: [0] ticket; layer l: A_l (8 shards) at 1 + 16l, B_l (8 shards) at 9 + 16l; then the
  // last layer's unsharded arrival count (its last tile writes the last slice's statistics), fail
  auto cntA = [&](int l) { return sync + 1 + 16 * l; };
  auto cntB = [&](int l) { return sync + 9 + 16 * l; };
  unsigned* lastfin = sync + 1 + 16 * a.nlayers;
  unsigned* fail = lastfin + 1;  // this launch gave up (zeroed with the counters)
  unsigned* tilecnt = fail + 1;  // [nlayers][nT] helper partials arrived per A tile
  float* partials = gsh(a.partials, go);
  int* err = gsh(a.err, go);
  const persist::FailSink fsink{err, gsh(a.stepflag, go), a.hostflag};
  float* scratch = gsh(a.scratch, go);
  unsigned long long* stamps = gsh(a.stamps, go);
  const unsigned max_polls = a.max_polls ? a.max_polls : DEFAULT_POLLS;

  __shared__ __attribute__((aligned(16))) Smem s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int HW = a.H * a.W, M = a.N * HW;
  const int nmt = (M + 31) / 32;
  // split K: an A tile's older channels are spread over KS work items -- KS-1 helpers (queued
  // first) hand fp32 partial tiles to the tile's finalizer, which adds them, runs the newest-slice
  // step and the epilogue
  const int KS = a.ksplit > 1 ? a.ksplit : 1;
  const int nT = 2 * nmt, nH = nT * (KS - 1);
  const int nA = nT * KS, nB = nmt;
  const int per = nA + nB, total = per * a.nlayers;
  const int taps = a.k2 * a.k2, pad = a.k2 >> 1;
  const float lo1 = act_lo(a.act1), hi1 = act_hi(a.act1);
  const float lo2 = act_lo(a.act2), hi2 = act_hi(a.act2);
  // the zero row past the staged t rows (never written by a tile: the A-phase buffers end before it)
  static_assert(sizeof(bf16_t) * 2 * 32 * APITCH <= sizeof(bf16_t) * DS_MAX_STAGE_ROWS * TPITCH, "zero row");
  for (int i = tid; i < TPITCH / 2; i += NT) reinterpret_cast<uint32_t*>(s.u.t + DS_MAX_STAGE_ROWS * TPITCH)[i] = 0u;

  for (;;) {
    // The ticket fetch is a thread-0 region enclosed by barriers on both sides (without the
    // leading barrier hipcc merged it with the previous tile's thread-0 publish and the other
    // waves re-ran the stale tile).  The LDS broadcast goes through readfirstlane so every control
    // decision of the loop is workgroup-uniform (no barrier in exec-masked flow).
    __syncthreads();
    if (tid == 0) s.task = (int)__hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(s.task);
    if (task >= total) return;
    stamp(stamps, task, 0);
    int l, r;  // layer and phase-local item (r < nA: A_l, else B_l item r - nA)
    if (!a.lookahead) {
      l = task / per;
      r = task - l * per;
    } else if (task < nA) {
      l = 0;
      r = task;
    } else {
      // lookahead order [A0][A1 B0][A2 B1]...[A_{L-1} B_{L-2}][B_{L-1}]: A_{l+1} is queued before
      // B_l, so its older-channel accumulation (needs B_{l-1} only) runs beside B_l instead of
      // after it; its newest-slice step then waits on B_l, a LATER ticket -- safe while more than
      // nA workgroups are resident (dense_stage_fwd enables it only then)
      const int t2 = task - nA, j = t2 / per + 1, rr = t2 - (j - 1) * per;
      if (j < a.nlayers && rr < nA) {
        l = j;
        r = rr;
      } else {
        l = j - 1;
        r = j < a.nlayers ? rr : nA + rr;
      }
    }
    const DenseLayerDesc d = layers[l];
    float* lslots = scratch + (size_t)l * DS_SCRATCH_PER_LAYER;  // [S][2][32] stats of B_l's slice
    float* tslots = lslots + S * 64;                              // [S][2][128] stats of A_l's t

    if (r < nA) {
      // ================================================= A_l: t = conv1x1(relu(bn1(x[:, :cin])))
      const bf16_t* __restrict__ w1 = gsh(d.w1, go);
      bf16_t* __restrict__ tb = gsh(d.t, go);
      const float* __restrict__ tsh = gsh(d.tshift, go);
      const float* __restrict__ g1 = gsh(d.g1, go);
      const float* __restrict__ b1 = gsh(d.b1, go);
      const bool helper = r < nH;
      const int tile = helper ? r / (KS - 1) : r - nH;
      const int ks = helper ? 1 + r % (KS - 1) : 0;
      const int mt = tile >> 1, n0 = (tile & 1) * 64, m0 = mt * 32;
      const int cin = d.cin;
      const int cold = l == 0 ? cin : cin - 32;  // channels final before B_{l-1}
      // this item's share of the older channels, in 32-channel k-steps
      const int nst = cold >> 5;
      const int k_lo = (ks * nst / KS) * 32, k_hi = ((ks + 1) * nst / KS) * 32;
      const bf16_t* wrow = w1 + (size_t)(n0 + wid * 16 + fr) * cin;  // this lane's B column
      const v8bf bnew = l > 0 ? *reinterpret_cast<const v8bf*>(wrow + cold + fk) : v8bf{};
      const int erow = tid >> 3, ecol = (tid & 7) * 8;
      float kq[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) kq[q] = tsh ? tsh[n0 + ecol + q] : 0.f;
      v4f acc[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};

      // ---- channels [0, cold): final once B_{l-2} is complete.  Their statistics: single-copy
      // rows for [0, cold-32) (written by A_{l-1}'s tile 0 at the latest -- A_{l-2} for the slice
      // of B_{l-3} -- hence complete before B_{l-2} started), B_{l-2}'s slots for [cold-32, cold)
      if (l >= 2) {
        if (wid == 0) {
          const bool ok = wait_sum8(cntB(l - 2), (unsigned)nB, fail, fsink, max_polls);
          if (lane == 0) s.bad = !ok;
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s.bad)) return;
      }
      stamp(stamps, task, 1);
      // staging: 8 threads per row, thread piece u at channels ((tid & 7) + 8u) * 8 -- each
      // wave-level access covers 128 contiguous bytes of a row (a 32-channel run per thread wrote
      // 16-B pieces at a 64-B stride: 2-way LDS bank conflicts, half-line global loads)
      const int srow = m0 + (tid >> 3), sseg = (tid & 7) * 8;
      uint4 ar[4];
      auto load_a = [&](int ch) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = k_lo + ch * ACH + sseg + u * 64;
          ar[u] = (srow < M && c < k_hi) ? ld_coh16(buf + (size_t)srow * a.ld + c) : make_uint4(0, 0, 0, 0);
        }
      };
      auto load_b = [&](int ch, v8bf (&bq)[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k_lo + ch * ACH + i * 32;
          bq[i] = k < k_hi ? *reinterpret_cast<const v8bf*>(wrow + k + fk) : v8bf{};
        }
      };
      auto stage = [&](int ch) {
        bf16_t* ab = s.u.a[ch & 1] + (tid >> 3) * APITCH + sseg;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = k_lo + ch * ACH + sseg + u * 64;
          const bool keep = srow < M && c < k_hi;
          const int cc = keep ? c : 0;
          *reinterpret_cast<v8bf*>(ab + u * 64) = bn_act8(ar[u], s.sc + cc, s.sh + cc, lo1, hi1, keep);
        }
      };
      auto mfma_chunk = [&](int ch, const v8bf (&bq)[8]) {
        const bf16_t* ab = s.u.a[ch & 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (k_lo + ch * ACH + i * 32 < k_hi) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const v8bf af = *reinterpret_cast<const v8bf*>(ab + (h * 16 + fr) * APITCH + i * 32 + fk);
              acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[i], acc[h], 0, 0, 0);
            }
          }
        }
      };
      const int nch = (k_hi - k_lo + ACH - 1) / ACH;
      v8bf bq0[8], bq1[8];
      load_a(0);
      load_b(0, bq0);
      const int ccanon = l >= 2 ? cold - 32 : cold;
      // inference-mode BN1 (a frozen layer in a fine-tuned stage, or the whole launch): the
      // layer's own moving statistics; the statistics of the stage buffer are still produced
      // for the trainable layers after it (unless the whole launch is inference mode)
      const bool inf1 = a.infer || (d.pad_ & 1);
      if (inf1) {  // inference mode: the layer's own moving statistics (the finalizer's newest slice too)
        const float* __restrict__ mm = gsh(d.mm1, go);
        const float* __restrict__ mv = gsh(d.mv1, go);
        const int c_end = helper ? k_hi : cin;
        for (int c = k_lo + tid; c < c_end; c += NT) {
          if (c >= k_hi && c < cold) continue;
          const float rr = g1[c] * rsqrtf(mv[c] + d.eps1);
          s.sc[c] = rr;
          s.sh[c] = b1[c] - mm[c] * rr;
        }
      } else {
        bn_table(sstats, a.ld, sshift, g1, b1, a.inv_count, d.eps1, k_lo, min(ccanon, k_hi), s.sc, s.sh);
      }
      if (!inf1 && l >= 2 && ccanon >= k_lo && ccanon < k_hi && tid < 32) {
        float s0, s1, mean, var;
        slot_sum<S>(lslots - 2 * DS_SCRATCH_PER_LAYER, 32, tid, s0, s1);
        const int c = ccanon + tid;
        shifted_mean_var(sshift ? sshift[c] : 0.f, s0, s1, a.inv_count, mean, var);
        const float rr = g1[c] * rsqrtf(var + d.eps1);
        s.sc[c] = rr;
        s.sh[c] = b1[c] - mean * rr;
      }
      __syncthreads();
      // chunk ch: stage it (BN1+ReLU into LDS buffer ch&1), barrier, put the next chunk's loads in
      // flight, then its MFMAs; the double buffer makes one barrier per chunk sufficient
      for (int ch = 0; ch < nch; ch += 2) {
        stage(ch);
        __syncthreads();
        if (ch + 1 < nch) {
          load_a(ch + 1);
          load_b(ch + 1, bq1);
        }
        mfma_chunk(ch, bq0);
        if (ch + 1 < nch) {
          stage(ch + 1);
          __syncthreads();
          if (ch + 2 < nch) {
            load_a(ch + 2);
            load_b(ch + 2, bq0);
          }
          mfma_chunk(ch + 1, bq1);
        }
      }

      stamp(stamps, task, 2);
      float* pslab = partials + (size_t)(l & 1) * nH * (NT * 8);  // layers l and l+2 alternate
      if (helper) {
        // ---- a helper's partial tile (MFMA register layout, 32 B per thread) to the finalizer.
        // The slab slot is free again: the previous layer of this parity finished its finalizers
        // before B of that layer ran, which this item's B_{l-2} wait (l >= 2) ordered before it
        float* dst = pslab + ((size_t)tile * (KS - 1) + (ks - 1)) * (NT * 8) + tid * 8;
        st_coh16(dst, __builtin_bit_cast(uint4, acc[0]));
        st_coh16(dst + 4, __builtin_bit_cast(uint4, acc[1]));
        publish(tilecnt + (size_t)l * nT + tile);
        continue;
      }
      // ---- the newest slice [cold, cin): wait for B_{l-1}; and this tile's helpers
      if (l > 0 || KS > 1) {
        if (wid == 0) {
          bool ok = l == 0 || wait_sum8(cntB(l - 1), (unsigned)nB, fail, fsink, max_polls);
          if (ok && KS > 1 && lane == 0)
            ok = wait_count(tilecnt + (size_t)l * nT + tile, (unsigned)(KS - 1), fail, fsink, max_polls);
          if (lane == 0) s.bad = !ok;
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s.bad)) return;
      }
      if (KS > 1) {  // the helpers' partials, all loads in flight together
        uint4 pv[2 * (DS_MAX_KSPLIT - 1)];
        const float* src = pslab + (size_t)tile * (KS - 1) * (NT * 8) + tid * 8;
#pragma unroll
        for (int h = 0; h < DS_MAX_KSPLIT - 1; ++h)
          if (h < KS - 1) {
            pv[2 * h] = ld_coh16(src + (size_t)h * (NT * 8));
            pv[2 * h + 1] = ld_coh16(src + (size_t)h * (NT * 8) + 4);
          }
#pragma unroll
        for (int h = 0; h < DS_MAX_KSPLIT - 1; ++h)
          if (h < KS - 1) {
            acc[0] += __builtin_bit_cast(v4f, pv[2 * h]);
            acc[1] += __builtin_bit_cast(v4f, pv[2 * h + 1]);
          }
      }
      stamp(stamps, task, 3);
      if (l > 0) {
        const float* pslots = lslots - DS_SCRATCH_PER_LAYER;  // B_{l-1}'s slice statistics
        const int nrow = m0 + (tid >> 2), nseg = (tid & 3) * 8;
        const uint4 an = (tid < 128 && nrow < M) ? ld_coh16(buf + (size_t)nrow * a.ld + cold + nseg)
                                                 : make_uint4(0, 0, 0, 0);
        if (!a.infer && tid < 32) {
          float s0, s1, mean, var;
          slot_sum<S>(pslots, 32, tid, s0, s1);
          const int c = cold + tid;
          shifted_mean_var(sshift ? sshift[c] : 0.f, s0, s1, a.inv_count, mean, var);
          if (!inf1) {
            const float rr = g1[c] * rsqrtf(var + d.eps1);
            s.sc[c] = rr;
            s.sh[c] = b1[c] - mean * rr;
          }
          if (tile == 0) {  // the slice's single-copy statistics (read by later layers' tables)
            st_coh(sstats + c, s0);
            st_coh(sstats + a.ld + c, s1);
          }
        }
        __syncthreads();
        if (tid < 128)
          *reinterpret_cast<v8bf*>(s.u.a[0] + (tid >> 2) * APITCH + nseg) =
              bn_act8(an, s.sc + cold + nseg, s.sh + cold + nseg, lo1, hi1, nrow < M);
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const v8bf af = *reinterpret_cast<const v8bf*>(s.u.a[0] + (h * 16 + fr) * APITCH + fk);
          acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bnew, acc[h], 0, 0, 0);
        }
      }
      stamp(stamps, task, 4);

      // ---- epilogue: bf16 t tile (16-B sc1 stores), shifted statistics into slot mt % S
      float* red = s.red[0];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[(h * 16 + (lane >> 4) * 4 + q) * RLDA + wid * 16 + fr] = acc[h][q];
      __syncthreads();
      stamp(stamps, task, 5);
      {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = red[erow * RLDA + ecol + q];
        const int m = m0 + erow;
        const uint4 pk = pack8(v);
        if (m < M) st_coh16(tb + (size_t)m * 128 + n0 + ecol, pk);
        float rv[8];
        unpack8(pk, rv);
#pragma unroll
        for (int q = 0; q < 8; ++q) red[erow * RLDA + ecol + q] = m < M ? rv[q] - kq[q] : 0.f;
      }
      __syncthreads();
      if (!a.infer && tid < 128) {
        const int c = tid & 63, which = tid >> 6;
        float sum = 0.f;
#pragma unroll 8
        for (int row = 0; row < 32; ++row) {
          const float x = red[row * RLDA + c];
          sum += which ? x * x : x;
        }
        atomicAdd(&tslots[(mt % S) * 256 + which * 128 + n0 + c], sum);
      }
      stamp(stamps, task, 6);
      {
        const unsigned o = publish_shard(cntA(l), tile);
        if (stamps && tid == 0) stamps[(size_t)task * NSTAMP + 7] = __builtin_amdgcn_s_memrealtime() + (o & 0u);
      }
    } else {
      // ================================================= B_l: buf[:, cin:cin+32] = conv3x3(relu(bn2(t)))
      const bf16_t* __restrict__ w2 = gsh(d.w2, go);
      const bf16_t* __restrict__ tb = gsh(d.t, go);
      float* __restrict__ tst = gsh(d.tstats, go);
      const float* __restrict__ tsh = gsh(d.tshift, go);
      const int j = r - nA, m0 = j * 32;
      const int cin = d.cin, Kc = taps * 128, nks = taps * 4;
      // weight fragments do not depend on earlier phases: in flight before the wait
      v8bf bq[9][2];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int ks = wid + 4 * i;
        const int tap = ks >> 2, c = (ks & 3) * 32 + fk;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          bq[i][jj] = ks < nks ? *reinterpret_cast<const v8bf*>(w2 + (size_t)(jj * 16 + fr) * Kc + tap * 128 + c)
                               : v8bf{};
      }
      const int erow = tid >> 3, ecol = (tid & 7) * 4;
      float kq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) kq[q] = sshift ? sshift[cin + ecol + q] : 0.f;
      float g2c = 0.f, b2c = 0.f, ksh = 0.f;
      if (tid < 128) {
        g2c = gsh(d.g2, go)[tid];
        b2c = gsh(d.b2, go)[tid];
        ksh = tsh ? tsh[tid] : 0.f;
      }
      const int mend = min(m0 + 32, M);
      const int img_lo = m0 / HW, img_hi = (mend - 1) / HW;
      const int row_lo = img_lo * HW, R = (img_hi - img_lo + 1) * HW;
      // LDS element offsets of this lane's A fragments (k-step wid + 4i, row fragment h) in the
      // staged t rows; zero padding is applied AFTER the activation (Keras 'same' conv of
      // relu(bn(t))), so padding taps read the all-zero row
      int aoff[2][9];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = m0 + h * 16 + fr;
        const int mm = m < M ? m : M - 1;
        const int img = mm / HW, rem = mm - img * HW;
        const int ph = rem / a.W, pw = rem - ph * a.W;
        const int ibase = img * HW - row_lo;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          const int ks = wid + 4 * i;
          const int tap = ks >> 2;
          const int kr = tap / a.k2, kc = tap - kr * a.k2;
          const int hh = ph + kr - pad, ww = pw + kc - pad;
          const bool ok = ks < nks && m < M && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
          const int lrow = ok ? ibase + hh * a.W + ww : DS_MAX_STAGE_ROWS;
          aoff[h][i] = lrow * TPITCH + (ks & 3) * 32 + fk;
        }
      }
      stamp(stamps, task, 1);
      if (wid == 0) {
        const bool ok = wait_sum8(cntA(l), (unsigned)nT, fail, fsink, max_polls);
        if (lane == 0) s.bad = !ok;
      }
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s.bad)) return;
      stamp(stamps, task, 2);
      // t rows under the tile's windows (raw) and the t statistics, all loads in flight together
      constexpr int TU = DS_MAX_STAGE_ROWS * 16 / NT;
      uint4 traw[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int idx = tid + u * NT;
        traw[u] = idx < R * 16 ? ld_coh16(tb + (size_t)(row_lo + (idx >> 4)) * 128 + (idx & 15) * 8)
                               : make_uint4(0, 0, 0, 0);
      }
      const bool inf2 = a.infer || (d.pad_ & 2);
      if (tid < 128 && inf2) {
        const float mean = gsh(d.mm2, go)[tid], var = gsh(d.mv2, go)[tid];
        const float rr = g2c * rsqrtf(var + d.eps2);
        s.sc[tid] = rr;
        s.sh[tid] = b2c - mean * rr;
      }
      if (tid < 128 && !a.infer) {
        float s0, s1, mean, var;
        slot_sum<S>(tslots, 128, tid, s0, s1);
        shifted_mean_var(ksh, s0, s1, a.inv_count, mean, var);
        if (!inf2) {
          const float rr = g2c * rsqrtf(var + d.eps2);
          s.sc[tid] = rr;
          s.sh[tid] = b2c - mean * rr;
        }
        if (j == 0) {  // t's single-copy statistics (backward, moving averages)
          tst[tid] = s0;
          tst[128 + tid] = s1;
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int idx = tid + u * NT;
        if (idx < R * 16) {
          const int c = (idx & 15) * 8;
          *reinterpret_cast<v8bf*>(s.u.t + (idx >> 4) * TPITCH + c) = bn_act8(traw[u], s.sc + c, s.sh + c, lo2, hi2, true);
        }
      }
      __syncthreads();
      stamp(stamps, task, 3);
      // every LDS read of the tile first (offsets computed before the wait), then the MFMAs
      v8bf af[2][9];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 9; ++i)
          if (wid + 4 * i < nks) af[h][i] = *reinterpret_cast<const v8bf*>(s.u.t + aoff[h][i]);
      v4f acc[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[h][jj] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 9; ++i)
        if (wid + 4 * i < nks) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              acc[h][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[h][i], bq[i][jj], acc[h][jj], 0, 0, 0);
        }
      float* red = s.red[wid];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int q = 0; q < 4; ++q) red[(h * 16 + (lane >> 4) * 4 + q) * RLD + jj * 16 + fr] = acc[h][jj][q];
      __syncthreads();
      stamp(stamps, task, 4);
      {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int o = erow * RLD + ecol + q;
          v[q] = s.red[0][o] + s.red[1][o] + s.red[2][o] + s.red[3][o];
        }
        const int mo = m0 + erow;
        const uint32_t p0 = pack2bf(v[0], v[1]), p1 = pack2bf(v[2], v[3]);
        if (mo < M) st_coh8(buf + (size_t)mo * a.ld + cin + ecol, p0, p1);
        const float rv[4] = {__uint_as_float(p0 << 16), __uint_as_float(p0 & 0xffff0000u),
                             __uint_as_float(p1 << 16), __uint_as_float(p1 & 0xffff0000u)};
#pragma unroll
        for (int q = 0; q < 4; ++q) s.red[0][erow * RLD + ecol + q] = mo < M ? rv[q] - kq[q] : 0.f;
      }
      __syncthreads();
      stamp(stamps, task, 5);
      if (!a.infer && tid < 64) {
        const int c = tid & 31, which = tid >> 5;
        float sum = 0.f;
#pragma unroll 8
        for (int row = 0; row < 32; ++row) {
          const float x = s.red[0][row * RLD + c];
          sum += which ? x * x : x;
        }
        atomicAdd(&lslots[(j % S) * 64 + which * 32 + c], sum);
      }
      stamp(stamps, task, 6);
      {
        const unsigned o = publish_shard(cntB(l), j);
        if (stamps && tid == 0) stamps[(size_t)task * NSTAMP + 7] = __builtin_amdgcn_s_memrealtime() + (o & 0u);
      }
      if (l == a.nlayers - 1 && !a.infer) {
        // the last slice has no in-launch consumer: the last tile to complete writes its
        // single-copy statistics
        if (tid == 0)
          s.bad = __hip_atomic_fetch_add(lastfin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nB - 1);
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s.bad) && tid < 32) {
          float s0, s1;
          slot_sum<S>(lslots, 32, tid, s0, s1);
          sstats[cin + tid] = s0;
          sstats[a.ld + cin + tid] = s1;
        }
      }
    }
  }
}

void dense_stage_phase_tiles(int M, int ksplit, int& nA, int& nB) {
  const int nmt = (M + 31) / 32;
  nA = 2 * nmt * (ksplit > 1 ? ksplit : 1);
  nB = nmt;
}

int dense_stage_tasks(const DenseStageArgs& a) {
  int nA, nB;
  dense_stage_phase_tiles(a.N * a.H * a.W, a.ksplit, nA, nB);
  return a.nlayers * (nA + nB);
}

int dense_stage_sync_words(int M, int nlayers) {
  const int nmt = (M + 31) / 32;
  return 3 + 16 * nlayers + 2 * nmt * nlayers;
}

long long dense_stage_partial_floats(int M, int ksplit) {
  if (ksplit <= 1) return 0;
  const long long nmt = (M + 31) / 32;
  return 2LL * (2 * nmt) * (ksplit - 1) * NT * 8;
}

int dense_stage_default_ksplit(int M, int grid) {
  // Opt-in (round 6, bench.py A/B on one box, DenseNet-121 bs 256): stage 4 split 8 ways took its
  // older-channel accumulation from 12.9 to 2.6 us, but the finalizers then waited ~12 us for the
  // previous 3x3 phase instead -- the per-layer chain is the two hand-offs, not the accumulation
  // -- and the step went 3.46-3.48 -> 3.52-3.56 ms (stage 3 split 3 as well: 3.69-3.72 ms).
  const char* e = std::getenv("IDC_DS_KSPLIT");
  int ks = 1;
  if (e && e[0]) {
    ks = std::atoi(e);
  } else if (const char* t = std::getenv("IDC_DS_KSPLIT_TARGET")) {
    const int target = t[0] ? std::atoi(t) : (grid > 0 ? grid : 256);
    ks = target / (2 * ((M + 31) / 32));
  }
  return ks < 1 ? 1 : ks > DS_MAX_KSPLIT ? DS_MAX_KSPLIT : ks;
}

bool dense_stage_shape_ok(int N, int H, int W, int max_cin) {
  if (N < 1 || H < 1 || W < 1 || max_cin > DS_MAX_CIN) return false;
  const int HW = H * W, M = N * HW;
  for (int m0 = 0; m0 < M; m0 += 32) {  // rows staged by each 3x3 tile
    const int mend = m0 + 32 < M ? m0 + 32 : M;
    if ((((mend - 1) / HW) - m0 / HW + 1) * HW > DS_MAX_STAGE_ROWS) return false;
  }
  return true;
}

hipError_t dense_stage_fwd(const DenseStageArgs& a, int grid, hipStream_t st) {
  if (a.rows == 2) return dense_img_fwd(a, st);  // per-image training launch (dense_infer.hip)
  if (a.nlayers < 1 || (a.k2 != 1 && a.k2 != 3) || a.ld % 8 != 0 || a.N < 1 || a.H < 1 || a.W < 1 ||
      a.buf == nullptr || a.layers == nullptr || a.sync == nullptr ||
      (!a.infer && (a.sstats == nullptr || a.scratch == nullptr)) || !dense_stage_shape_ok(a.N, a.H, a.W, 0) ||
      a.ksplit > DS_MAX_KSPLIT || (a.ksplit > 1 && a.partials == nullptr))
    return hipErrorInvalidValue;
  if (a.rows && dense_rows_fwd(a, st) == hipSuccess) return hipSuccess;
  const int tasks = dense_stage_tasks(a);
  if (grid <= 0) grid = 256;
  // a grouped launch (K copies, each with its own queue) shares the CUs
  const int k = launch_groups().k;
  if (k > 1) grid = grid / k > 8 ? grid / k : 8;
  if (grid > tasks) grid = tasks;
  // the lookahead queue order lets an A phase wait on the B phase queued after it: it needs more
  // than nT (A tiles) workgroups of this queue resident at once, so it is used for one ungrouped
  // launch whose grid (one workgroup per CU, 2 fit) exceeds nT with margin (IDC_DS_LOOKAHEAD=0: off)
  static const bool la_on = [] {
    const char* e = std::getenv("IDC_DS_LOOKAHEAD");
    return !(e && e[0] == '0');
  }();
  // (split K: only the finalizers, one per A tile, wait on a later ticket -- their B phase)
  const int nT = 2 * ((a.N * a.H * a.W + 31) / 32);
  DenseStageArgs b = a;
  b.lookahead = (a.lookahead >= 0 && la_on && k == 1 && a.nlayers > 1 && grid >= nT + 16) ? 1 : 0;
  hipLaunchKernelGGL(dense_stage_kernel, ggrid(grid), dim3(NT), 0, st, b, garg());
  return hipGetLastError();
}

}  // namespace idc
