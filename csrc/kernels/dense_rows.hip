// Row-resident dense-stage forward for DenseNet (gfx950): every dense layer of a late stage in ONE
// launch in which each workgroup OWNS a group of whole images for the whole stage.
//
// A dense layer is  y = conv3x3(ReLU(BN2(conv1x1(ReLU(BN1(x[:, :cin]))))))  into channels
// [cin, cin+32) of the stage buffer (reference: the Keras DenseNet of
// /root/reference/dist_model_tf_dense.py:131-133).  Both convolutions are local to an
// image (1x1: per pixel; 3x3 'same': inside the image), so the only cross-workgroup dependencies of
// a layer are its two BatchNorms' BATCH statistics.  The work-queue launch (dense_stage.hip) hands
// every activation tile between workgroups through agent-coherent memory -- two data hand-offs per
// layer on the dependent chain, with tiles holding workgroups while they wait (round-6 stamps: stage
// 4 stays at ~12 us per layer even when the 1x1 accumulation is split 8 ways).  Here:
//
//   * workgroup g holds rows [g * ipg * HW, ...) -- ipg whole images, at most 16 * RB rows -- of the
//     stage buffer in LDS (raw bf16, channels [0, ld)) for the whole launch; a layer's new slice is
//     appended there and to the global stage buffer (for the consumers after the launch);
//   * per layer:  BN1 table -> act1 = relu(bn1(x)) staged in LDS -> 1x1 MFMA (wave w: t columns
//     16w..16w+15, weights streamed from L2 in 8-k-step chunks, the first chunk issued during the
//     previous layer's barrier) -> t (bf16) to LDS + global -> t statistics into slot copies ->
//     BARRIER 1 -> BN2 table from the slot sums -> act2 in LDS -> 3x3 MFMA (K split over the waves
//     of an output block, reduced in LDS; the 3x3 weight fragments were issued at the layer's start)
//     -> slice to LDS + global, slice statistics into slots -> BARRIER 2 -> the slice's mean / var;
//   * a barrier is a sharded arrival counter (persist.h publish_shard / wait_sum8): the only data
//     that crosses workgroups are the statistics slots (agent-coherent loads after the barrier).
// Inference-mode launches (a frozen base, evaluation: moving statistics) have no barrier at all.
// Workgroup 0 writes the single-copy statistics (t: tstats, slices: sstats) that the backward and
// the moving averages read after the launch; the last slice's are written by the last arrival.
// All workgroups must be co-resident (grid <= 256 at one workgroup per CU): the launcher checks.
#include "dense_stage.h"
#include "persist.h"

namespace idc {
namespace {

using namespace persist;

constexpr int NTR = 512;      // 8 waves
constexpr int TPR = 128 + 8;  // t / act2 row pitch (bf16)
constexpr int YP = 33;        // fp32 slice tile pitch
constexpr int S = DS_SLOTS;
constexpr int KC = 8;         // 1x1 weight chunk (k-steps of 32): two chunks = cin 512

struct RowsLayout {
  int xs, act1, tb, act2, red, ybuf, mean, var, sc, sh, lay, total;
};

__host__ __device__ inline RowsLayout rows_layout(int RB, int ld, int nlayers) {
  RowsLayout L{};
  const int R = 16 * RB, ldp = ld + 8;
  const int nblk = 2 * RB, wpb = 8 / nblk;
  int o = 0;
  L.xs = o;
  o += R * ldp * 2;
  L.act1 = o;
  // t, act2, the 3x3 partials and the slice tile alias act1 (dead once a layer's 1x1 is done)
  L.tb = o;
  L.act2 = L.tb + R * TPR * 2;
  L.red = L.act2 + (R + 1) * TPR * 2;
  L.ybuf = L.red + nblk * (wpb - 1) * 256 * 4;
  const int alias_end = L.ybuf + R * YP * 4;
  o += (R * ldp * 2 > alias_end - L.act1) ? R * ldp * 2 : alias_end - L.act1;
  // per-channel tables: the stage's channels, and bn2's 128 (a narrow test stage has ld < 128)
  const int tl = ld > 128 ? ld : 128;
  L.mean = o;
  o += tl * 4;
  L.var = o;
  o += tl * 4;
  L.sc = o;
  o += tl * 4;
  L.sh = o;
  o += tl * 4;
  L.lay = o;  // the layer table (LDS copy)
  o += nlayers * (int)sizeof(DenseLayerDesc);
  L.total = o;
  return L;
}

constexpr int LDS_MAX = 160 * 1024;

__device__ __forceinline__ v8bf bnr8(const uint4& x, const float* sc, const float* sh, float lo, float hi, bool keep) {
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

template <int RB>
__global__ __launch_bounds__(NTR) void dense_rows_kernel(DenseStageArgs a, GroupArg ga) {
  prefetch_kernargs<sizeof(DenseStageArgs) + sizeof(GroupArg)>();
  constexpr int R = 16 * RB;
  constexpr int NBLK = 2 * RB, WPB = 8 / NBLK;  // 3x3 output blocks (16 x 16), waves per block
  constexpr int MAXK2 = 36 / WPB;               // 3x3 k-steps per wave at most (9 taps x 4)
  const long long go = goff(ga);
  bf16_t* __restrict__ buf = gsh(a.buf, go);
  float* __restrict__ sstats = gsh(a.sstats, go);
  const float* __restrict__ sshift = gsh(a.sshift, go);
  const DenseLayerDesc* __restrict__ layers = gsh(a.layers, go);
  unsigned* sync = gsh(a.sync, go);
  auto cnt1 = [&](int l) { return sync + 1 + 16 * l; };  // t statistics of layer l complete
  auto cnt2 = [&](int l) { return sync + 9 + 16 * l; };  // slice statistics of layer l complete
  unsigned* lastfin = sync + 1 + 16 * a.nlayers;
  unsigned* fail = lastfin + 1;
  int* err = gsh(a.err, go);
  const persist::FailSink fsink{err, gsh(a.stepflag, go), a.hostflag};
  float* scratch = gsh(a.scratch, go);
  const unsigned max_polls = a.max_polls ? a.max_polls : DEFAULT_POLLS;
  unsigned long long* stamps = gsh(a.stamps, go);  // [layer][group][NSTAMP] (diagnostics)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const RowsLayout LY = rows_layout(RB, a.ld, a.nlayers);
  const int ld = a.ld, ldp = ld + 8;
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem + LY.xs);
  bf16_t* act1 = reinterpret_cast<bf16_t*>(smem + LY.act1);
  bf16_t* tb = reinterpret_cast<bf16_t*>(smem + LY.tb);
  bf16_t* act2 = reinterpret_cast<bf16_t*>(smem + LY.act2);
  float* red = reinterpret_cast<float*>(smem + LY.red);
  float* ybuf = reinterpret_cast<float*>(smem + LY.ybuf);
  float* s_mean = reinterpret_cast<float*>(smem + LY.mean);
  float* s_var = reinterpret_cast<float*>(smem + LY.var);
  float* s_sc = reinterpret_cast<float*>(smem + LY.sc);
  float* s_sh = reinterpret_cast<float*>(smem + LY.sh);
  DenseLayerDesc* s_lay = reinterpret_cast<DenseLayerDesc*>(smem + LY.lay);
  __shared__ int s_bad;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int HW = a.H * a.W, M = a.N * HW;
  const int G = (int)gridDim.x;
  const int gi = (int)blockIdx.x;
  const int row0 = gi * a.rows_ipg * HW;
  const int Rg = min(a.rows_ipg * HW, M - row0);
  const int c0 = layers[0].cin;
  const float inv_n = a.inv_count;
  const bool infer = a.infer != 0;
  const float lo1 = act_lo(a.act1), hi1 = act_hi(a.act1);
  const float lo2 = act_lo(a.act2), hi2 = act_hi(a.act2);
  const int taps = a.k2 * a.k2, pad = a.k2 >> 1, Kc = taps * 128, nks2 = taps * 4;

  {
    const int nw = a.nlayers * (int)sizeof(DenseLayerDesc) / 4;
    for (int i = tid; i < nw; i += NTR) reinterpret_cast<unsigned*>(s_lay)[i] = reinterpret_cast<const unsigned*>(layers)[i];
  }
  // ---- the group's rows of the stage input (channels [0, c0); the rest zero) and their moments
  for (int idx = tid; idx < R * (ld / 8); idx += NTR) {
    const int r = idx / (ld / 8), c = (idx - r * (ld / 8)) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < Rg && c < c0) v = *reinterpret_cast<const uint4*>(buf + (size_t)(row0 + r) * ld + c);
    *reinterpret_cast<uint4*>(xs + r * ldp + c) = v;
  }
  if (!infer)
    for (int c = tid; c < c0; c += NTR) {
      float mean, var;
      shifted_mean_var(sshift ? sshift[c] : 0.f, sstats[c], sstats[ld + c], inv_n, mean, var);
      s_mean[c] = mean;
      s_var[c] = var;
    }

  // this wave's 1x1 weight rows (t channel 16 * wid + fr) and its 3x3 output block / k share
  const int blk = wid / WPB, kp = wid - blk * WPB, rb = blk >> 1, cb = blk & 1;
  // image-local position of the lane's 3x3 A-fragment row (fixed for the launch)
  const int m_loc = rb * 16 + fr;
  int img_base = 0, ph = 0, pw = 0;
  {
    const int mm = m_loc < Rg ? m_loc : 0;
    const int img = mm / HW, rem = mm - img * HW;
    img_base = img * HW;
    ph = rem / a.W;
    pw = rem - ph * a.W;
  }

  v8bf wq[2][KC];  // 1x1 weight chunks (double buffer; the first two are issued a layer ahead)
  auto load_w1 = [&](const bf16_t* w1, int cin, int ch, v8bf (&q)[KC]) {
    const bf16_t* wrow = w1 + (size_t)(16 * wid + fr) * cin + fk;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int k = (ch * KC + i) * 32;
      q[i] = k < cin ? *reinterpret_cast<const v8bf*>(wrow + k) : v8bf{};
    }
  };
  // a layer's BN1 affine parameters of this thread's channels (tid + 512 j), issued a layer ahead
  constexpr int GJ = (DS_MAX_CIN + NTR - 1) / NTR;
  float g1r[GJ], b1r[GJ];
  auto prefetch_layer = [&](const DenseLayerDesc& dn) {
    load_w1(gsh(dn.w1, go), dn.cin, 0, wq[0]);
    load_w1(gsh(dn.w1, go), dn.cin, 1, wq[1]);
    const float* g = gsh(dn.g1, go);
    const float* b = gsh(dn.b1, go);
#pragma unroll
    for (int j = 0; j < GJ; ++j) {
      const int c = tid + NTR * j;
      g1r[j] = c < dn.cin ? g[c] : 0.f;
      b1r[j] = c < dn.cin ? b[c] : 0.f;
    }
  };
  prefetch_layer(layers[0]);

  for (int l = 0; l < a.nlayers; ++l) {
    __syncthreads();  // the previous layer's moments, slice rows and tile reads are complete
    const int sti = l * G + gi;  // stamp row
    stamp(stamps, sti, 0);
    const DenseLayerDesc d = s_lay[l];
    const int cin = d.cin, nks1 = cin >> 5, nch = (nks1 + KC - 1) / KC;
    const bf16_t* __restrict__ w1 = gsh(d.w1, go);
    const bf16_t* __restrict__ w2 = gsh(d.w2, go);
    const float* __restrict__ tsh = gsh(d.tshift, go);
    float* lslots = scratch + (size_t)l * DS_SCRATCH_PER_LAYER;  // [S][2][32] slice statistics
    float* tslots = lslots + S * 64;                              // [S][2][128] t statistics
    // 3x3 weight fragments of this wave's block and k share (issued once the t statistics are
    // published: in flight during the barrier)
    v8bf bw[MAXK2];
    auto load_w2 = [&]() {
#pragma unroll
      for (int i = 0; i < MAXK2; ++i) {
        const int ks = kp + WPB * i;
        bw[i] = ks < nks2 ? *reinterpret_cast<const v8bf*>(w2 + (size_t)(16 * cb + fr) * Kc + (ks >> 2) * 128 +
                                                           (ks & 3) * 32 + fk)
                          : v8bf{};
      }
    };

    // ---- BN1 table [0, cin) (batch moments, or the layer's moving statistics) and act1
    const bool inf1 = infer || (d.pad_ & 1);
    {
      const float* __restrict__ mm = inf1 ? gsh(d.mm1, go) : nullptr;
      const float* __restrict__ mv = inf1 ? gsh(d.mv1, go) : nullptr;
#pragma unroll
      for (int j = 0; j < GJ; ++j) {
        const int c = tid + NTR * j;
        if (c < cin) {
          const float mean = inf1 ? mm[c] : s_mean[c], var = inf1 ? mv[c] : s_var[c];
          const float r = g1r[j] * rsqrtf(var + d.eps1);
          s_sc[c] = r;
          s_sh[c] = b1r[j] - mean * r;
        }
      }
    }
    stamp(stamps, sti, 1);
    __syncthreads();  // tables; the previous layer's reads of the act1 region are done
    // act1: thread -> one 8-channel chunk (its scale / shift held in registers) x every 4th row
    for (int c8 = tid & 127; c8 < cin / 8; c8 += 128) {
      const int c = c8 * 8;
      const float4 a0 = *reinterpret_cast<const float4*>(s_sc + c), a1 = *reinterpret_cast<const float4*>(s_sc + c + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(s_sh + c), h1 = *reinterpret_cast<const float4*>(s_sh + c + 4);
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int rr = 0; rr < R / 4; ++rr) {
        const int r = (tid >> 7) + 4 * rr;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xs + r * ldp + c), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = r < Rg ? clampf(f[j] * av[j] + hv[j], lo1, hi1) : 0.f;
        *reinterpret_cast<uint4*>(act1 + r * ldp + c) = pack8(f);
      }
    }
    __syncthreads();
    stamp(stamps, sti, 2);

    // ---- 1x1: t[:, 16 wid .. +16) over all RB row blocks, weight chunks double-buffered
    v4f acc[RB];
#pragma unroll
    for (int h = 0; h < RB; ++h) acc[h] = v4f{0.f, 0.f, 0.f, 0.f};
    auto mfma1 = [&](int ch, const v8bf (&q)[KC]) {
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        const int ks = ch * KC + i;
        if (ks < nks1) {
#pragma unroll
          for (int h = 0; h < RB; ++h) {
            const v8bf af = *reinterpret_cast<const v8bf*>(act1 + (h * 16 + fr) * ldp + ks * 32 + fk);
            acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, q[i], acc[h], 0, 0, 0);
          }
        }
      }
    };
    // chunks 0 and 1 were issued a layer ahead; later chunks (cin > 1024) stream behind them
    for (int ch = 0; ch < nch; ch += 2) {
      mfma1(ch, wq[0]);
      if (ch + 2 < nch) load_w1(w1, cin, ch + 2, wq[0]);
      if (ch + 1 < nch) {
        mfma1(ch + 1, wq[1]);
        if (ch + 3 < nch) load_w1(w1, cin, ch + 3, wq[1]);
      }
    }
    __syncthreads();  // every wave done reading act1: t may overwrite it
    stamp(stamps, sti, 3);
    {
#pragma unroll
      for (int h = 0; h < RB; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = h * 16 + (lane >> 4) * 4 + q;
          tb[r * TPR + 16 * wid + fr] = (bf16_t)(pack2bf(acc[h][q], 0.f) & 0xffffu);
        }
      __syncthreads();
    }
    // t to global (16-B stores, rows of the group): after the barrier's publish, which need not
    // wait for them
    auto store_t = [&]() {
      bf16_t* tg = gsh(d.t, go);
      for (int idx = tid; idx < Rg * 16; idx += NTR) {
        const int r = idx >> 4, c = (idx & 15) * 8;
        *reinterpret_cast<uint4*>(tg + (size_t)(row0 + r) * 128 + c) = *reinterpret_cast<const uint4*>(tb + r * TPR + c);
      }
    };

    // ---- t statistics -> slots, barrier 1, BN2 table
    const bool inf2 = infer || (d.pad_ & 2);
    if (!infer) {
      if (tid < 256) {
        const int c = tid & 127, which = tid >> 7;
        const float k = tsh ? tsh[c] : 0.f;
        float sum = 0.f;
        for (int r = 0; r < Rg; ++r) {
          const float x = bf2f(tb[r * TPR + c]) - k;
          sum += which ? x * x : x;
        }
        atomicAdd(&tslots[(gi % S) * 256 + which * 128 + c], sum);
      }
      publish_shard(cnt1(l), gi);
      load_w2();
      store_t();
      if (wid == 0) {
        const bool ok = wait_sum8(cnt1(l), (unsigned)G, fail, fsink, max_polls);
        if (lane == 0) s_bad = !ok;
      }
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s_bad)) return;
    } else {
      load_w2();
      store_t();
    }
    stamp(stamps, sti, 4);
    if (tid < 128) {
      const int c = tid;
      const float g2 = gsh(d.g2, go)[c], b2 = gsh(d.b2, go)[c];
      float mean = 0.f, var = 1.f;
      if (!infer) {
        float s0, s1;
        slot_sum<S>(tslots, 128, c, s0, s1);
        if (gi == 0) {  // single copy: backward, moving averages
          float* tst = gsh(d.tstats, go);
          tst[c] = s0;
          tst[128 + c] = s1;
        }
        if (!inf2) shifted_mean_var(tsh ? tsh[c] : 0.f, s0, s1, inv_n, mean, var);
      }
      if (inf2) {
        mean = gsh(d.mm2, go)[c];
        var = gsh(d.mv2, go)[c];
      }
      const float r = g2 * rsqrtf(var + d.eps2);
      s_sc[c] = r;
      s_sh[c] = b2 - mean * r;
    }
    __syncthreads();
    // act2 = relu(bn2(t)) (+ the all-zero row R for padding taps and rows past the group)
    for (int idx = tid; idx < (R + 1) * 16; idx += NTR) {
      const int r = idx >> 4, c = (idx & 15) * 8;
      const uint4 x = r < R ? *reinterpret_cast<const uint4*>(tb + r * TPR + c) : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<v8bf*>(act2 + r * TPR + c) = bnr8(x, s_sc + c, s_sh + c, lo2, hi2, r < Rg);
    }
    __syncthreads();
    stamp(stamps, sti, 5);

    // ---- 3x3 (or centre tap): block (rb, cb) = rows 16 rb.., slice channels 16 cb..; k share kp
    {
      v4f acc2 = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MAXK2; ++i) {
        const int ks = kp + WPB * i;
        if (ks < nks2) {
          const int tap = ks >> 2, c = (ks & 3) * 32 + fk;
          const int kr = tap / a.k2, kc = tap - kr * a.k2;
          const int hh = ph + kr - pad, ww = pw + kc - pad;
          const bool ok = m_loc < Rg && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
          const int lrow = ok ? img_base + hh * a.W + ww : R;
          const v8bf af = *reinterpret_cast<const v8bf*>(act2 + lrow * TPR + c);
          acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[i], acc2, 0, 0, 0);
        }
      }
      if (WPB > 1 && kp > 0) *reinterpret_cast<v4f*>(red + ((blk * (WPB - 1) + kp - 1) * 64 + lane) * 4) = acc2;
      __syncthreads();
      if (kp == 0) {
#pragma unroll
        for (int j = 1; j < WPB; ++j) acc2 += *reinterpret_cast<const v4f*>(red + ((blk * (WPB - 1) + j - 1) * 64 + lane) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = rb * 16 + (lane >> 4) * 4 + q;
          const uint32_t p = pack2bf(acc2[q], 0.f);
          ybuf[r * YP + cb * 16 + fr] = __uint_as_float(p << 16);  // the bf16-rounded value
        }
      }
      __syncthreads();
    }
    stamp(stamps, sti, 6);
    // ---- the slice: LDS rows (later layers), global stage buffer (after the barrier's publish),
    // statistics
    for (int idx = tid; idx < Rg * 4; idx += NTR) {
      const int r = idx >> 2, c = (idx & 3) * 8;
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = ybuf[r * YP + c + j];
      *reinterpret_cast<uint4*>(xs + r * ldp + cin + c) = pack8(f);
    }
    auto store_slice = [&]() {
      for (int idx = tid; idx < Rg * 4; idx += NTR) {
        const int r = idx >> 2, c = (idx & 3) * 8;
        *reinterpret_cast<uint4*>(buf + (size_t)(row0 + r) * ld + cin + c) =
            *reinterpret_cast<const uint4*>(xs + r * ldp + cin + c);
      }
    };
    if (!infer) {
      if (tid < 64) {
        const int c = tid & 31, which = tid >> 5;
        const float k = sshift ? sshift[cin + c] : 0.f;
        float sum = 0.f;
        for (int r = 0; r < Rg; ++r) {
          const float x = ybuf[r * YP + c] - k;
          sum += which ? x * x : x;
        }
        atomicAdd(&lslots[(gi % S) * 64 + which * 32 + c], sum);
      }
      if (l + 1 < a.nlayers) {
        __syncthreads();  // the slice rows in LDS (store_slice reads them)
        publish_shard(cnt2(l), gi);
        // the next layer's first weight chunks and BN1 parameters, in flight while this barrier waits
        prefetch_layer(s_lay[l + 1]);
        store_slice();
        if (wid == 0) {
          const bool ok = wait_sum8(cnt2(l), (unsigned)G, fail, fsink, max_polls);
          if (lane == 0) s_bad = !ok;
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s_bad)) return;
        stamp(stamps, sti, 7);
        if (tid < 32) {
          float s0, s1, mean, var;
          slot_sum<S>(lslots, 32, tid, s0, s1);
          shifted_mean_var(sshift ? sshift[cin + tid] : 0.f, s0, s1, inv_n, mean, var);
          s_mean[cin + tid] = mean;
          s_var[cin + tid] = var;
          if (gi == 0) {
            sstats[cin + tid] = s0;
            sstats[ld + cin + tid] = s1;
          }
        }
      } else {
        // the last slice has no in-launch consumer: the last arrival writes its statistics
        __syncthreads();
        store_slice();
        const unsigned old = publish(lastfin);
        if (tid == 0) s_bad = old == (unsigned)(G - 1);
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s_bad) && tid < 32) {
          float s0, s1;
          slot_sum<S>(lslots, 32, tid, s0, s1);
          sstats[cin + tid] = s0;
          sstats[ld + cin + tid] = s1;
        }
      }
    } else {
      __syncthreads();
      store_slice();
      if (l + 1 < a.nlayers) prefetch_layer(s_lay[l + 1]);
    }
  }
}

// images per group and row blocks for a stage: one 16-row block per workgroup where it holds an
// image (round 6: stage 3 of DenseNet-121 at bs 256, 256 workgroups of one image, 382 us against
// 519 us with two row blocks -- 86 workgroups, spills, a longer 3x3 and barrier), every workgroup
// resident at once (grid <= 256); IDC_DS_ROWS_RB=1|2 forces the row blocks
bool dense_rows_geometry(int N, int H, int W, int ld, int max_cin, int& rb, int& ipg, int& grid) {
  const int HW = H * W;
  if (ld % 32 || max_cin > ld - 32 || max_cin > DS_MAX_CIN) return false;
  const char* e = std::getenv("IDC_DS_ROWS_RB");
  const int force = (e && e[0]) ? std::atoi(e) : 0;
  for (int r = 1; r <= 2; ++r) {
    if (force && r != force) continue;
    const int ip = 16 * r / HW;
    if (ip < 1) continue;
    if (rows_layout(r, ld, 64).total > LDS_MAX) continue;
    const int g = (N + ip - 1) / ip;
    if (g > 256) continue;
    rb = r;
    ipg = ip;
    grid = g;
    return true;
  }
  return false;
}

hipError_t dense_rows_fwd(const DenseStageArgs& a, hipStream_t st) {
  int rb = 0, ipg = 0, grid = 0;
  // (the builder validated the layer table host-side: cin = c0 + 32 l < ld)
  const int max_cin = a.ld - 32;
  if (!dense_rows_geometry(a.N, a.H, a.W, a.ld, max_cin, rb, ipg, grid) || launch_groups().k > 1)
    return hipErrorInvalidValue;
  DenseStageArgs b = a;
  b.rows_ipg = ipg;
  if (a.nlayers > 64) return hipErrorInvalidValue;
  const int shm = rows_layout(rb, a.ld, a.nlayers).total;
  if (rb == 2)
    hipLaunchKernelGGL(dense_rows_kernel<2>, ggrid(grid), dim3(NTR), shm, st, b, garg());
  else
    hipLaunchKernelGGL(dense_rows_kernel<1>, ggrid(grid), dim3(NTR), shm, st, b, garg());
  return hipGetLastError();
}

}  // namespace idc
