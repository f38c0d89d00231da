// A whole DenseNet dense block in inference mode as ONE launch, gfx950 (dense_stage.h).
//
// Inference (evaluation, the frozen base of phase 1, the frozen stages of the fine-tune phase)
// turns every BatchNorm into a constant per-channel affine, so a dense layer of one image depends
// on nothing but that image: a workgroup owns `ipg` whole images, stages their block input (the
// stage buffer's first c0 channels) into an LDS concat buffer and runs all L layers there:
//   GEMM1  t  = (ReLU(bn1(cat[:, :cin]))) . W1^T       MFMA 16x16x32, the BN1 affine + ReLU applied
//                                                       to each A fragment as it is read (each layer
//                                                       has its own BN1 over the same raw channels)
//          z2 = ReLU(bn2(t)) -> a zero-bordered (H+2) x (W+2) grid per image in LDS
//   GEMM2  n  = conv3x3(z2) . W2^T                      MFMA, A rows read straight from the padded
//                                                       grid (no bounds checks), K = 9 taps x 128
//          cat[:, cin:cin+32] = n (raw: later layers' BN1 normalise it)
// and finally writes the new 32 L channels of its images to the stage buffer once.  No statistics,
// no grid barriers, no global round trips between layers.  Each wave holds its N tile's W1
// fragments (16 K steps at a time) and its W2 fragments (two halves of 18) in registers, loaded
// once per layer; the next layer's BN tables are written while the 3x3 runs.  The per-layer path it
// replaces runs 2 launches per layer (36 for stages 1-2 of DenseNet-121 at 50x50: ~390 us of the
// frozen-base step against 143 + 215 us here, profiles/densenet121_frozen_dense_infer_*).  On the
// 3x3 / 1x1 maps of stages 3-4 (a <2, 24> instantiation, centre tap only on 1x1) it is correct but
// slower than the row-resident / work-queue launches, so those stay the default there.
//
// TRAINING mode (dense_img_fwd, DenseStageArgs::rows == 2: stages 1-2 of DenseNet-121 at 50x50,
// 13x13 / 6x6 images that the row-resident launch of dense_rows.hip cannot hold): the same
// per-image data flow, with the two BatchNorms on BATCH statistics.  Those are the only data that
// cross workgroups: after GEMM1 the raw t (bf16) goes to the z2 grid and to global memory (the
// backward's operand), the workgroup's shifted t moments go to slot copies, one sharded barrier,
// BN2 from the slot sums, then BN2 + ReLU in place over the grid; after GEMM2 the slice's moments
// go to slot copies, a second barrier, and the next layer's BN1 table takes their mean / variance.
// It writes exactly what the per-layer convs write (t, tstats, the stage buffer, sstats), so the
// backward is unchanged.  Every workgroup must be co-resident (grid <= 256: one image each at
// batch 256); a wait that outlives max_polls gives up through the fail flag (persist.h).
// Reference: the dense blocks of dist_model_tf_dense.py:131-133 (inference passes).
#include "dense_stage.h"
#include "persist.h"

namespace idc {

namespace {

constexpr int NT = 512, NW = NT / 64;
constexpr int ZS = 128 + 8;    // z2 grid row stride (elements)
// two instantiations: <12, 16> (up to 12 M tiles = 192 rows; GEMM1 B fragments in chunks of 16 K
// steps = 512 channels) for the large maps, <2, 24> (32 rows; 768 channels of B fragments in one
// memory latency; 32 steps spill) for the small ones
constexpr int BIG_MT = 12, BIG_KS = 16, SMALL_MT = 2, SMALL_KS = 24;
constexpr int MAXCT = 2048;    // widest stage (concat channels)

struct DiGeo {
  int HW, P, RP, MT, CT, CS, GW, GP;
};
__host__ __device__ inline DiGeo di_geo(const DenseInferArgs& a) {
  DiGeo g;
  g.HW = a.H * a.W;
  g.P = a.ipg * g.HW;
  g.MT = (g.P + 15) / 16;
  g.RP = g.MT * 16;
  g.CT = a.c0 + 32 * a.L;
  g.CS = g.CT + 8;
  g.GW = a.W + 2;
  g.GP = (a.H + 2) * g.GW;
  return g;
}
// (training launches add the stage channels' batch mean / variance: 2 CT floats)
__host__ __device__ inline long long di_bytes(const DenseInferArgs& a, const DiGeo& g, bool train) {
  return (long long)g.RP * g.CS * 2 + (long long)a.ipg * g.GP * ZS * 2 + (2LL * g.CT + 256 + g.RP) * 4 +
         (train ? 8LL * g.CT : 0);
}

// training-mode extras of a launch (dense_img_fwd fills them from DenseStageArgs)
struct DiTrain {
  float* sstats;          // [2][ld] shifted statistics of the stage buffer (single copy)
  const float* sshift;    // [ld] (nullable)
  unsigned* sync;         // dense_rows.hip layout: [1 + 16 l] t counters, [9 + 16 l] slice counters,
                          // [1 + 16 L] last-slice arrivals, then the fail flag
  float* scratch;         // [L][DS_SCRATCH_PER_LAYER] statistics slots (zeroed per step)
  persist::FailSink fs;
  float inv_n;
  unsigned max_polls;
  unsigned long long* stamps;  // nullable: NSTAMP s_memrealtime stamps per (layer, workgroup)
};

__device__ __forceinline__ v8bf ld_frag(const bf16_t* p) { return *reinterpret_cast<const v8bf*>(p); }

// BN tables of layer e: sc1/sf1 over its cin input channels, sc2/sf2 over the 128 bottleneck
// channels.  Every load of the thread's (up to TU) channels is issued before any is used, so the
// tables cost one memory latency at every width (a plain strided loop pays one per 512 channels).
__device__ __forceinline__ void layer_tables(const DenseLayerDesc& e, float* sc1, float* sf1, float* sc2,
                                             float* sf2, int tid) {
  constexpr int TU = (MAXCT + 128 + NT - 1) / NT;
  const int n = e.cin + 128;
  float gg[TU], bb[TU], mm[TU], vv[TU];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int c = tid + u * NT;
    gg[u] = 1.f; bb[u] = 0.f; mm[u] = 0.f; vv[u] = 1.f;
    if (c < e.cin) {
      if (e.g1) gg[u] = e.g1[c];
      if (e.b1) bb[u] = e.b1[c];
      mm[u] = e.mm1[c]; vv[u] = e.mv1[c];
    } else if (c < n) {
      const int k = c - e.cin;
      if (e.g2) gg[u] = e.g2[k];
      if (e.b2) bb[u] = e.b2[k];
      mm[u] = e.mm2[k]; vv[u] = e.mv2[k];
    }
  }
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int c = tid + u * NT;
    if (c >= n) continue;
    const float sc = gg[u] * rsqrtf(vv[u] + (c < e.cin ? e.eps1 : e.eps2));
    const float sf = bb[u] - mm[u] * sc;
    if (c < e.cin) { sc1[c] = sc; sf1[c] = sf; }
    else { sc2[c - e.cin] = sc; sf2[c - e.cin] = sf; }
  }
}

// training mode: BN1 table of layer e over [0, cin) from the stage channels' batch moments in LDS
// (a frozen layer inside a trained stage, pad_ bit 0: its moving statistics); loads first
__device__ __forceinline__ void bn1_table_train(const DenseLayerDesc& e, const float* s_mean, const float* s_var,
                                                float* sc1, float* sf1, int tid) {
  constexpr int TU = (MAXCT + NT - 1) / NT;
  const bool mov = e.pad_ & 1;
  float gg[TU], bb[TU], mm[TU], vv[TU];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int c = tid + u * NT;
    gg[u] = 1.f; bb[u] = 0.f; mm[u] = 0.f; vv[u] = 1.f;
    if (c < e.cin) {
      if (e.g1) gg[u] = e.g1[c];
      if (e.b1) bb[u] = e.b1[c];
      mm[u] = mov ? e.mm1[c] : s_mean[c];
      vv[u] = mov ? e.mv1[c] : s_var[c];
    }
  }
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int c = tid + u * NT;
    if (c >= e.cin) continue;
    const float sc = gg[u] * rsqrtf(vv[u] + e.eps1);
    sc1[c] = sc;
    sf1[c] = bb[u] - mm[u] * sc;
  }
}

}  // namespace

template <int MAXMT, int MAXKS, bool TRAIN>
__device__ __forceinline__ void dense_block(const DenseInferArgs& a, const DiTrain& tr) {
  using namespace persist;
  constexpr int MAXG2 = (2 * MAXMT + NW - 1) / NW;  // GEMM2 tiles per wave
  constexpr int S = DS_SLOTS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const DiGeo g = di_geo(a);
  bf16_t* Cat = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Z2 = Cat + g.RP * g.CS;
  float* sc1 = reinterpret_cast<float*>(Z2 + a.ipg * g.GP * ZS);
  float* sf1 = sc1 + g.CT;
  float* sc2 = sf1 + g.CT;
  float* sf2 = sc2 + 128;
  // per row: the top-left cell of its 3x3 window in the padded z2 grid (its own cell is + GW + 1);
  // read from LDS where needed rather than kept in registers across the layer loop
  int* gtl = reinterpret_cast<int*>(sf2 + 128);
  float* s_mean = reinterpret_cast<float*>(gtl + g.RP);  // (training) batch moments of the stage
  float* s_var = s_mean + g.CT;
  float* red = sc1;  // (training) moment partials: sc1 / sf1 (>= 512 floats) are dead while in use
  __shared__ int s_bad;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img0 = blockIdx.x * a.ipg;
  const int nimg = min(a.ipg, a.N - img0);
  const int pv = nimg * g.HW;  // valid rows
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  const float lo = act_lo(a.act), hi = act_hi(a.act);
  const int gi = (int)blockIdx.x, G = (int)gridDim.x;
  const int row0 = img0 * g.HW;

  // ---- stage the block input, zero the z2 grids (their borders are the 3x3's padding)
  {
    const int C8 = a.c0 / 8, nx = g.RP * C8;
    constexpr int U = 8;
    for (int base = 0; base < nx; base += U * NT) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        const int p = i / C8, c = (i - p * C8) * 8;
        v[u] = (i < nx && p < pv)
                   ? *reinterpret_cast<const uint4*>(a.buf + ((size_t)img0 * g.HW + p) * a.ld + c)
                   : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        if (i < nx) {
          const int p = i / C8, c = (i - p * C8) * 8;
          *reinterpret_cast<uint4*>(Cat + p * g.CS + c) = v[u];
        }
      }
    }
    const int nz = a.ipg * g.GP * ZS / 8;
    for (int i = tid; i < nz; i += NT) reinterpret_cast<uint4*>(Z2)[i] = make_uint4(0, 0, 0, 0);
    for (int row = tid; row < g.RP; row += NT) {
      const int rr = row < pv ? row : 0;
      const int im = rr / g.HW, rem = rr - im * g.HW, h = rem / a.W, w = rem - h * a.W;
      gtl[row] = im * g.GP + h * g.GW + w;
    }
  }

  // 3x3 on 1x1 maps (stage 4 at 50x50): only the centre tap sees data, and w2 is the centre
  // slice [32][128] (dense_stage.h DenseLayerDesc::w2, k2 = 1)
  const bool c1 = a.H == 1 && a.W == 1;
  // BN tables of layer 0; those of layer l + 1 are written during layer l's GEMM2 (the tables are
  // last read by GEMM1 and its epilogue), so a layer costs two barriers
  if constexpr (TRAIN) {
    for (int c = tid; c < a.c0; c += NT)
      shifted_mean_var(tr.sshift ? tr.sshift[c] : 0.f, tr.sstats[c], tr.sstats[a.ld + c], tr.inv_n, s_mean[c], s_var[c]);
    __syncthreads();
    bn1_table_train(a.layers[0], s_mean, s_var, sc1, sf1, tid);
  } else {
    layer_tables(a.layers[0], sc1, sf1, sc2, sf2, tid);
  }
  __syncthreads();

  for (int l = 0; l < a.L; ++l) {
    const DenseLayerDesc& d = a.layers[l];
    const int cin = d.cin;
    const bf16_t* __restrict__ w1 = d.w1;
    const bf16_t* __restrict__ w2 = d.w2;
    if constexpr (TRAIN) stamp(tr.stamps, l * G + gi, 0);

    // ---- GEMM1: t = z1 . W1^T.  Wave w owns N tile w (16 of the 128 bottleneck channels) over
    // every M tile, so its B fragments -- all K steps of one 16-row slice of W1 -- are loaded ONCE
    // per layer (one memory latency, issued with the tables) instead of streamed per K step
    {
      const int KS = cin / 32;
      v4f acc[MAXMT];
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) acc[mt] = (v4f){0.f, 0.f, 0.f, 0.f};
      // chunks of MAXKS K steps (one chunk up to cin 512; stages 3-4 take two)
      for (int kc = 0; kc < KS; kc += MAXKS) {
      v8bf bw[MAXKS];
#pragma unroll
      for (int ks = 0; ks < MAXKS; ++ks)
        if (kc + ks < KS) bw[ks] = ld_frag(w1 + (size_t)(wid * 16 + frow) * cin + (kc + ks) * 32 + fk);
#pragma unroll
      for (int ks = 0; ks < MAXKS; ++ks) {
        if (kc + ks < KS) {
          const int k0 = (kc + ks) * 32 + fk;
          const float4 s0 = *reinterpret_cast<const float4*>(sc1 + k0);
          const float4 s1 = *reinterpret_cast<const float4*>(sc1 + k0 + 4);
          const float4 f0 = *reinterpret_cast<const float4*>(sf1 + k0);
          const float4 f1 = *reinterpret_cast<const float4*>(sf1 + k0 + 4);
          const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sfv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
          for (int mt = 0; mt < MAXMT; ++mt) {
            if (mt < g.MT) {
              float x[8];
              unpack8(*reinterpret_cast<const uint4*>(Cat + (mt * 16 + frow) * g.CS + k0), x);
#pragma unroll
              for (int q = 0; q < 8; ++q) x[q] = clampf(fmaf(x[q], scv[q], sfv[q]), lo, hi);
              const v8bf af = __builtin_bit_cast(v8bf, pack8(x));
              acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[ks], acc[mt], 0, 0, 0);
            }
          }
          // (keeps the scheduler from hoisting every step's A fragments into registers at once)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      }
      const int col = wid * 16 + frow;
      const float s2 = TRAIN ? 1.f : sc2[col], f2 = TRAIN ? 0.f : sf2[col];
      const float tk = (TRAIN && d.tshift) ? d.tshift[col] : 0.f;
      float ps = 0.f, pq = 0.f;  // (training) shifted moments of the lane's t values
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) {
        if (mt >= g.MT) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row >= pv) continue;
          if constexpr (TRAIN) {
            // the raw t (BN2 needs the whole batch's moments first), its moments from the
            // bf16-rounded value the backward will read
            const bf16_t tb = f2bf(acc[mt][q]);
            Z2[(size_t)(gtl[row] + g.GW + 1) * ZS + col] = tb;
            const float x = bf2f(tb) - tk;
            ps += x;
            pq = fmaf(x, x, pq);
          } else {
            Z2[(size_t)(gtl[row] + g.GW + 1) * ZS + col] = f2bf(clampf(fmaf(acc[mt][q], s2, f2), lo, hi));
          }
        }
      }
      if constexpr (TRAIN) {
        // column sums over the wave's 4 row groups; lanes 0-15 add the sums, 16-31 the squares
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
        pq += __shfl_xor(pq, 16, 64);
        pq += __shfl_xor(pq, 32, 64);
        float* tslots = tr.scratch + (size_t)l * DS_SCRATCH_PER_LAYER + S * 64;
        if (lane < 32) atomicAdd(&tslots[(gi % S) * 256 + (lane >> 4) * 128 + col], lane < 16 ? ps : pq);
      }
    }
    __syncthreads();

    if constexpr (TRAIN) {
      stamp(tr.stamps, l * G + gi, 1);
      // ---- (the t moments went to the slot copies in GEMM1's epilogue) t -> global; barrier 1
      float* lslots = tr.scratch + (size_t)l * DS_SCRATCH_PER_LAYER;  // [S][2][32] slice moments
      float* tslots = lslots + S * 64;                                 // [S][2][128] t moments
      const float* __restrict__ tsh = d.tshift;
      {
        bf16_t* tg = d.t;
        for (int i = tid; i < pv * 16; i += NT) {
          const int r = i >> 4, c = (i & 15) * 8;
          *reinterpret_cast<uint4*>(tg + (size_t)(row0 + r) * 128 + c) =
              *reinterpret_cast<const uint4*>(Z2 + (size_t)(gtl[r] + g.GW + 1) * ZS + c);
        }
      }
      publish_shard(tr.sync + 1 + 16 * l, gi);
      stamp(tr.stamps, l * G + gi, 2);
      if (wid == 0) {
        const bool ok = wait_sum8(tr.sync + 1 + 16 * l, (unsigned)G, tr.sync + 2 + 16 * a.L, tr.fs, tr.max_polls);
        if (lane == 0) s_bad = !ok;
      }
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane(s_bad)) return;
      stamp(tr.stamps, l * G + gi, 3);
      if (tid < 128) {
        const int c = tid;
        float s0, s1, mean, var;
        slot_sum<S>(tslots, 128, c, s0, s1);
        if (gi == 0) {  // single copy: backward, moving averages
          d.tstats[c] = s0;
          d.tstats[128 + c] = s1;
        }
        if (d.pad_ & 2) {
          mean = d.mm2[c];
          var = d.mv2[c];
        } else {
          shifted_mean_var(tsh ? tsh[c] : 0.f, s0, s1, tr.inv_n, mean, var);
        }
        const float sc = (d.g2 ? d.g2[c] : 1.f) * rsqrtf(var + d.eps2);
        sc2[c] = sc;
        sf2[c] = (d.b2 ? d.b2[c] : 0.f) - mean * sc;
      }
      __syncthreads();
      // BN2 + ReLU in place over the grid's image cells (the zero border stays zero)
      for (int i = tid; i < pv * 16; i += NT) {
        const int r = i >> 4, c = (i & 15) * 8;
        uint4* p = reinterpret_cast<uint4*>(Z2 + (size_t)(gtl[r] + g.GW + 1) * ZS + c);
        float f[8];
        unpack8(*p, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = clampf(fmaf(f[j], sc2[c + j], sf2[c + j]), lo, hi);
        *p = pack8(f);
      }
      __syncthreads();
      stamp(tr.stamps, l * G + gi, 4);
    }

    // ---- GEMM2: n = conv3x3(z2) . W2^T (tiles wid + 8 j, all of one N tile), epilogue into cat
    if (c1) {
      const int nt = wid & 1;
      const bf16_t* __restrict__ wrow = w2 + (size_t)(nt * 16 + frow) * 128 + fk;
      v8bf wc[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wc[kk] = ld_frag(wrow + kk * 32);
      if (!TRAIN && l + 1 < a.L) layer_tables(a.layers[l + 1], sc1, sf1, sc2, sf2, tid);
#pragma unroll
      for (int j = 0; j < MAXG2; ++j) {
        const int mt = (wid + NW * j) >> 1;
        if (mt >= g.MT) continue;
        const int zc = gtl[mt * 16 + frow] + g.GW + 1;
        v4f acc = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_frag(Z2 + (size_t)zc * ZS + kk * 32 + fk), wc[kk], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row < pv) Cat[row * g.CS + cin + nt * 16 + frow] = f2bf(acc[q]);
        }
      }
    } else {
      const int nt = wid & 1;
      // the 3x3's B fragments of this wave's N tile, in two halves of 18 K steps: the second half
      // is issued once the first 9 steps have consumed their fragments (27 in registers at most)
      const bf16_t* __restrict__ wrow = w2 + (size_t)(nt * 16 + frow) * 1152 + fk;
      v8bf w2f[36];
#pragma unroll
      for (int kk = 0; kk < 18; ++kk) w2f[kk] = ld_frag(wrow + kk * 32);
      if (!TRAIN && l + 1 < a.L) layer_tables(a.layers[l + 1], sc1, sf1, sc2, sf2, tid);
      v4f acc[MAXG2];
      int gb[MAXG2];
#pragma unroll
      for (int j = 0; j < MAXG2; ++j) {
        acc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
        const int mt = (wid + NW * j) >> 1;
        gb[j] = mt < g.MT ? gtl[mt * 16 + frow] : 0;  // top-left of the 3x3 window
      }
#pragma unroll
      for (int kk = 0; kk < 36; ++kk) {
        if (kk == 9) {
#pragma unroll
          for (int k2 = 18; k2 < 36; ++k2) w2f[k2] = ld_frag(wrow + k2 * 32);
        }
        const int tap = kk >> 2, cc = (kk & 3) * 32;
        const int r = tap / 3, s = tap - r * 3;
#pragma unroll
        for (int j = 0; j < MAXG2; ++j) {
          if (((wid + NW * j) >> 1) < g.MT) {
            const v8bf af = ld_frag(Z2 + (size_t)(gb[j] + r * g.GW + s) * ZS + cc + fk);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, w2f[kk], acc[j], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      const float yk = (TRAIN && tr.sshift) ? tr.sshift[cin + nt * 16 + frow] : 0.f;
      float ps = 0.f, pq = 0.f;  // (training) shifted moments of the lane's slice values
#pragma unroll
      for (int j = 0; j < MAXG2; ++j) {
        const int mt = (wid + NW * j) >> 1;
        if (mt >= g.MT) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row < pv) {
            const bf16_t yb = f2bf(acc[j][q]);
            Cat[row * g.CS + cin + nt * 16 + frow] = yb;
            if constexpr (TRAIN) {
              const float x = bf2f(yb) - yk;
              ps += x;
              pq = fmaf(x, x, pq);
            }
          }
        }
      }
      if constexpr (TRAIN) {
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
        pq += __shfl_xor(pq, 16, 64);
        pq += __shfl_xor(pq, 32, 64);
        if (lane < 32) red[wid * 32 + lane] = lane < 16 ? ps : pq;  // [wave][sum | sumsq][16]
      }
    }
    __syncthreads();

    if constexpr (TRAIN) {
      // ---- slice moments -> slot copies; barrier 2; the slice's mean / variance for later BN1s
      stamp(tr.stamps, l * G + gi, 5);
      float* lslots = tr.scratch + (size_t)l * DS_SCRATCH_PER_LAYER;
      if (tid < 64) {  // channel c of the slice: the waves of its N tile (wid & 1 == c / 16)
        const int c = tid & 31, which = tid >> 5;
        float sum = 0.f;
#pragma unroll
        for (int w = 0; w < NW / 2; ++w) sum += red[(2 * w + (c >> 4)) * 32 + which * 16 + (c & 15)];
        atomicAdd(&lslots[(gi % S) * 64 + which * 32 + c], sum);
      }
      if (l + 1 < a.L) {
        publish_shard(tr.sync + 9 + 16 * l, gi);
        stamp(tr.stamps, l * G + gi, 6);
        if (wid == 0) {
          const bool ok = wait_sum8(tr.sync + 9 + 16 * l, (unsigned)G, tr.sync + 2 + 16 * a.L, tr.fs, tr.max_polls);
          if (lane == 0) s_bad = !ok;
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s_bad)) return;
        if (tid < 32) {
          float s0, s1;
          slot_sum<S>(lslots, 32, tid, s0, s1);
          shifted_mean_var(tr.sshift ? tr.sshift[cin + tid] : 0.f, s0, s1, tr.inv_n, s_mean[cin + tid], s_var[cin + tid]);
          if (gi == 0) {
            tr.sstats[cin + tid] = s0;
            tr.sstats[a.ld + cin + tid] = s1;
          }
        }
        __syncthreads();
        bn1_table_train(a.layers[l + 1], s_mean, s_var, sc1, sf1, tid);
        __syncthreads();
        stamp(tr.stamps, l * G + gi, 7);
      } else {
        // the last slice has no in-launch consumer: the last arrival writes its statistics
        const unsigned old = publish(tr.sync + 1 + 16 * a.L);
        if (tid == 0) s_bad = old == (unsigned)(G - 1);
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s_bad) && tid < 32) {
          float s0, s1;
          slot_sum<S>(lslots, 32, tid, s0, s1);
          tr.sstats[cin + tid] = s0;
          tr.sstats[a.ld + cin + tid] = s1;
        }
      }
    }
  }

  // ---- the block's new channels to the stage buffer
  {
    const int N8 = 4 * a.L, nx = pv * N8;
    for (int i = tid; i < nx; i += NT) {
      const int p = i / N8, c = a.c0 + (i - p * N8) * 8;
      *reinterpret_cast<uint4*>(a.buf + ((size_t)img0 * g.HW + p) * a.ld + c) =
          *reinterpret_cast<const uint4*>(Cat + p * g.CS + c);
    }
  }
}

template <int MAXMT, int MAXKS>
__global__ __launch_bounds__(NT) void dense_infer_kernel(DenseInferArgs a) {
  dense_block<MAXMT, MAXKS, false>(a, DiTrain{});
}
template <int MAXMT, int MAXKS>
__global__ __launch_bounds__(NT) void dense_img_kernel(DenseInferArgs a, DiTrain t) {
  dense_block<MAXMT, MAXKS, true>(a, t);
}

static long long di_smem(const DenseInferArgs& a, bool train) {
  if (a.N < 1 || a.ipg < 1 || a.L < 1 || a.H < 1 || a.W < 1) return -1;
  if (a.c0 % 32 || a.ld % 8 || a.c0 + 32 * a.L > a.ld) return -1;
  if ((uintptr_t)a.buf % 16) return -1;
  const DiGeo g = di_geo(a);
  if (g.MT > BIG_MT) return -1;
  if (g.CT > MAXCT) return -1;
  const long long b = di_bytes(a, g, train);
  return b <= 160 * 1024 ? b : -1;
}

long long dense_infer_smem(const DenseInferArgs& a) { return di_smem(a, false); }

// training-mode launch geometry of a stage (DenseStageArgs::rows == 2): images per workgroup so the
// grid stays co-resident (<= 256 workgroups, one per CU), and the launch's dynamic LDS (-1: no fit)
static long long dense_img_geometry(const DenseStageArgs& s, DenseInferArgs& a) {
  a = DenseInferArgs{};
  a.buf = s.buf;
  a.ld = s.ld;
  a.N = s.N;
  a.H = s.H;
  a.W = s.W;
  a.L = s.nlayers;
  a.c0 = s.ld - 32 * s.nlayers;  // (the builder checks: the stage buffer is exactly c0 + 32 L wide)
  a.act = s.act1;
  a.ipg = (s.N + 255) / 256;
  a.layers = s.layers;
  if (a.c0 < 32 || s.k2 != 3 || s.act1 != s.act2 || s.infer || a.H * a.W <= 1) return -1;
  if (2 * a.ld < 512) return -1;  // the moment partials alias sc1 / sf1
  return di_smem(a, true);
}

bool dense_img_ok(const DenseStageArgs& s) {
  DenseInferArgs a;
  return dense_img_geometry(s, a) > 0;
}

hipError_t dense_img_fwd(const DenseStageArgs& s, hipStream_t st) {
  DenseInferArgs a;
  const long long smem = dense_img_geometry(s, a);
  if (smem < 0 || launch_groups().k > 1 || s.sstats == nullptr || s.scratch == nullptr || s.sync == nullptr)
    return hipErrorInvalidValue;
  DiTrain t{};
  t.sstats = s.sstats;
  t.sshift = s.sshift;
  t.sync = s.sync;
  t.scratch = s.scratch;
  t.fs = persist::FailSink{s.err, s.stepflag, s.hostflag};
  t.inv_n = s.inv_count;
  t.max_polls = s.max_polls ? s.max_polls : persist::DEFAULT_POLLS;
  t.stamps = s.stamps;
  const DiGeo g = di_geo(a);
  const dim3 grid((a.N + a.ipg - 1) / a.ipg);
  if (g.MT <= SMALL_MT)
    hipLaunchKernelGGL((dense_img_kernel<SMALL_MT, SMALL_KS>), grid, dim3(NT), (size_t)smem, st, a, t);
  else
    hipLaunchKernelGGL((dense_img_kernel<BIG_MT, BIG_KS>), grid, dim3(NT), (size_t)smem, st, a, t);
  return hipGetLastError();
}

hipError_t dense_infer(const DenseInferArgs& a, hipStream_t st) {
  const long long smem = dense_infer_smem(a);
  if (smem < 0) return hipErrorInvalidValue;
  const DiGeo g = di_geo(a);
  const dim3 grid((a.N + a.ipg - 1) / a.ipg);
  if (g.MT <= SMALL_MT)
    hipLaunchKernelGGL((dense_infer_kernel<SMALL_MT, SMALL_KS>), grid, dim3(NT), (size_t)smem, st, a);
  else
    hipLaunchKernelGGL((dense_infer_kernel<BIG_MT, BIG_KS>), grid, dim3(NT), (size_t)smem, st, a);
  return hipGetLastError();
}

}  // namespace idc
