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
// no grid barriers, no global round trips between layers; weights stream from L2 into MFMA B
// fragments.  The per-layer path it replaces runs 2 launches per layer (12 + 24 for stages 1-2 of
// DenseNet-121 at 50x50, ~390 us of the frozen-base step, profiles/densenet121_frozen_*).
// Reference: the dense blocks of dist_model_tf_dense.py:131-133 (inference passes).
#include "dense_stage.h"

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
__host__ __device__ inline long long di_bytes(const DenseInferArgs& a, const DiGeo& g) {
  return (long long)g.RP * g.CS * 2 + (long long)a.ipg * g.GP * ZS * 2 + (2LL * g.CT + 256 + g.RP) * 4;
}

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

}  // namespace

template <int MAXMT, int MAXKS>
__global__ __launch_bounds__(NT) void dense_infer_kernel(DenseInferArgs a) {
  constexpr int MAXG2 = (2 * MAXMT + NW - 1) / NW;  // GEMM2 tiles per wave
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
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img0 = blockIdx.x * a.ipg;
  const int nimg = min(a.ipg, a.N - img0);
  const int pv = nimg * g.HW;  // valid rows
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  const float lo = act_lo(a.act), hi = act_hi(a.act);

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
  layer_tables(a.layers[0], sc1, sf1, sc2, sf2, tid);
  __syncthreads();

  for (int l = 0; l < a.L; ++l) {
    const DenseLayerDesc& d = a.layers[l];
    const int cin = d.cin;
    const bf16_t* __restrict__ w1 = d.w1;
    const bf16_t* __restrict__ w2 = d.w2;

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
      const float s2 = sc2[col], f2 = sf2[col];
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) {
        if (mt >= g.MT) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row >= pv) continue;
          Z2[(size_t)(gtl[row] + g.GW + 1) * ZS + col] = f2bf(clampf(fmaf(acc[mt][q], s2, f2), lo, hi));
        }
      }
    }
    __syncthreads();

    // ---- GEMM2: n = conv3x3(z2) . W2^T (tiles wid + 8 j, all of one N tile), epilogue into cat
    if (c1) {
      const int nt = wid & 1;
      const bf16_t* __restrict__ wrow = w2 + (size_t)(nt * 16 + frow) * 128 + fk;
      v8bf wc[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wc[kk] = ld_frag(wrow + kk * 32);
      if (l + 1 < a.L) layer_tables(a.layers[l + 1], sc1, sf1, sc2, sf2, tid);
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
      if (l + 1 < a.L) layer_tables(a.layers[l + 1], sc1, sf1, sc2, sf2, tid);
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
#pragma unroll
      for (int j = 0; j < MAXG2; ++j) {
        const int mt = (wid + NW * j) >> 1;
        if (mt >= g.MT) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row < pv) Cat[row * g.CS + cin + nt * 16 + frow] = f2bf(acc[j][q]);
        }
      }
    }
    __syncthreads();
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

long long dense_infer_smem(const DenseInferArgs& a) {
  if (a.N < 1 || a.ipg < 1 || a.L < 1 || a.H < 1 || a.W < 1) return -1;
  if (a.c0 % 32 || a.ld % 8 || a.c0 + 32 * a.L > a.ld) return -1;
  if ((uintptr_t)a.buf % 16) return -1;
  const DiGeo g = di_geo(a);
  if (g.MT > BIG_MT) return -1;
  if (g.CT > MAXCT) return -1;
  const long long b = di_bytes(a, g);
  return b <= 160 * 1024 ? b : -1;
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
