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
constexpr int MAXMT = 12;      // M tiles of a workgroup (rows <= 192)
constexpr int MAXKS = 16;      // GEMM1 K steps (cin <= 512)
constexpr int MAXG2 = 3;       // GEMM2 tiles per wave (MT * 2 <= 24)

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

// BatchNorm (moving statistics) scale / shift of channel c
__device__ __forceinline__ void inf_coeff(const float* g, const float* b, const float* mm, const float* mv,
                                          float eps, int c, float& sc, float& sf) {
  const float r = rsqrtf(mv[c] + eps);
  const float gg = g ? g[c] : 1.f, bb = b ? b[c] : 0.f;
  sc = gg * r;
  sf = bb - mm[c] * sc;
}

}  // namespace

__global__ __launch_bounds__(NT) void dense_infer_kernel(DenseInferArgs a) {
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

  for (int l = 0; l < a.L; ++l) {
    const DenseLayerDesc& d = a.layers[l];
    const int cin = d.cin;
    const bf16_t* __restrict__ w1 = d.w1;
    const bf16_t* __restrict__ w2 = d.w2;
    // ---- BN tables of the layer (one memory latency; the previous layer's barrier orders reuse)
    for (int c = tid; c < cin + 128; c += NT) {
      if (c < cin) inf_coeff(d.g1, d.b1, d.mm1, d.mv1, d.eps1, c, sc1[c], sf1[c]);
      else inf_coeff(d.g2, d.b2, d.mm2, d.mv2, d.eps2, c - cin, sc2[c - cin], sf2[c - cin]);
    }
    __syncthreads();

    // ---- GEMM1: t = z1 . W1^T.  Wave w owns N tile w (16 of the 128 bottleneck channels) over
    // every M tile, so its B fragments -- all K steps of one 16-row slice of W1 -- are loaded ONCE
    // per layer (one memory latency, issued with the tables) instead of streamed per K step
    {
      const int KS = cin / 32;
      v8bf bw[MAXKS];
#pragma unroll
      for (int ks = 0; ks < MAXKS; ++ks)
        if (ks < KS) bw[ks] = ld_frag(w1 + (size_t)(wid * 16 + frow) * cin + ks * 32 + fk);
      v4f acc[MAXMT];
#pragma unroll
      for (int mt = 0; mt < MAXMT; ++mt) acc[mt] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < MAXKS; ++ks) {
        if (ks < KS) {
          const int k0 = ks * 32 + fk;
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
    {
      const int nt = wid & 1;
      // the 3x3's B fragments of this wave's N tile, in two halves of 18 K steps: the second half
      // is issued once the first 9 steps have consumed their fragments (27 in registers at most)
      const bf16_t* __restrict__ wrow = w2 + (size_t)(nt * 16 + frow) * 1152 + fk;
      v8bf w2f[36];
#pragma unroll
      for (int kk = 0; kk < 18; ++kk) w2f[kk] = ld_frag(wrow + kk * 32);
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
  if (g.MT > MAXMT || 2 * g.MT > NW * MAXG2) return -1;
  for (int l = 0; l < a.L; ++l)
    if ((a.c0 + 32 * l) / 32 > MAXKS) return -1;
  const long long b = di_bytes(a, g);
  return b <= 160 * 1024 ? b : -1;
}

hipError_t dense_infer(const DenseInferArgs& a, hipStream_t st) {
  const long long smem = dense_infer_smem(a);
  if (smem < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dense_infer_kernel, dim3((a.N + a.ipg - 1) / a.ipg), dim3(NT), (size_t)smem, st, a);
  return hipGetLastError();
}

}  // namespace idc
