// Image-resident weight gradient of the stem convolution, gfx950 (the first conv of DenseNet,
// MobileNetV2 and VGG16: the staged 8-channel image, 3 real channels, KxK taps, <= 64 outputs).
//
//   dW[(r*KW + c)*cr + ch][co] = sum_p X[img(p), ho(p)*S - PT + r, wo(p)*S - PL + c, ch] * G[p][co]
//
// The general wgrad kernel gathers im2col rows of 8-channel pixels through VGPRs for every tap and
// pixel step; it ran 55-61 us on the main lane at the very end of the backward (DenseNet-121 and
// VGG16 bench profiles, round 5) for 1.5 GFLOP of real work.  Here a workgroup owns a band of
// output rows of ONE image:
//   * the band's input rows (zero padding materialised, 16 B per pixel) are copied into LDS once;
//   * per 32-pixel chunk the workgroup builds the transposed im2col tile X^T [real k rows][32 px]
//     and G^T [co][32 px] in LDS (G through the stem BatchNorm's pending backward affine when
//     `gpro` is set -- DenseNet), so both MFMA operands are contiguous 16-B fragment reads;
//   * v_mfma_f32_16x16x32_bf16 with the 32 pixels as the reduction: wave w owns output-column
//     fragment w % NCF and every (4/NCF)-th k-row fragment; its accumulators live for the band;
//   * the band's partial dW goes to its slice of the `part` slab with plain stores (the plan sums
//     the slices in order right after: wgrad_reduce) -- float atomics from ~1k workgroups onto the
//     same 9.4k addresses measured 81 us -- or, without a slab, is added with float atomics.
// Selected automatically by conv_wgrad (conv_wgrad.hip) where wgrad_stem_ok() holds.
#include "conv_wgrad.h"

#include <cstdlib>

namespace idc {

namespace {

constexpr int NT = 256;
constexpr int PC = 32;            // pixels per chunk (the MFMA reduction depth)
constexpr int TP = PC + 8;        // bf16 per transposed row (80 B: 16-B aligned, bank skew)
constexpr int MAXRF = 10;         // k-row fragments (7 x 7 taps x 3 channels = 147 -> 160)
constexpr int SMEM_MAX = 64 * 1024;

struct WsGeo {
  int nb, rows, lrows, wp, kr, krf;
};

inline WsGeo ws_geo(const WgradArgs& a) {
  WsGeo g{};
  const int cr = a.cin_real ? a.cin_real : a.Cin;
  g.kr = a.KH * a.KW * cr;
  g.krf = (g.kr + 15) / 16;
  g.wp = (a.Wo - 1) * a.SW + a.KW;
  const int fixed = (g.krf * 16 + a.Cout) * TP * 2 + 3 * a.Cout * 4 + PC * 4;
  int nb = (512 + a.N - 1) / a.N;  // >= 2 workgroups per CU where the images allow it
  if (nb > a.Ho) nb = a.Ho;
  if (nb < 1) nb = 1;
  for (;;) {
    g.rows = (a.Ho + nb - 1) / nb;
    g.lrows = (g.rows - 1) * a.SH + a.KH;
    if (g.lrows * g.wp * 16 + fixed <= SMEM_MAX || nb >= a.Ho) break;
    ++nb;
  }
  g.nb = (a.Ho + g.rows - 1) / g.rows;
  return g;
}

inline int ws_smem(const WgradArgs& a, const WsGeo& g) {
  return g.lrows * g.wp * 16 + (g.krf * 16 + a.Cout) * TP * 2 + 3 * a.Cout * 4 + PC * 4;
}

}  // namespace

// (outside the anonymous namespace so profiles name it)
template <int NCF>
__global__ __launch_bounds__(NT) void wgrad_stem_kernel(WgradArgs a, WsGeo g, GroupArg ga) {
  prefetch_kernargs<sizeof(WgradArgs) + sizeof(WsGeo) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RSTEP = 4 / NCF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cf = wid % NCF, rf0 = wid / NCF;
  const int img = blockIdx.x / g.nb, band = blockIdx.x - img * g.nb;
  const int ho0 = band * g.rows, ho1 = min(a.Ho, ho0 + g.rows);
  const int npix = (ho1 - ho0) * a.Wo;
  const int cr = a.cin_real ? a.cin_real : a.Cin;
  const int C = a.Cout;
  uint4* simg = reinterpret_cast<uint4*>(smem);
  bf16_t* xt = reinterpret_cast<bf16_t*>(smem + g.lrows * g.wp * 16);  // [krf*16][TP]
  bf16_t* gt = xt + g.krf * 16 * TP;                                    // [C][TP]
  float* tA = reinterpret_cast<float*>(gt + C * TP);                    // gpro table [3][C]
  float* tB = tA + C;
  float* tC = tB + C;
  int* poff = reinterpret_cast<int*>(tC + C);                           // [PC] chunk pixel offsets
  const bf16_t* __restrict__ X = a.x;
  const bf16_t* __restrict__ G = reinterpret_cast<const bf16_t*>(a.g);
  const bool aff = a.gpro.mode != 0;

  if (aff) bwd_aff_table<NT>(a.gpro, 0, C, C, tA, tB, tC);
  // ---- the band's input rows into LDS
  {
    const int h_base = ho0 * a.SH - a.PT;
    const int items = g.lrows * g.wp;
    const size_t ib = (size_t)img * a.H * a.W;
    for (int i0 = tid; i0 < items; i0 += 4 * NT) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT;
        const int j = i / g.wp, cw = i - j * g.wp;
        const int h = h_base + j, w = cw - a.PL;
        const bool ok = i < items && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        v[u] = ok ? *reinterpret_cast<const uint4*>(X + (ib + (size_t)h * a.W + w) * a.ldx) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT;
        if (i < items) simg[i] = v[u];
      }
    }
  }

  v4f acc[MAXRF];
#pragma unroll
  for (int i = 0; i < MAXRF; ++i) acc[i] = (v4f){0.f, 0.f, 0.f, 0.f};
  const size_t pbase = ((size_t)img * a.Ho + ho0) * a.Wo;  // first output pixel of the band
  const int q = lane >> 4;
  const int gitems = PC * (C / 8);   // G chunk: (pixel, 8 channels) items
  const int xitems = g.kr * (PC / 8); // X^T chunk: (k row, 8 pixels) items

  for (int p0 = 0; p0 < npix; p0 += PC) {
    // ---- G chunk: loads first (bf16 g, and the BatchNorm input when the affine applies)
    uint4 gv[2], xv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = tid + u * NT;
      const int pj = it / (C / 8), c8 = it - pj * (C / 8);
      const bool ok = it < gitems && p0 + pj < npix;
      const size_t m = pbase + p0 + pj;
      gv[u] = ok ? *reinterpret_cast<const uint4*>(G + m * a.ldg + c8 * 8) : make_uint4(0u, 0u, 0u, 0u);
      xv[u] = (ok && aff) ? *reinterpret_cast<const uint4*>(a.gpro.x + m * a.gpro.ldx + c8 * 8)
                          : make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();  // the previous chunk's fragment reads are done (and, first time: tables, image)
    if (tid < PC) {  // LDS pixel offset (bf16 elements) of each chunk pixel's window origin, -1 past the band
      const int pj = p0 + tid;
      const int ho = pj / a.Wo, wo = pj - ho * a.Wo;
      poff[tid] = pj < npix ? ((ho * a.SH) * g.wp + wo * a.SW) * 8 : -1;
    }
    __syncthreads();
    // ---- X^T chunk: row k = (tap, ch), 8 consecutive pixels per item
    {
      const bf16_t* simg16 = reinterpret_cast<const bf16_t*>(simg);
      for (int it = tid; it < xitems; it += NT) {
        const int kr = it / (PC / 8), j8 = it - kr * (PC / 8);
        const int t = kr / cr, ch = kr - t * cr;
        const int r = t / a.KW, c = t - r * a.KW;
        const int koff = (r * g.wp + c) * 8 + ch;
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const int o0 = poff[j8 * 8 + e], o1 = poff[j8 * 8 + e + 1];
          const uint32_t v0 = o0 >= 0 ? simg16[o0 + koff] : 0u;
          const uint32_t v1 = o1 >= 0 ? simg16[o1 + koff] : 0u;
          w4[e / 2] = v0 | (v1 << 16);
        }
        *reinterpret_cast<uint4*>(xt + kr * TP + j8 * 8) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
    // (k rows past kr up to the fragment boundary are zero: written once below, never dirtied)
    // ---- G^T chunk: transposed scatter of the (pixel, 8 channels) items
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = tid + u * NT;
      if (it < gitems) {
        const int pj = it / (C / 8), c8 = it - pj * (C / 8);
        float f[8], xf[8];
        unpack8(gv[u], f);
        if (aff) {
          unpack8(xv[u], xf);
          bwd_aff8(f, xf, tA + c8 * 8, tB + c8 * 8, tC + c8 * 8);
          if (p0 + pj >= npix) {
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) gt[(c8 * 8 + e) * TP + pj] = f2bf(f[e]);
      }
    }
    if (p0 == 0) {
      for (int i = g.kr * (PC / 8) + tid; i < g.krf * 16 * (PC / 8); i += NT) {
        const int kr = i / (PC / 8), j8 = i - kr * (PC / 8);
        *reinterpret_cast<uint4*>(xt + kr * TP + j8 * 8) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    __syncthreads();
    // ---- MFMAs: C[k rows][co] += X^T[k][px] . G[px][co]
    const v8bf bfr = *reinterpret_cast<const v8bf*>(gt + (cf * 16 + (lane & 15)) * TP + 8 * q);
#pragma unroll
    for (int i = 0; i < MAXRF; ++i) {
      const int rf = rf0 + i * RSTEP;
      if (rf < g.krf) {
        const v8bf af = *reinterpret_cast<const v8bf*>(xt + (rf * 16 + (lane & 15)) * TP + 8 * q);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i], 0, 0, 0);
      }
    }
  }
  // ---- the band's partial dW: rows 16 rf + 4 q + j, column 16 cf + lane % 16
  const int co = cf * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < MAXRF; ++i) {
    const int rf = rf0 + i * RSTEP;
    if (rf < g.krf) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = rf * 16 + 4 * q + j;
        if (k < g.kr) {
          if (a.part) a.part[(size_t)blockIdx.x * g.kr * C + (size_t)k * C + co] = acc[i][j] * a.scale;
          else atomicAdd(&a.dw[(size_t)k * C + co], acc[i][j] * a.scale);
        }
      }
    }
  }
}

namespace {

}  // namespace

bool wgrad_stem_ok(const WgradArgs& a, bool g_f32) {
  static const bool on = [] {
    const char* e = std::getenv("IDC_WGRAD_STEM");
    return e && e[0] == '1';  // opt-in: measured no faster than the general kernel (round 5)
  }();
  const int cr = a.cin_real ? a.cin_real : a.Cin;
  if (!on || g_f32 || a.Cin != 8 || cr > 8 || a.ldx % 8 || a.ldg % 8) return false;
  if (a.Cout % 16 || a.Cout > 64 || a.Cout < 16 || (64 % a.Cout) != 0) return false;
  if (a.KH != a.KW || a.KH > 7 || a.SH != a.SW || (a.SH != 1 && a.SH != 2)) return false;
  if (a.pro.mode != 0 || a.pro.act != ACT_NONE || a.PT < 0 || a.PL < 0 || a.PT >= a.KH || a.PL >= a.KW) return false;
  if (a.gpro.mode != 0 && (a.gpro.x == nullptr || a.gpro.ldx % 8 || a.gpro.mode != 1)) return false;
  const WsGeo g = ws_geo(a);
  const int rsteps = 4 / (a.Cout / 16);
  if (a.part && (long long)a.N * g.nb * g.kr * a.Cout > a.part_floats) return false;
  return g.krf <= MAXRF * rsteps && (g.krf + rsteps - 1) / rsteps <= MAXRF && ws_smem(a, g) <= SMEM_MAX;
}

// workgroups of the launch = partial slices of its `part` slab (one full partial dW each)
int wgrad_stem_slices(const WgradArgs& a) { return a.N * ws_geo(a).nb; }

hipError_t wgrad_stem(const WgradArgs& a, hipStream_t st) {
  if (!wgrad_stem_ok(a, false)) return hipErrorInvalidValue;
  const WsGeo g = ws_geo(a);
  const dim3 grid = ggrid(dim3(a.N * g.nb));
  const size_t smem = ws_smem(a, g);
  switch (a.Cout / 16) {
    case 1: hipLaunchKernelGGL(wgrad_stem_kernel<1>, grid, dim3(NT), smem, st, a, g, garg()); break;
    case 2: hipLaunchKernelGGL(wgrad_stem_kernel<2>, grid, dim3(NT), smem, st, a, g, garg()); break;
    default: hipLaunchKernelGGL(wgrad_stem_kernel<4>, grid, dim3(NT), smem, st, a, g, garg()); break;
  }
  return hipGetLastError();
}

}  // namespace idc
