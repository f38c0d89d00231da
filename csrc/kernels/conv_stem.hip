// Image-resident stem convolution, gfx950: the first conv of every model family, whose input is
// the staged image (8 channels: RGB zero-padded by the input op) -- DenseNet's 7x7 / 2,
// MobileNetV2's 3x3 / 2 and VGG16's 3x3 / 1 on 50 x 50 patches.
//
// The implicit GEMM (conv_igemm_impl.h) gathers one 16-B pixel per tap and K step through VGPRs and
// re-reads every input pixel KH*KW / (SH*SW) times from L2; with 8 input channels its tiles are
// almost all gather: DenseNet's stem took 52 us for 0.8 GFLOP of real work (bench profile, round
// 5), VGG16's conv1_1 54 us.  Here a workgroup owns a band of output rows of ONE image:
//   * the band's input rows (with the zero padding materialised) are copied into LDS once,
//     16 B per pixel -- every tap of every output pixel is then one aligned ds_read_b128;
//   * K = KH*KW taps x 8 channels, 4 taps per v_mfma_f32_16x16x32_bf16 step; the B fragments of
//     all K steps stay in registers for the whole band (wave w owns output columns
//     16*(w % NCF) .. +16, NCF = Cout / 16 column fragments, and every 4/NCF-th row fragment);
//   * one accumulator per 16-pixel row fragment (the dependent MFMA chain runs at full rate,
//     MI355X_MICROARCH.md "Per-instruction cycle constants"), then bias + activation into the
//     band's bf16 output tile in LDS, written out as whole pixel rows with 16-B stores, and the
//     shifted per-channel statistics kept in registers for the band (one column per lane).
// Selected by the autotuner as conv tile TILE_STEM (conv_igemm.hip) where conv_stem_ok() holds.
#include "conv_igemm.h"

namespace idc {

namespace {

constexpr int NT = 256;
constexpr int MAXKS = 13;      // K steps (7 x 7 taps: 49 -> 13 steps of 4 taps)
constexpr int SMEM_MAX = 64 * 1024;

struct StemGeo {
  int nb, rows;   // bands per image, output rows per band
  int lrows, wp;  // LDS rows / row width (pixels) of a band
};

// bytes of LDS for one band: the input rows (16 B per pixel) + the bf16 output tile (row pitch
// Cout + 8 elements)
inline int stem_lds(const ConvArgs& a, const StemGeo& g) {
  return g.lrows * g.wp * 16 + g.rows * a.Wo * (a.Cout + 8) * 2;
}

inline StemGeo stem_geo(const ConvArgs& a) {
  StemGeo g{};
  g.wp = (a.Wo - 1) * a.SW + a.KW;
  // bands so that a launch has >= 1024 workgroups (four per CU: one workgroup per CU left every
  // SIMD a single wave, its fragment reads and MFMA chain exposed -- 55 us, as slow as the
  // implicit GEMM) where the images allow it, each band's input rows fitting the LDS budget
  int nb = (1024 + a.N - 1) / a.N;
  if (nb > a.Ho) nb = a.Ho;
  if (nb < 1) nb = 1;
  for (;;) {
    g.rows = (a.Ho + nb - 1) / nb;
    g.lrows = (g.rows - 1) * a.SH + a.KH;
    if (stem_lds(a, g) <= SMEM_MAX || nb >= a.Ho) break;
    ++nb;
  }
  g.nb = (a.Ho + g.rows - 1) / g.rows;
  return g;
}

}  // namespace

// (outside the anonymous namespace so profiles name it)
template <int NCF>
__global__ __launch_bounds__(NT) void conv_stem_kernel(ConvArgs a, StemGeo g, GroupArg ga) {
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(StemGeo) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RSTEP = 4 / NCF;  // row fragments are dealt round-robin over the waves of a column
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cf = wid % NCF, r0 = wid / NCF;
  const int img = blockIdx.x / g.nb, band = blockIdx.x - img * g.nb;
  const int ho0 = band * g.rows, ho1 = min(a.Ho, ho0 + g.rows);
  const int npix = (ho1 - ho0) * a.Wo;
  const int taps = a.KH * a.KW, nks = (taps + 3) / 4;
  uint4* simg = reinterpret_cast<uint4*>(smem);
  constexpr int OP = NCF * 16 + 8;  // output tile row pitch (bf16): 16-B aligned rows
  bf16_t* sout = reinterpret_cast<bf16_t*>(smem + g.lrows * g.wp * 16);
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(a.x);

  // ---- B fragments of every K step (column n = 16 cf + lane % 16, taps 4 s + lane / 16)
  const int n = cf * 16 + (lane & 15), q = lane >> 4;
  v8bf bq[MAXKS];
#pragma unroll
  for (int s = 0; s < MAXKS; ++s) {
    const int t = 4 * s + q;
    bq[s] = (s < nks && t < taps) ? *reinterpret_cast<const v8bf*>(a.w + ((size_t)n * taps + t) * 8) : v8bf{};
  }
  const float bias = a.bias ? a.bias[n] : 0.f;
  const float kk = a.stats_shift ? a.stats_shift[n] : 0.f;
  const float lo = act_lo(a.epi_act), hi = act_hi(a.epi_act);

  // ---- the band's input rows into LDS (zero padding materialised)
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
  // LDS offset (pixels) of each K step's tap for this lane's quarter (t = 4 s + q), relative to
  // the output pixel's window origin
  int toff[MAXKS];
#pragma unroll
  for (int s = 0; s < MAXKS; ++s) {
    const int t = min(4 * s + q, taps - 1);
    const int r = t / a.KW, c = t - r * a.KW;
    toff[s] = r * g.wp + c;
  }
  __syncthreads();

  float ps = 0.f, pq = 0.f;
  const int nfr = (npix + 15) / 16;
  for (int fr = r0; fr < nfr; fr += RSTEP) {
    // this lane's A row: pixel fr*16 + lane % 16 of the band
    const int p = min(fr * 16 + (lane & 15), npix - 1);
    const int ho = p / a.Wo, wo = p - ho * a.Wo;
    const int base = ho * a.SH * g.wp + wo * a.SW;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    // every fragment read of the K loop in flight before the first MFMA
    v8bf af[MAXKS];
#pragma unroll
    for (int s = 0; s < MAXKS; ++s)
      af[s] = s < nks ? __builtin_bit_cast(v8bf, simg[base + toff[s]]) : v8bf{};
#pragma unroll
    for (int s = 0; s < MAXKS; ++s) {
      if (s < nks)  // (wave-uniform; no early exit: the fragment arrays stay in registers)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s], bq[s], acc, 0, 0, 0);
    }
    // rows 4*(lane/16) + j of the fragment, column lane % 16, into the band's output tile
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rl = 4 * q + j;
      const float v = clampf(acc[j] + bias, lo, hi);
      const bf16_t h = f2bf(v);
      if (fr * 16 + rl < npix) {
        sout[(fr * 16 + rl) * OP + n] = h;
        const float d = bf2f(h) - kk;
        ps += d;
        pq += d * d;
      }
    }
  }
  __syncthreads();
  // whole output rows (Cout * 2 B, one pixel each) with 16-B stores: partial-line writes of one
  // wave's 16 columns ran the store path at ~1 TB/s
  {
    constexpr int C8 = NCF * 2;
    const size_t obase = ((size_t)img * a.Ho + ho0) * a.Wo;
    for (int i = tid; i < npix * C8; i += NT) {
      const int pp = i / C8, c8 = i - pp * C8;
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.y) + (obase + pp) * a.ldy + c8 * 8) =
          *reinterpret_cast<const uint4*>(sout + pp * OP + c8 * 8);
    }
  }
  if (a.stats_out) {
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    pq += __shfl_xor(pq, 16, 64);
    pq += __shfl_xor(pq, 32, 64);
    if (lane < 16) {
      float* so = a.stats_out + (size_t)(blockIdx.x % stat_slots(a.stats_slots)) * 2 * a.stats_ld + a.stats_off;
      atomicAdd(so + n, ps);
      atomicAdd(so + a.stats_ld + n, pq);
    }
  }
}

namespace {

}  // namespace

bool conv_stem_ok(const ConvArgs& a, bool a_f32) {
  if (a_f32 || a.Cin != 8 || a.ldx % 8 || a.ldy % 8) return false;
  if (a.Cout % 16 || a.Cout > 64 || a.Cout < 16 || (64 % a.Cout) != 0) return false;
  if (a.KH != a.KW || a.KH > 7 || a.KH < 1 || a.SH != a.SW || (a.SH != 1 && a.SH != 2)) return false;
  if (a.pro.mode != 0 || a.pro.act != ACT_NONE || a.bpro.mode != 0 || a.epi_mode != 0 || a.out_mode != OUT_BF16)
    return false;
  if (a.ksplit > 1 || a.PT < 0 || a.PL < 0 || a.PT >= a.KH || a.PL >= a.KW) return false;
  const StemGeo g = stem_geo(a);
  return stem_lds(a, g) <= SMEM_MAX;
}

hipError_t conv_stem(const ConvArgs& a, bool a_f32, hipStream_t st) {
  if (!conv_stem_ok(a, a_f32)) return hipErrorInvalidValue;
  const StemGeo g = stem_geo(a);
  const size_t smem = stem_lds(a, g);
  const dim3 grid = ggrid(dim3(a.N * g.nb));
  switch (a.Cout / 16) {
    case 1: hipLaunchKernelGGL(conv_stem_kernel<1>, grid, dim3(NT), smem, st, a, g, garg()); break;
    case 2: hipLaunchKernelGGL(conv_stem_kernel<2>, grid, dim3(NT), smem, st, a, g, garg()); break;
    default: hipLaunchKernelGGL(conv_stem_kernel<4>, grid, dim3(NT), smem, st, a, g, garg()); break;
  }
  return hipGetLastError();
}

}  // namespace idc
