// MobileNetV2 inverted-residual block, inference mode, as ONE launch (gfx950).
//
// In inference (evaluate(), the frozen-base phase of the transfer recipe, the frozen prefix of the
// fine-tune phase) every BatchNorm is a constant per-channel affine, so nothing in a block needs a
// batch-wide reduction and the whole block can run image by image: a workgroup owns `ipg` whole
// images and
//   1. stages its images' block input once into LDS (x_eff = act(xbn(x)) + res: the previous
//      block's pending project BN and shortcut applied on load), channels zero-padded to KX;
//   2. walks the expanded channels in chunks of MBI_CC = 32:
//        E = ReLU6(ebn(x_eff . We[chunk]^T))   MFMA (v_mfma_f32_16x16x32_bf16), LDS -> LDS
//        D = ReLU6(dbn(depthwise3x3(E)))       VALU from LDS, zero padding by bounds
//        Y += D . Wp[:, chunk]^T               MFMA, accumulators stay in registers
//      so the 6x-expanded tensor never leaves LDS and exists only one 32-channel slice at a time;
//   3. writes y = pbn(Y) (+ x_eff, identity shortcut) once, bf16.
// The per-layer path this replaces runs three launches per block (expand conv, depthwise,
// project conv) with the expanded tensor through L2/HBM twice (profiles: 55 forward dispatches,
// ~13 us each, for the MobileNetV2 frozen-base step).
//
// Weights stream from global (L2-resident) straight into MFMA B-fragment registers (a B fragment
// of W[n][k] is 8 consecutive k of one row: one 16-B load per lane).  Chunk i's project fragments
// are issued at the start of chunk i (they land during its expand and depthwise), chunk i+1's
// expand fragments during chunk i's depthwise, so no chunk waits a full memory latency.
// Reference: the MobileNetV2 backbone of dist_model_tf_mobile.py:119-122, 134-138 (inference passes).
#include "mb_infer.h"

namespace idc {

namespace {

constexpr int NT = 256;
constexpr int CC = MBI_CC;
constexpr int ES = CC + 8;  // E / D row stride (elements): 80-B rows spread the fragment reads
constexpr int KSMAX = MBI_MAX_KX / 32;

struct MbiGeo {
  int KX, XS, CEP, PIN, POUT, MTI, RIN, MTO, ROUT, NTO;
};

__host__ __device__ inline MbiGeo mbi_geo(const MbInferArgs& a) {
  MbiGeo g;
  g.KX = (a.Cin + 31) / 32 * 32;
  g.XS = g.KX + 8;
  g.CEP = (a.Cexp + CC - 1) / CC * CC;
  g.PIN = a.ipg * a.H * a.W;
  g.POUT = a.ipg * a.Ho * a.Wo;
  g.MTI = (g.PIN + 15) / 16;
  g.RIN = g.MTI * 16;
  g.MTO = (g.POUT + 15) / 16;
  g.ROUT = g.MTO * 16;
  g.NTO = (a.Cout + 15) / 16;
  return g;
}

__host__ __device__ inline long long mbi_bytes(const MbInferArgs& a, const MbiGeo& g) {
  const long long xs = (long long)g.RIN * g.XS * 2;
  const long long es = a.we ? (long long)g.RIN * ES * 2 : 0;
  const long long ds = (long long)g.ROUT * ES * 2;
  const long long tab = (2LL * g.KX + 4LL * g.CEP + 2LL * g.NTO * 16 + 9LL * g.CEP) * 4;
  return xs + es + ds + tab;
}

__device__ __forceinline__ v8bf ld_frag(const bf16_t* p) { return *reinterpret_cast<const v8bf*>(p); }

}  // namespace

__global__ __launch_bounds__(NT) void mb_infer_kernel(MbInferArgs a) {
  prefetch_kernargs<sizeof(MbInferArgs)>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MbiGeo g = mbi_geo(a);
  const bool expand = a.we != nullptr;
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Es = Xs + g.RIN * g.XS;
  bf16_t* Ds = Es + (expand ? g.RIN * ES : 0);
  float* x_sc = reinterpret_cast<float*>(Ds + g.ROUT * ES);
  float* x_sf = x_sc + g.KX;
  float* e_sc = x_sf + g.KX;
  float* e_sf = e_sc + g.CEP;
  float* d_sc = e_sf + g.CEP;
  float* d_sf = d_sc + g.CEP;
  float* p_sc = d_sf + g.CEP;
  float* p_sf = p_sc + g.NTO * 16;
  float* s_wd = p_sf + g.NTO * 16;  // [9][CEP] depthwise taps

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img0 = blockIdx.x * a.ipg;
  const int nimg = min(a.ipg, a.N - img0);
  const int HWi = a.H * a.W, HWo = a.Ho * a.Wo;
  const int pin = nimg * HWi, pout = nimg * HWo;
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  const v8bf zf = {};

  // ---- chunk-0 expand fragments first: their latency overlaps the tables and the input stage
  const int KS = g.KX / 32;
  v8bf bfe[2][KSMAX];
  auto load_bfe = [&](int c0) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < KSMAX; ++ks) {
        const int col = c0 + n * 16 + frow, k = ks * 32 + fk;
        bfe[n][ks] = (ks < KS && col < a.Cexp && k < a.Cin) ? ld_frag(a.we + (size_t)col * a.Cin + k) : zf;
      }
  };
  if (expand) load_bfe(0);

  // ---- per-channel affine tables and the depthwise taps
  for (int c = tid; c < g.KX; c += NT) {
    float s = 0.f, f = 0.f;
    if (c < a.Cin) bn_coeffs(a.xbn, c, s, f);
    x_sc[c] = s;
    x_sf[c] = f;
  }
  for (int c = tid; c < g.CEP; c += NT) {
    float s = 0.f, f = 0.f, s2 = 0.f, f2 = 0.f;
    if (c < a.Cexp) {
      if (expand) bn_coeffs(a.ebn, c, s, f);
      bn_coeffs(a.dbn, c, s2, f2);
    }
    e_sc[c] = s;
    e_sf[c] = f;
    d_sc[c] = s2;
    d_sf[c] = f2;
  }
  for (int c = tid; c < g.NTO * 16; c += NT) {
    float s = 0.f, f = 0.f;
    if (c < a.Cout) bn_coeffs(a.pbn, c, s, f);
    p_sc[c] = s;
    p_sf[c] = f;
  }
  for (int i = tid; i < 9 * g.CEP; i += NT) {
    const int t = i / g.CEP, c = i - t * g.CEP;
    s_wd[i] = c < a.Cexp ? a.wd[(size_t)t * a.Cexp + c] : 0.f;
  }
  __syncthreads();

  // ---- stage x_eff = act(xbn(x)) + res: 8 chunk loads in flight per thread
  {
    const float lo = act_lo(a.xbn.act), hi = act_hi(a.xbn.act);
    const int KX8 = g.KX / 8, total = g.RIN * KX8;
    constexpr int U = 8;
    for (int base = 0; base < total; base += U * NT) {
      uint4 xv[U], rv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        const int p = i / KX8, c = (i - p * KX8) * 8;
        const bool ok = i < total && p < pin && c < a.Cin;
        const size_t pix = (size_t)img0 * HWi + (ok ? p : 0);
        xv[u] = ok ? *reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c) : make_uint4(0, 0, 0, 0);
        rv[u] = (ok && a.res) ? *reinterpret_cast<const uint4*>(a.res + pix * a.ldres + c) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        if (i >= total) break;
        const int p = i / KX8, c = (i - p * KX8) * 8;
        uint4 out = make_uint4(0, 0, 0, 0);
        if (p < pin && c < a.Cin) {
          float v[8], r[8];
          unpack8(xv[u], v);
          unpack8(rv[u], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = clampf(fmaf(v[j], x_sc[c + j], x_sf[c + j]), lo, hi) + r[j];
          out = pack8(v);
        }
        *reinterpret_cast<uint4*>(Xs + p * g.XS + c) = out;
      }
    }
  }
  __syncthreads();

  // ---- project accumulators: tile t = wid + 4 j of the MTO x NTO output tiles
  const int ntile = g.MTO * g.NTO;
  v4f pacc[MBI_MAX_ACC];
#pragma unroll
  for (int j = 0; j < MBI_MAX_ACC; ++j) pacc[j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const float elo = act_lo(a.ebn.act), ehi = act_hi(a.ebn.act);
  const float dlo = act_lo(a.dbn.act), dhi = act_hi(a.dbn.act);
  const bf16_t* Esrc = expand ? Es : Xs;
  const int esl = expand ? ES : g.XS;
  const int nchunk = g.CEP / CC;

  for (int ch = 0; ch < nchunk; ++ch) {
    const int c0 = ch * CC;
    // (A) this chunk's project fragments (consumed in C), then the expand GEMM
    v8bf bfp[MBI_MAX_ACC];
#pragma unroll
    for (int j = 0; j < MBI_MAX_ACC; ++j) {
      const int t = wid + 4 * j;
      const int nt = t % g.NTO;
      const int col = nt * 16 + frow, k = c0 + fk;
      bfp[j] = (t < ntile && col < a.Cout && k < a.Cexp) ? ld_frag(a.wp + (size_t)col * a.Cexp + k) : zf;
    }
    if (expand) {
      for (int mt = wid; mt < g.MTI; mt += 4) {
        v4f e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KSMAX; ++ks) {
          if (ks < KS) {
            const v8bf af = ld_frag(Xs + (mt * 16 + frow) * g.XS + ks * 32 + fk);
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfe[0][ks], e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfe[1][ks], e1, 0, 0, 0);
          }
        }
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const v4f& e = n ? e1 : e0;
          const int cl = n * 16 + frow, c = c0 + cl;
          const float sc = e_sc[c], sf = e_sf[c];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = mt * 16 + (lane >> 4) * 4 + q;
            const float v = (row < pin && c < a.Cexp) ? clampf(fmaf(e[q], sc, sf), elo, ehi) : 0.f;
            Es[row * ES + cl] = f2bf(v);
          }
        }
      }
    }
    __syncthreads();
    // (B) next chunk's expand fragments in flight; depthwise 3x3 of this chunk: E -> D
    if (expand && ch + 1 < nchunk) load_bfe(c0 + CC);
    const int coff = expand ? 0 : c0;
    for (int i = tid; i < g.ROUT * (CC / 8); i += NT) {
      const int o = i / (CC / 8), cv = (i % (CC / 8)) * 8;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (o < pout) {
        const int im = o / HWo, r0 = o - im * HWo, ho = r0 / a.Wo, wo = r0 - ho * a.Wo;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int h = ho * a.S - a.PT + r;
          if ((unsigned)h >= (unsigned)a.H) continue;
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const int w = wo * a.S - a.PL + s;
            if ((unsigned)w >= (unsigned)a.W) continue;
            float e[8];
            unpack8(*reinterpret_cast<const uint4*>(Esrc + (im * HWi + h * a.W + w) * esl + coff + cv), e);
            const float* wt = s_wd + (r * 3 + s) * g.CEP + c0 + cv;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(e[j], wt[j], acc[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = c0 + cv + j;
          acc[j] = c < a.Cexp ? clampf(fmaf(acc[j], d_sc[c], d_sf[c]), dlo, dhi) : 0.f;
        }
      }
      *reinterpret_cast<uint4*>(Ds + o * ES + cv) = pack8(acc);
    }
    __syncthreads();
    // (C) project partial: Y += D . Wp[:, chunk]^T
#pragma unroll
    for (int j = 0; j < MBI_MAX_ACC; ++j) {
      const int t = wid + 4 * j;
      if (t < ntile) {
        const int mt = t / g.NTO;
        const v8bf af = ld_frag(Ds + (mt * 16 + frow) * ES + fk);
        pacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfp[j], pacc[j], 0, 0, 0);
      }
    }
    // (the next chunk's expand writes E only, and its depthwise writes D after the next barrier,
    //  which every wave reaches after finishing this step)
  }

  // ---- epilogue: y = pbn(Y) (+ x_eff)
#pragma unroll
  for (int j = 0; j < MBI_MAX_ACC; ++j) {
    const int t = wid + 4 * j;
    if (t < ntile) {
      const int mt = t / g.NTO, nt = t - mt * g.NTO;
      const int col = nt * 16 + frow;
      if (col < a.Cout) {
        const float sc = p_sc[col], sf = p_sf[col];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          if (row < pout) {
            float v = fmaf(pacc[j][q], sc, sf);
            if (a.residual) v += bf2f(Xs[row * g.XS + col]);
            a.y[((size_t)img0 * HWo + row) * a.ldy + col] = f2bf(v);
          }
        }
      }
    }
  }
}

long long mb_infer_smem(const MbInferArgs& a) {
  if (a.N < 1 || a.ipg < 1 || a.H < 1 || a.W < 1 || a.Ho < 1 || a.Wo < 1) return -1;
  if (a.Cin % 8 || a.Cexp % 8 || a.Cout % 8 || a.ldx % 8 || a.ldy % 8 || (a.res && a.ldres % 8)) return -1;
  if (a.S != 1 && a.S != 2) return -1;
  if (a.we == nullptr && a.Cexp != a.Cin) return -1;
  if (a.residual && (a.S != 1 || a.Cin != a.Cout || a.H != a.Ho || a.W != a.Wo)) return -1;
  const MbiGeo g = mbi_geo(a);
  if (g.KX > MBI_MAX_KX) return -1;
  if (g.MTO * g.NTO > 4 * MBI_MAX_ACC) return -1;
  // every 16-B fragment / vector access must be aligned
  const uintptr_t al = (uintptr_t)a.x | (uintptr_t)a.res | (uintptr_t)a.we | (uintptr_t)a.wp | (uintptr_t)a.y;
  if (al % 16) return -1;
  const long long b = mbi_bytes(a, g);
  return b <= 160 * 1024 ? b : -1;
}

hipError_t mb_infer(const MbInferArgs& a, hipStream_t st) {
  const long long smem = mb_infer_smem(a);
  if (smem < 0) return hipErrorInvalidValue;
  const int grid = (a.N + a.ipg - 1) / a.ipg;
  hipLaunchKernelGGL(mb_infer_kernel, dim3(grid), dim3(NT), (size_t)smem, st, a);
  return hipGetLastError();
}

}  // namespace idc
