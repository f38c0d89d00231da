// MobileNetV2 inverted-residual block, inference mode, as ONE launch (gfx950).
//
// In inference (evaluate(), the frozen base of the transfer recipe's phase 1, the frozen prefix of
// the fine-tune phase) every BatchNorm is a constant per-channel affine, so nothing in a block needs
// a batch-wide reduction and the block can run image by image.  A workgroup owns `ipg` whole
// images and a slice of `cs` expanded channels:
//   0. it loads its weight slices (expand rows, project columns), the affine tables and depthwise
//      taps of the slice, and its images' block input x_eff = act(xbn(x)) + res (the previous
//      block's pending project BN and shortcut, applied once) into LDS -- every global load of
//      the launch issued up front, 8 in flight per thread, so the block pays ~one memory latency;
//   1. walks its slice in chunks of MBI_CC = 32 expanded channels:
//        E = ReLU6(ebn(x_eff . We[chunk]^T))   MFMA (v_mfma_f32_16x16x32_bf16), LDS -> LDS
//        D = ReLU6(dbn(depthwise3x3(E)))       VALU from LDS, zero padding by bounds
//        Y += D . Wp[:, chunk]^T               MFMA, accumulators in registers
//      so the 6x-expanded tensor never leaves LDS and exists one 32-channel slice at a time;
//   2. writes y = pbn(Y) (+ x_eff) once, bf16.  With several slices per image group (the wide late
//      blocks: 2x2 / 4x4 maps, 384-960 expanded channels, where one workgroup per group would
//      leave most CUs idle and walk 30 chunks in a row) each slice publishes its fp32 partial tile
//      and the group's last arriver (agent-scope release / ticket / acquire, as conv_big.hip's
//      split-K) sums them in slice order and stores.
// The per-layer path this replaces runs three launches per block with the expanded tensor through
// L2/HBM twice (MobileNetV2 frozen-base step: 55 forward dispatches of ~13 us).
// Reference: the MobileNetV2 backbone of dist_model_tf_mobile.py:119-122, 134-138 (inference passes).
#include "mb_infer.h"
#include "persist.h"

// phase timestamps for tools/micro/mbi_phases.hip (compiled out everywhere else)
#ifndef IDC_MBI_STAMP
#define IDC_MBI_STAMP(i)
#endif

namespace idc {

namespace {

constexpr int NT = MBI_NT, NW = NT / 64;
constexpr int CC = MBI_CC;
constexpr int ES = CC + 8;  // E / D row stride (elements): 80-B rows spread the fragment reads

struct MbiGeo {
  int KX, XS, CS, WPS, NSPLIT, NGROUP, PIN, POUT, MTI, RIN, MTO, ROUT, NTO;
};

__host__ __device__ inline MbiGeo mbi_geo(const MbInferArgs& a) {
  MbiGeo g;
  g.KX = (a.Cin + 31) / 32 * 32;
  g.XS = g.KX + 8;
  g.CS = a.cs;
  g.WPS = g.CS + 8;
  g.NSPLIT = (a.Cexp + g.CS - 1) / g.CS;
  g.NGROUP = (a.N + a.ipg - 1) / a.ipg;
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
  const long long wes = a.we ? (long long)g.CS * g.XS * 2 : 0;
  const long long wps = (long long)g.NTO * 16 * g.WPS * 2;
  const long long tab = (2LL * g.KX + 4LL * g.CS + 2LL * g.NTO * 16 + 9LL * g.CS) * 4;
  return xs + es + ds + wes + wps + tab;
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
  bf16_t* Wes = Ds + g.ROUT * ES;                  // [CS][XS]: expand rows of the slice
  bf16_t* Wps = Wes + (expand ? g.CS * g.XS : 0);  // [NTO*16][WPS]: project columns of the slice
  float* x_sc = reinterpret_cast<float*>(Wps + g.NTO * 16 * g.WPS);
  float* x_sf = x_sc + g.KX;
  float* e_sc = x_sf + g.KX;
  float* e_sf = e_sc + g.CS;
  float* d_sc = e_sf + g.CS;
  float* d_sf = d_sc + g.CS;
  float* p_sc = d_sf + g.CS;
  float* p_sf = p_sc + g.NTO * 16;
  float* s_wd = p_sf + g.NTO * 16;  // [9][CS] depthwise taps of the slice

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int group = blockIdx.x / g.NSPLIT, split = blockIdx.x - group * g.NSPLIT;
  const int cs0 = split * g.CS;                 // first expanded channel of the slice
  const int csn = min(g.CS, a.Cexp - cs0);      // its channels (a multiple of 8)
  const int img0 = group * a.ipg;
  const int nimg = min(a.ipg, a.N - img0);
  const int HWi = a.H * a.W, HWo = a.Ho * a.Wo;
  const int pin = nimg * HWi, pout = nimg * HWo;
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  IDC_MBI_STAMP(0);

  // ---- 0. weight slices, x_eff, affine tables and depthwise taps into LDS, 8 loads in flight per
  // thread.  The tables' loads are issued after the first round of weight / input loads, so both
  // arrive in one memory latency (the input transform needs the x table: it runs after the barrier)
  {
    const int KX8 = g.KX / 8, CS8 = g.CS / 8;
    const int n_we = expand ? g.CS * KX8 : 0, n_wp = g.NTO * 16 * CS8, n_x = g.RIN * KX8;
    const int total = n_we + n_wp + n_x;
    const float xlo = act_lo(a.xbn.act), xhi = act_hi(a.xbn.act);
    constexpr int U = 8;
    for (int base = 0; base < total; base += U * NT) {
      uint4 v[U], r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        v[u] = make_uint4(0, 0, 0, 0);
        r[u] = make_uint4(0, 0, 0, 0);
        if (i < n_we) {
          const int row = i / KX8, k = (i - row * KX8) * 8;
          if (row < csn && k < a.Cin) v[u] = *reinterpret_cast<const uint4*>(a.we + (size_t)(cs0 + row) * a.Cin + k);
        } else if (i < n_we + n_wp) {
          const int j = i - n_we, col = j / CS8, k = (j - col * CS8) * 8;
          if (col < a.Cout && k < csn) v[u] = *reinterpret_cast<const uint4*>(a.wp + (size_t)col * a.Cexp + cs0 + k);
        } else if (i < total) {
          const int j = i - n_we - n_wp, p = j / KX8, c = (j - p * KX8) * 8;
          if (p < pin && c < a.Cin) {
            const size_t pix = (size_t)img0 * HWi + p;
            v[u] = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx + c);
            if (a.res) r[u] = *reinterpret_cast<const uint4*>(a.res + pix * a.ldres + c);
          }
        }
      }
      if (base == 0) {
        const int nx = g.KX, nes = g.CS, np = g.NTO * 16, nwd = 9 * g.CS;
        for (int i = tid; i < nx + nes + np + nwd; i += NT) {
          if (i < nx) {
            float s = 0.f, f = 0.f;
            if (i < a.Cin) bn_coeffs(a.xbn, i, s, f);
            x_sc[i] = s;
            x_sf[i] = f;
          } else if (i < nx + nes) {
            const int lc = i - nx, c = cs0 + lc;
            float s = 0.f, f = 0.f, s2 = 0.f, f2 = 0.f;
            if (lc < csn) {
              if (expand) bn_coeffs(a.ebn, c, s, f);
              bn_coeffs(a.dbn, c, s2, f2);
            }
            e_sc[lc] = s;
            e_sf[lc] = f;
            d_sc[lc] = s2;
            d_sf[lc] = f2;
          } else if (i < nx + nes + np) {
            const int c = i - nx - nes;
            float s = 0.f, f = 0.f;
            if (c < a.Cout) bn_coeffs(a.pbn, c, s, f);
            p_sc[c] = s;
            p_sf[c] = f;
          } else {
            const int j = i - nx - nes - np, t = j / g.CS, lc = j - t * g.CS;
            s_wd[j] = lc < csn ? a.wd[(size_t)t * a.Cexp + cs0 + lc] : 0.f;
          }
        }
        __syncthreads();  // x_sc / x_sf feed the input transform below
        IDC_MBI_STAMP(1);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * NT + tid;
        if (i < n_we) {
          const int row = i / KX8, k = (i - row * KX8) * 8;
          *reinterpret_cast<uint4*>(Wes + row * g.XS + k) = v[u];
        } else if (i < n_we + n_wp) {
          const int j = i - n_we, col = j / CS8, k = (j - col * CS8) * 8;
          *reinterpret_cast<uint4*>(Wps + col * g.WPS + k) = v[u];
        } else if (i < total) {
          const int j = i - n_we - n_wp, p = j / KX8, c = (j - p * KX8) * 8;
          uint4 out = make_uint4(0, 0, 0, 0);
          if (p < pin && c < a.Cin) {
            float xv[8], rv[8];
            unpack8(v[u], xv);
            unpack8(r[u], rv);
#pragma unroll
            for (int q = 0; q < 8; ++q) xv[q] = clampf(fmaf(xv[q], x_sc[c + q], x_sf[c + q]), xlo, xhi) + rv[q];
            out = pack8(xv);
          }
          *reinterpret_cast<uint4*>(Xs + p * g.XS + c) = out;
        }
      }
    }
  }
  __syncthreads();
  IDC_MBI_STAMP(2);

  // ---- 1. chunks of the slice
  const int ntile = g.MTO * g.NTO;
  v4f pacc[MBI_MAX_ACC];
#pragma unroll
  for (int j = 0; j < MBI_MAX_ACC; ++j) pacc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
  const float elo = act_lo(a.ebn.act), ehi = act_hi(a.ebn.act);
  const float dlo = act_lo(a.dbn.act), dhi = act_hi(a.dbn.act);
  const int KS = g.KX / 32;
  const int nch = (csn + CC - 1) / CC;

  for (int ch = 0; ch < nch; ++ch) {
    const int l0 = ch * CC;  // slice-local first channel of the chunk
    // (A) expand: tiles (mt, nt) of the RIN x 32 chunk over the waves
    if (expand) {
      for (int t = wid; t < g.MTI * 2; t += NW) {
        const int mt = t >> 1, nt = t & 1;
        v4f e = {0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < KS; ++ks) {
          const v8bf af = ld_frag(Xs + (mt * 16 + frow) * g.XS + ks * 32 + fk);
          const v8bf bf = ld_frag(Wes + (l0 + nt * 16 + frow) * g.XS + ks * 32 + fk);
          e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, e, 0, 0, 0);
        }
        const int cl = nt * 16 + frow, lc = l0 + cl;
        const float sc = e_sc[lc], sf = e_sf[lc];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + (lane >> 4) * 4 + q;
          const float v = (row < pin && lc < csn) ? clampf(fmaf(e[q], sc, sf), elo, ehi) : 0.f;
          Es[row * ES + cl] = f2bf(v);
        }
      }
      __syncthreads();
    }
    // (B) depthwise 3x3 of the chunk: E -> D
    {
      const bf16_t* src = expand ? Es : Xs + l0;  // (no expand: one slice, x_eff is E)
      const int sl = expand ? ES : g.XS;
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
              unpack8(*reinterpret_cast<const uint4*>(src + (im * HWi + h * a.W + w) * sl + cv), e);
              const float* wt = s_wd + (r * 3 + s) * g.CS + l0 + cv;
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[j] = fmaf(e[j], wt[j], acc[j]);
            }
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int lc = l0 + cv + j;
            acc[j] = lc < csn ? clampf(fmaf(acc[j], d_sc[lc], d_sf[lc]), dlo, dhi) : 0.f;
          }
        }
        *reinterpret_cast<uint4*>(Ds + o * ES + cv) = pack8(acc);
      }
    }
    __syncthreads();
    if (ch == 0) IDC_MBI_STAMP(3);
    // (C) project partial: Y += D . Wp[:, chunk]^T
#pragma unroll
    for (int j = 0; j < MBI_MAX_ACC; ++j) {
      const int t = wid + NW * j;
      if (t < ntile) {
        const int mt = t / g.NTO, nt = t - mt * g.NTO;
        const v8bf af = ld_frag(Ds + (mt * 16 + frow) * ES + fk);
        const v8bf bf = ld_frag(Wps + (nt * 16 + frow) * g.WPS + l0 + fk);
        pacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, pacc[j], 0, 0, 0);
      }
    }
    // (the next chunk's expand writes E only; its depthwise writes D after the next barrier,
    //  which every wave reaches after finishing this step)
  }

  IDC_MBI_STAMP(4);
  // ---- 2. several slices: publish the partial, the group's last arriver sums them in order
  if (g.NSPLIT > 1) {
    constexpr int PT = NW * MBI_MAX_ACC * 64;  // float4 slots of one slice's partial
    float4* gslab = reinterpret_cast<float4*>(a.slab) + (size_t)group * g.NSPLIT * PT;
    float4* mine = gslab + (size_t)split * PT;
    // (persist.h memory model: agent-scope stores, drained before one lane's ticket increment;
    //  the last arriver reads them with agent-scope loads -- no L2 write-back / invalidate fences)
#pragma unroll
    for (int j = 0; j < MBI_MAX_ACC; ++j)
      if (wid + NW * j < ntile)
        persist::st_coh16(mine + (j * NW + wid) * 64 + lane,
                          make_uint4(__float_as_uint(pacc[j][0]), __float_as_uint(pacc[j][1]),
                                     __float_as_uint(pacc[j][2]), __float_as_uint(pacc[j][3])));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* s_flag = reinterpret_cast<int*>(Ds);  // (D is free: every wave is past the chunk loop)
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(&a.tickets[group], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[0] = (prev % (unsigned)g.NSPLIT) == (unsigned)(g.NSPLIT - 1);
    }
    __syncthreads();
    const int last = s_flag[0];
    IDC_MBI_STAMP(5);
    if (!last) return;
#pragma unroll
    for (int j = 0; j < MBI_MAX_ACC; ++j) pacc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
    // two slices' tiles in flight per round trip, summed in slice order
    for (int sl = 0; sl < g.NSPLIT; sl += 2) {
      uint4 q0[MBI_MAX_ACC], q1[MBI_MAX_ACC];
      const float4* o0 = gslab + (size_t)sl * PT;
      const float4* o1 = gslab + (size_t)(sl + 1) * PT;
      const bool two = sl + 1 < g.NSPLIT;
#pragma unroll
      for (int j = 0; j < MBI_MAX_ACC; ++j)
        if (wid + NW * j < ntile) {
          q0[j] = persist::ld_coh16(o0 + (j * NW + wid) * 64 + lane);
          q1[j] = two ? persist::ld_coh16(o1 + (j * NW + wid) * 64 + lane) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
      for (int j = 0; j < MBI_MAX_ACC; ++j)
        if (wid + NW * j < ntile) {
          pacc[j][0] += __uint_as_float(q0[j].x);
          pacc[j][1] += __uint_as_float(q0[j].y);
          pacc[j][2] += __uint_as_float(q0[j].z);
          pacc[j][3] += __uint_as_float(q0[j].w);
          pacc[j][0] += __uint_as_float(q1[j].x);
          pacc[j][1] += __uint_as_float(q1[j].y);
          pacc[j][2] += __uint_as_float(q1[j].z);
          pacc[j][3] += __uint_as_float(q1[j].w);
        }
    }
  }

  IDC_MBI_STAMP(6);
  // ---- 3. y = pbn(Y) (+ x_eff)
#pragma unroll
  for (int j = 0; j < MBI_MAX_ACC; ++j) {
    const int t = wid + NW * j;
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
  IDC_MBI_STAMP(7);
}

long long mb_infer_smem(const MbInferArgs& a) {
  if (a.N < 1 || a.ipg < 1 || a.H < 1 || a.W < 1 || a.Ho < 1 || a.Wo < 1) return -1;
  if (a.Cin % 8 || a.Cexp % 8 || a.Cout % 8 || a.ldx % 8 || a.ldy % 8 || (a.res && a.ldres % 8)) return -1;
  if (a.S != 1 && a.S != 2) return -1;
  if (a.cs < MBI_CC || a.cs % MBI_CC) return -1;
  if (a.we == nullptr && (a.Cexp != a.Cin || a.cs < a.Cexp)) return -1;  // no expand: one slice
  if (a.residual && (a.S != 1 || a.Cin != a.Cout || a.H != a.Ho || a.W != a.Wo)) return -1;
  const MbiGeo g = mbi_geo(a);
  if (g.KX > MBI_MAX_KX) return -1;
  if (g.MTO * g.NTO > NW * MBI_MAX_ACC) return -1;
  if (g.NSPLIT > 1 && (a.slab == nullptr || a.tickets == nullptr)) return -1;
  // every 16-B fragment / vector access must be aligned
  const uintptr_t al = (uintptr_t)a.x | (uintptr_t)a.res | (uintptr_t)a.we | (uintptr_t)a.wp | (uintptr_t)a.y;
  if (al % 16) return -1;
  const long long b = mbi_bytes(a, g);
  return b <= 160 * 1024 ? b : -1;
}

long long mb_infer_slab_floats(const MbInferArgs& a) {
  const MbiGeo g = mbi_geo(a);
  return g.NSPLIT > 1 ? (long long)g.NGROUP * g.NSPLIT * NW * MBI_MAX_ACC * 64 * 4 : 0;
}

hipError_t mb_infer(const MbInferArgs& a, hipStream_t st) {
  const long long smem = mb_infer_smem(a);
  if (smem < 0) return hipErrorInvalidValue;
  const MbiGeo g = mbi_geo(a);
  hipLaunchKernelGGL(mb_infer_kernel, dim3(g.NGROUP * g.NSPLIT), dim3(NT), (size_t)smem, st, a);
  return hipGetLastError();
}

}  // namespace idc
