// Row-block 1x1 data gradient with the DenseNet concat-gradient epilogue (conv_igemm PRO 2 +
// EPI 2), gfx950.
//
// dgrad cv1 of a dense layer: dt = A2*z2 + B2*t + C2 (bn2's pending backward, 128 channels) times
// the transposed 1x1 kernel gives the gradient of the layer's input concat [0, cin); the epilogue
// masks it through bn1 + ReLU of the saved input x (= the stage buffer), reduces bn1's sums and
// ACCUMULATES gamma1*rstd1*dZ1 plus the previous BatchNorm's pending B'*x + C' into the fp32
// concat-gradient buffer.  On the 13x13 / 6x6 stages this op is a read-modify-write of M x cin
// fp32 (plus x) per layer: memory-bound.  The implicit-GEMM tiles re-stage the 128-deep A operand
// (z2 and t through the affine) once per 64-column tile, 2-8 times per layer, and ran at 1.4 TB/s
// (profiles/densenet121_bs256_bytes.md).
//
// Here a workgroup owns BM rows and a range of 32-column chunks.  The affine-applied A tile
// (BM x 128 bf16) is staged ONCE in LDS; its four waves then sweep the column chunks (wave w
// takes chunks w, w + 4, ...) without any further workgroup barrier: B fragments come straight
// from L2 into registers, the fp32 accumulators go through a per-wave LDS staging tile so every
// thread owns 8 consecutive channels of a row (32-B fp32 / 16-B bf16 accesses), and the next
// chunk's old accumulator and x are loaded before the current chunk is computed.  bn1's sums are
// reduced per wave with lane shuffles and added once per chunk.
// Selected by the autotuner as conv tile TILE_ROWS (conv_igemm.hip) where conv_rows_ok() holds.
#include "conv_igemm.h"

#include <algorithm>

namespace idc {

namespace {

constexpr int NT = 256;
constexpr int KD = 128;             // reduction depth (the bottleneck width)
constexpr int AS = KD * 2 + 32;     // A row stride in LDS (bytes): conflict-free fragment reads
constexpr int CW = 32;              // columns per chunk
constexpr int SLD = CW + 4;         // per-wave fp32 staging row (floats)
constexpr int MAXC = 2048;          // widest concat (LDS tables)

template <int BM>
int rows_smem_bytes(int cout) {
  return BM * AS + 4 * BM * SLD * 4 + (3 * KD + 6 * cout) * 4;
}

}  // namespace

template <int BM>
__global__ __launch_bounds__(256) void dgrad1x1_rows_kernel(ConvArgs a, GroupArg ga, int cpg) {
  prefetch_kernargs<sizeof(ConvArgs) + sizeof(GroupArg)>();
  gshift(a, goff(ga));
  constexpr int RF = BM / 16;       // row fragments per wave (every wave covers all BM rows)
  constexpr int IPL = BM * 4 / 64;  // epilogue items (row, 8 columns) per lane per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;
  float* stg_all = reinterpret_cast<float*>(smem + BM * AS);
  float* tA = stg_all + 4 * BM * SLD;  // bpro A / B / C [128]
  float* tB = tA + KD;
  float* tC = tB + KD;
  const int C = a.Cout;
  float* e0 = tC + KD;                 // bn1 scale, shift, mean, rstd [C]; bepi B', C' [C]
  float* e1 = e0 + C;
  float* e2 = e1 + C;
  float* e3 = e2 + C;
  float* pb = e3 + C;
  float* pc = pb + C;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.N * a.Ho * a.Wo;
  const int rb = blockIdx.x, g = blockIdx.y;
  const int m0 = rb * BM;
  const int nch = C / CW;
  const int ch0 = g * cpg, ch1 = min(nch, ch0 + cpg);

  // ---- A tile loads (z2 and the bpro input t), 16-B chunks, issued before the tables -----------
  constexpr int AQ = BM * (KD / 8) / NT;  // chunks per thread
  uint4 za[AQ], xa[AQ];
  const bf16_t* __restrict__ Z = reinterpret_cast<const bf16_t*>(a.x);
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    const int q = tid + i * NT, r = q / (KD / 8), c8 = q % (KD / 8);
    const int m = m0 + r < M ? m0 + r : 0;
    za[i] = *reinterpret_cast<const uint4*>(Z + (size_t)m * a.ldx + c8 * 8);
    xa[i] = *reinterpret_cast<const uint4*>(a.bpro.x + (size_t)m * a.bpro.ldx + c8 * 8);
  }
  // ---- tables -----------------------------------------------------------------------------------
  bwd_aff_table<NT>(a.bpro, 0, KD, KD, tA, tB, tC);
  bwd_aff_table<NT>(a.bepi, 0, C, C, e0, pb, pc);  // (e0 is scratch here: overwritten below)
  for (int c = tid; c < C; c += NT) {
    float sc = 1.f, sh = 0.f, mean = 0.f, rstd = 1.f;
    if (a.mbn.mode) {
      bn_mean_rstd(a.mbn, c, mean, rstd);
      const float gm = a.mbn.gamma ? a.mbn.gamma[c] : 1.f;
      const float be = a.mbn.beta ? a.mbn.beta[c] : 0.f;
      sc = gm * rstd;
      sh = be - mean * sc;
    }
    e0[c] = sc; e1[c] = sh; e2[c] = mean; e3[c] = rstd;
  }
  bwd_aff_fold<NT>(a.bpro);  // (every workgroup folds its share)
  __syncthreads();
  // ---- stage A once: dt = A2*z2 + B2*t + C2 (bf16), also stored for the side-lane wgrad ----------
  const bool aout_on = a.aout != nullptr && g == 0;
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    const int q = tid + i * NT, r = q / (KD / 8), c8 = q % (KD / 8);
    float f[8], xf[8];
    unpack8(za[i], f);
    unpack8(xa[i], xf);
    bwd_aff8(f, xf, tA + c8 * 8, tB + c8 * 8, tC + c8 * 8);
    uint4 v = pack8(f);
    const bool ok = m0 + r < M;
    if (aout_on && ok) *reinterpret_cast<uint4*>(a.aout + (size_t)(m0 + r) * a.ldaout + c8 * 8) = v;
    if (!ok) v = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(sA + r * AS + c8 * 16) = v;
  }
  __syncthreads();

  // ---- column chunks, one wave each, no workgroup barrier from here on -------------------------
  float* stg = stg_all + wid * BM * SLD;
  const float mlo = act_lo(a.mbn.act), mhi = act_hi(a.mbn.act);
  const int kc = lane >> 4;
  // epilogue items of this lane: row er = (lane >> 2) + 16 * i, columns (lane & 3) * 8 .. + 8
  const int ec8 = lane & 3;
  float4 o0[IPL], o1[IPL];
  uint4 xv[IPL];
  auto load_epi = [&](int ch) {
#pragma unroll
    for (int i = 0; i < IPL; ++i) {
      const int r = (lane >> 2) + 16 * i;
      const int m = m0 + r < M ? m0 + r : 0;
      const int n = ch * CW + ec8 * 8;
      const float* yp = reinterpret_cast<const float*>(a.y) + (size_t)m * a.ldy + n;
      o0[i] = *reinterpret_cast<const float4*>(yp);
      o1[i] = *reinterpret_cast<const float4*>(yp + 4);
      xv[i] = *reinterpret_cast<const uint4*>(a.mx + (size_t)m * a.ldmx + n);
    }
  };
  const bf16_t* __restrict__ Wt = a.w;
  int ch = ch0 + wid;
  if (ch < ch1) load_epi(ch);
  for (; ch < ch1; ch += 4) {
    // B fragments of this chunk (L2): column n = ch*32 + 16 j + (lane & 15), k = 32 s + 8 kc
    v8bf bfr[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[s][j] = *reinterpret_cast<const v8bf*>(Wt + (size_t)(ch * CW + 16 * j + (lane & 15)) * KD + 32 * s + 8 * kc);
    v4f acc[RF][2];
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        const v8bf af = *reinterpret_cast<const v8bf*>(sA + (16 * i + (lane & 15)) * AS + (32 * s + 8 * kc) * 2);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[s][j], acc[i][j], 0, 0, 0);
      }
    // stage the fp32 tile (wave-private), then this lane's (row, 8 columns) items
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          stg[(16 * i + (lane >> 4) * 4 + q) * SLD + 16 * j + (lane & 15)] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the staging writes landed (wave-local)
    __builtin_amdgcn_wave_barrier();
    float4 c0[IPL], c1[IPL];
    uint4 cx[IPL];
#pragma unroll
    for (int i = 0; i < IPL; ++i) { c0[i] = o0[i]; c1[i] = o1[i]; cx[i] = xv[i]; }
    const int cur = ch;
    if (ch + 4 < ch1) load_epi(ch + 4);  // next chunk's accumulator and x, in flight meanwhile
    const int nb = cur * CW + ec8 * 8;
    float t0[8], t1[8], t2[8], t3[8], tpb[8], tpc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      t0[j] = e0[nb + j]; t1[j] = e1[nb + j]; t2[j] = e2[nb + j]; t3[j] = e3[nb + j];
      tpb[j] = pb[nb + j]; tpc[j] = pc[nb + j];
    }
    float psum[8], psq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { psum[j] = 0.f; psq[j] = 0.f; }
#pragma unroll
    for (int i = 0; i < IPL; ++i) {
      const int r = (lane >> 2) + 16 * i;
      const float4 lo = *reinterpret_cast<const float4*>(&stg[r * SLD + ec8 * 8]);
      const float4 hi = *reinterpret_cast<const float4*>(&stg[r * SLD + ec8 * 8 + 4]);
      const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const float old[8] = {c0[i].x, c0[i].y, c0[i].z, c0[i].w, c1[i].x, c1[i].y, c1[i].z, c1[i].w};
      float xf[8], o[8];
      unpack8(cx[i], xf);
      const bool ok = m0 + r < M;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = xf[j] * t0[j] + t1[j];
        const float d = (ok && z > mlo && z < mhi) ? v[j] : 0.f;
        psum[j] += d;
        psq[j] += d * (xf[j] - t2[j]) * t3[j];
        o[j] = old[j] + fmaf(t0[j], d, fmaf(tpb[j], xf[j], tpc[j]));
      }
      if (ok) {
        float* yp = reinterpret_cast<float*>(a.y) + (size_t)(m0 + r) * a.ldy + nb;
        *reinterpret_cast<float4*>(yp) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(yp + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
    }
    // bn1's sums over this workgroup's rows: lanes with equal (lane & 3) share columns
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int sh = 4; sh < 64; sh <<= 1) {
        psum[j] += __shfl_xor(psum[j], sh, 64);
        psq[j] += __shfl_xor(psq[j], sh, 64);
      }
    }
    if (lane < 4) {
      const size_t so = (size_t)(rb % stat_slots(a.gsum_slots)) * a.gsum_ld;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (a.gsum) atomicAdd(&a.gsum[so + nb + j], psum[j]);
        if (a.gsumx) atomicAdd(&a.gsumx[so + nb + j], psq[j]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the staging tile is rewritten by the next chunk
  }
}

// ---------------------------------------------------------------------------------------------
bool conv_rows_ok(const ConvArgs& a, bool a_f32) {
  return !a_f32 && a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0 &&
         a.H == a.Ho && a.W == a.Wo && a.Cin == KD && a.bpro.mode != 0 && a.bpro.x != nullptr &&
         a.epi_mode == 2 && a.mx != nullptr && a.Cout % CW == 0 && a.Cout <= MAXC && a.ksplit <= 1 &&
         (a.ldx % 8) == 0 && (a.ldy % 8) == 0 && (a.ldmx % 8) == 0 && (a.bpro.ldx % 8) == 0 &&
         (a.aout == nullptr || (a.ldaout % 8) == 0) && a.pro.mode == 0 && a.pro.act == ACT_NONE;
}

hipError_t conv_rows(const ConvArgs& a, bool a_f32, hipStream_t st) {
  if (!conv_rows_ok(a, a_f32)) return hipErrorInvalidValue;
  const int M = a.N * a.Ho * a.Wo;
  const int nch = a.Cout / CW;
  // 64-row blocks where they make >= 512 workgroups, else 32-row blocks; columns split so that a
  // launch has ~512 workgroups while every wave keeps >= 1 chunk
  const bool big = (M + 63) / 64 >= 512;
  const int bm = big ? 64 : 32;
  const int rbs = (M + bm - 1) / bm;
  int groups = (512 + rbs - 1) / rbs;
  groups = std::max(1, std::min(groups, (nch + 3) / 4));
  const int cpg = (nch + groups - 1) / groups;
  groups = (nch + cpg - 1) / cpg;
  const dim3 grid = ggrid(dim3(rbs, groups));
  if (big)
    hipLaunchKernelGGL(dgrad1x1_rows_kernel<64>, grid, dim3(NT), rows_smem_bytes<64>(a.Cout), st, a,
                       garg(), cpg);
  else
    hipLaunchKernelGGL(dgrad1x1_rows_kernel<32>, grid, dim3(NT), rows_smem_bytes<32>(a.Cout), st, a,
                       garg(), cpg);
  return hipGetLastError();
}

}  // namespace idc
