// Phase timing of the MobileNetV2 inference-block kernel (csrc/kernels/mb_infer.hip) on the
// MobileNetV2 @50x50, batch 256 block shapes: s_memrealtime stamps (100 MHz) from thread 0 of every
// workgroup at the IDC_MBI_STAMP hooks, median over workgroups in microseconds since the
// workgroup's entry, plus the event-timed launch and the spread of workgroup start times.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -Icsrc/kernels \
//       -o /tmp/mbi_phases tools/micro/mbi_phases.hip
// Phases: 1 tables, 2 weights + input staged, 3 first chunk through the depthwise, 4 chunk loop
// done, 5 partial published / ticket taken (split launches), 6 last arriver summed, 7 stored.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ unsigned long long g_stamps[8192][8];
#define IDC_MBI_STAMP(i)                                                                  \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#include "mb_infer.hip"

using namespace idc;

static void* dalloc(size_t bytes) {
  void* p = nullptr;
  hipMalloc(&p, bytes);
  hipMemset(p, 0, bytes);
  return p;
}

static BnArgs bn_inf(int C, int act) {
  float* p = (float*)dalloc(4 * C * 4);
  std::vector<float> h(4 * C);
  for (int c = 0; c < C; ++c) { h[c] = 1.f; h[C + c] = 0.1f; h[2 * C + c] = 0.f; h[3 * C + c] = 1.f; }
  hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  return BnArgs{nullptr, p, p + C, p + 2 * C, p + 3 * C, 1.f, 1e-3f, 2, act, C, 1, nullptr};
}

static void run(const char* name, int N, int H, int Cin, int Cexp, int Cout, int S, int res, int ipg, int cs) {
  MbInferArgs a{};
  const int pt = S == 1 ? 1 : (H % 2 ? 1 : 0), pl = pt;
  const int Ho = S == 1 ? H : (H + 1) / 2, Wo = Ho;
  a.x = (const bf16_t*)dalloc((size_t)N * H * H * Cin * 2); a.ldx = Cin;
  a.xbn = BnArgs{nullptr, nullptr, nullptr, nullptr, nullptr, 1.f, 1e-3f, 0, 0, Cin, 1, nullptr};
  a.we = Cexp != Cin || S == 2 ? (const bf16_t*)dalloc((size_t)Cexp * Cin * 2) : nullptr;
  a.ebn = bn_inf(Cexp, 2);
  a.wd = (const float*)dalloc((size_t)9 * Cexp * 4);
  a.dbn = bn_inf(Cexp, 2);
  a.wp = (const bf16_t*)dalloc((size_t)Cout * Cexp * 2);
  a.pbn = bn_inf(Cout, 0);
  a.y = (bf16_t*)dalloc((size_t)N * Ho * Wo * Cout * 2); a.ldy = Cout;
  a.N = N; a.H = H; a.W = H; a.Cin = Cin; a.Cexp = Cexp; a.Cout = Cout; a.Ho = Ho; a.Wo = Wo;
  a.S = S; a.PT = pt; a.PL = pl; a.residual = res; a.ipg = ipg; a.cs = cs;
  a.tickets = (unsigned*)dalloc(4 * 4096);
  a.slab = (float*)dalloc((size_t)mb_infer_slab_floats(a) * 4 + 16);
  const long long smem = mb_infer_smem(a);
  if (smem < 0) { printf("%s: shape rejected\n", name); return; }
  const int grid = ((N + ipg - 1) / ipg) * ((Cexp + cs - 1) / cs);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) mb_infer(a, nullptr);
  hipDeviceSynchronize();
  hipEventRecord(e0, nullptr);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) mb_infer(a, nullptr);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(8192 * 8);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  printf("%s: grid %d, LDS %lld B, %.2f us/launch (err %s)\n  phase median us since entry:", name, grid, smem,
         ms * 1e3 / reps, hipGetErrorString(hipGetLastError()));
  for (int k = 1; k < 8; ++k) {
    std::vector<long long> d;
    for (int b = 0; b < grid && b < 8192; ++b)
      if (st[b * 8 + k] >= st[b * 8]) d.push_back((long long)(st[b * 8 + k] - st[b * 8]));
    std::sort(d.begin(), d.end());
    if (d.empty()) { printf(" [%d] -", k); continue; }
    printf(" [%d] %.2f", k, d[d.size() / 2] / 100.0);
  }
  std::vector<long long> s0;
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < grid && b < 8192; ++b) t0 = std::min(t0, st[b * 8]);
  for (int b = 0; b < grid && b < 8192; ++b) s0.push_back((long long)(st[b * 8] - t0));
  std::sort(s0.begin(), s0.end());
  printf("\n  workgroup starts (us after the first): p50 %.2f p90 %.2f max %.2f\n", s0[s0.size() / 2] / 100.0,
         s0[s0.size() * 9 / 10] / 100.0, s0.back() / 100.0);
}

int main() {
  run("b0 25x25 32->32->16", 256, 25, 32, 32, 16, 1, 0, 1, 32);
  run("b1 25x25 16->96->24 s2", 256, 25, 16, 96, 24, 2, 0, 1, 96);
  run("b2 13x13 24->144->24", 256, 13, 24, 144, 24, 1, 1, 1, 160);
  run("b4 7x7 32->192->32 ipg2", 256, 7, 32, 192, 32, 1, 1, 2, 96);
  run("b7 4x4 64->384->64 ipg4 cs96", 256, 4, 64, 384, 64, 1, 1, 4, 96);
  run("b7 4x4 64->384->64 ipg4 cs384", 256, 4, 64, 384, 64, 1, 1, 4, 384);
  run("b14 2x2 160->960->160 ipg16 cs64", 256, 2, 160, 960, 160, 1, 1, 16, 64);
  run("b14 2x2 160->960->160 ipg4 cs128", 256, 2, 160, 960, 160, 1, 1, 4, 128);
  run("b16 2x2 160->960->320 ipg16 cs64", 256, 2, 160, 960, 320, 1, 0, 16, 64);
  return 0;
}
