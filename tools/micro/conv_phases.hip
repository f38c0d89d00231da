// Phase timing of the implicit-GEMM conv kernel on DenseNet tail shapes: s_memtime stamps
// (IDC_PHASE_STAMP hooks in conv_igemm_impl.h) from thread 0 of every workgroup, median over
// workgroups and launches, in shader cycles since kernel entry.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels -o /tmp/conv_phases tools/micro/conv_phases.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ unsigned long long g_stamps[4096][16];
__device__ unsigned long long g_rt[4096][2];  // s_memrealtime (100 MHz, chip-wide) at entry / end
#define IDC_PHASE_STAMP(i)                                                                  \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                            \
      g_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                               \
      if ((i) == 0) g_rt[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();                 \
      if ((i) == 10) g_rt[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();                \
    }                                                                                       \
  } while (0)
#include "conv_igemm_impl.h"

using namespace idc;
namespace idc {
LaunchGroups& launch_groups() {  // (defined in nn_kernels.hip in the extension)
  static LaunchGroups l;
  return l;
}
}  // namespace idc

static void* dalloc(size_t bytes) {
  void* p = nullptr;
  hipMalloc(&p, bytes);
  hipMemset(p, 0, bytes);
  return p;
}

struct Case {
  const char* name;
  int M, Cin, Cout, pro, epi, a_f32, tile;
};

template <int BM, int BN, int BK, int WM, int WN>
static void run_case(const Case& c) {
  ConvArgs a{};
  const int M = c.M;
  a.N = M; a.H = 1; a.W = 1; a.Ho = 1; a.Wo = 1;
  a.Cin = c.Cin; a.ldx = c.Cin; a.Cout = c.Cout; a.ldy = c.Cout;
  a.KH = a.KW = a.SH = a.SW = 1;
  a.x = dalloc((size_t)M * c.Cin * 4);
  a.w = (const bf16_t*)dalloc((size_t)c.Cout * c.Cin * 2);
  a.y = dalloc((size_t)M * c.Cout * 4);
  float* stats = (float*)dalloc(1 << 20);
  float* gam = (float*)dalloc(1 << 16);
  a.ksplit = 1;
  a.stats_slots = a.gsum_slots = 1;
  if (const char* e = getenv("IDC_MICRO_GSUM_SLOTS")) a.gsum_slots = atoi(e);  // epilogue sum copies
  a.gsum_ld = c.Cout;
  if (c.pro == 1) {
    a.pro = BnArgs{stats, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 1, c.Cin, 1};
  }
  if (c.pro == 2) {
    a.bpro.x = (const bf16_t*)dalloc((size_t)M * c.Cin * 2);
    a.bpro.ldx = c.Cin;
    a.bpro.bn = BnArgs{stats, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 1, c.Cin, 1};
    a.bpro.gsum = stats + 8192; a.bpro.gsumx = stats + 16384;
    a.bpro.gsum_slots = 1; a.bpro.gsum_ld = c.Cin; a.bpro.inv_n = 1.f / M; a.bpro.mode = 1;
    a.bpro.unit_alpha = c.a_f32;
  }
  if (c.epi == 0) {
    a.out_mode = OUT_BF16; a.stats_out = stats + 32768; a.stats_ld = c.Cout;
  } else {
    a.mx = (const bf16_t*)dalloc((size_t)M * c.Cout * 2); a.ldmx = c.Cout;
    a.mbn = BnArgs{stats, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 1, c.Cout, 1};
    a.gsum = stats + 65536; a.gsumx = stats + 131072;
    if (c.epi == 2) {
      a.bepi = a.bpro;
      a.bepi.x = a.mx; a.bepi.ldx = c.Cout; a.bepi.bn.C = c.Cout; a.bepi.unit_alpha = 1;
      a.bepi.gsum_ld = c.Cout;
    }
  }
  hipStream_t st;
  hipStreamCreate(&st);
  const int R = 30;
  std::vector<std::vector<long long>> ph(15);
  std::vector<long long> tot;
  for (int r = 0; r < R; ++r) {
    hipMemset(g_stamps, 0, 0);  // no-op keeps symbol referenced
    if (launch_cfg<BM, BN, BK, WM, WN>(a, true, c.a_f32, c.pro, c.epi, st) != hipSuccess) {
      printf("%s: launch failed\n", c.name);
      return;
    }
    hipStreamSynchronize(st);
    static unsigned long long h[4096][16];
    hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamps), sizeof(h));
    const int tiles = ((M + BM - 1) / BM) * ((c.Cout + BN - 1) / BN);
    if (r < 3) continue;
    for (int b = 0; b < std::min(tiles, 4096); ++b) {
      for (int i = 1; i <= 14; ++i)
        if (h[b][i] >= h[b][0] && h[b][i] - h[b][0] < 1000000) ph[i].push_back((long long)(h[b][i] - h[b][0]));
    }
  }
  // kernel span and per-workgroup lifetime (entry -> end, s_memrealtime: 100 MHz, chip-wide) of
  // the last launch; start-time deciles show how fast workgroups get a slot
  {
    static unsigned long long h[4096][2];
    hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rt), sizeof(h));
    const int tiles = std::min(4096, ((M + BM - 1) / BM) * ((c.Cout + BN - 1) / BN));
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<long long> life, starts;
    for (int b = 0; b < tiles; ++b) {
      if (!h[b][0] || !h[b][1] || h[b][1] < h[b][0]) continue;
      t0 = std::min(t0, h[b][0]);
      t1 = std::max(t1, h[b][1]);
      life.push_back((long long)(h[b][1] - h[b][0]));
      starts.push_back((long long)h[b][0]);
    }
    if (!life.empty()) {
      long long sum = 0;
      for (long long v : life) sum += v;
      std::sort(life.begin(), life.end());
      std::sort(starts.begin(), starts.end());
      const size_t n = life.size();
      printf("%-34s span=%.1f us  WG life p10/p50/p90/max=%.1f/%.1f/%.1f/%.1f us  mean concurrency=%.0f WGs  start "
             "deciles(us):", c.name, (t1 - t0) / 100.0, life[n / 10] / 100.0, life[n / 2] / 100.0,
             life[n * 9 / 10] / 100.0, life[n - 1] / 100.0, (double)sum / (double)(t1 - t0));
      for (int d = 1; d <= 9; ++d) printf(" %.1f", (starts[n * d / 10] - t0) / 100.0);
      printf("\n");
    }
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, st);
  for (int r = 0; r < 20; ++r) launch_cfg<BM, BN, BK, WM, WN>(a, true, c.a_f32, c.pro, c.epi, st);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-34s back-to-back %.2f us/launch\n", c.name, ms * 1000.f / 20);
  a.epi_mode = c.epi;
  printf("%-34s tiles=%d  cycles since entry (median over WGs x launches):", c.name,
         ((M + BM - 1) / BM) * ((c.Cout + BN - 1) / BN));
  const char* lbl[] = {"", "tiles_issued", "pro_tab", "epi2_tab", "epi_tab", "ep_prefetch", "loop_start", "loop_end",
                       "epilogue", "stats_red", "end", "epi_start", "epi_p0_sync", "wave_red", "red_sync1"};
  for (int i = 1; i <= 14; ++i) {
    auto& v = ph[i];
    if (v.empty()) { printf(" %s=-", lbl[i]); continue; }
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    printf(" %s=%lld", lbl[i], v[v.size() / 2]);
  }
  printf("\n");
  hipStreamDestroy(st);
}

int main() {
  // DenseNet-121 bs256 concat-gradient dgrads (cv1, PRO 2 + EPI 2) of stages 1 / 2
  run_case<64, 64, 32, 2, 2>({"bwd s1 dg1 pro2 epi2 K128 N224 t3", 43264, 128, 224, 2, 2, 0, 0});
  run_case<64, 64, 32, 2, 2>({"bwd s1 dg1 pro2 epi2 K128 N64 t3", 43264, 128, 64, 2, 2, 0, 0});
  run_case<128, 32, 64, 4, 1>({"bwd s1 dg1 pro2 epi2 K128 N64 t7", 43264, 128, 64, 2, 2, 0, 0});
  run_case<64, 64, 32, 2, 2>({"bwd s2 dg1 pro2 epi2 K128 N480 t3", 9216, 128, 480, 2, 2, 0, 0});
  run_case<64, 64, 64, 2, 2>({"bwd s2 dg1 pro2 epi2 K128 N480 t8", 9216, 128, 480, 2, 2, 0, 0});
  if (getenv("IDC_PHASES_DG_ONLY")) return 0;
  // DenseNet-121 bs256 stage-1/2 1x1 shapes (M = 43264 / 9216)
  run_case<256, 32, 32, 4, 1>({"fwd s1 1x1 pro1 epi0 K64 t2", 43264, 64, 128, 1, 0, 0, 0});
  run_case<64, 32, 64, 2, 2>({"fwd s1 1x1 pro1 epi0 K64 t9", 43264, 64, 128, 1, 0, 0, 0});
  run_case<64, 32, 64, 2, 2>({"fwd s1 1x1 pro0 epi0 K64 t9", 43264, 64, 128, 0, 0, 0, 0});
  run_case<64, 32, 64, 2, 2>({"fwd s2 1x1 pro1 epi0 K480 t9", 9216, 480, 128, 1, 0, 0, 0});
  // DenseNet-121 bs256 tail shapes (stage 4: M=256, stage 3: M=2304)
  run_case<64, 32, 64, 2, 2>({"fwd s4 1x1 pro1 epi0 K544", 256, 544, 128, 1, 0, 0, 0});
  run_case<64, 32, 64, 2, 2>({"fwd s3 1x1 pro1 epi0 K544", 2304, 544, 128, 1, 0, 0, 0});
  run_case<64, 32, 32, 2, 2>({"bwd s4 dg2 pro2 epi1 f32 K32", 256, 32, 128, 2, 1, 1, 0});
  run_case<64, 32, 64, 2, 2>({"bwd s4 dg1 pro2 epi2 K128 N992", 256, 128, 992, 2, 2, 0, 0});
  run_case<64, 64, 32, 2, 2>({"bwd s3 dg1 pro2 epi2 K128 N992", 2304, 128, 992, 2, 2, 0, 0});
  run_case<64, 32, 32, 2, 2>({"fwd s4 1x1 pro0 epi0 K544", 256, 544, 128, 0, 0, 0, 0});
  return 0;
}
