// Phase timing of the image-resident 3x3 kernel (csrc/kernels/conv_img.hip) on DenseNet-121
// stage-1 / stage-2 shapes at batch 256: s_memtime stamps from thread 0 of every workgroup (the
// IDC_IMG_STAMP hooks), median over workgroups, in shader cycles since kernel entry; plus the
// event-timed launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels -o /tmp/img_phases tools/micro/img_phases.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ unsigned long long g_stamps[4096][16];
__device__ unsigned long long g_real[4096][2];
#define IDC_IMG_STAMP(i)                                                                     \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                            \
      g_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                               \
      if (i == 0) g_real[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();                 \
      if (i == 9) g_real[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();                 \
    }                                                                                       \
  } while (0)
#include "conv_img.hip"

using namespace idc;
namespace idc {
LaunchGroups& launch_groups() {
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

static void run(const char* name, int N, int H, int form) {
  ConvArgs a{};
  const int M = N * H * H;
  const int cin = form == 1 ? 128 : 32, cout = form == 1 ? 32 : 128;
  a.N = N; a.H = H; a.W = H; a.Ho = H; a.Wo = H;
  a.Cin = cin; a.ldx = cin; a.Cout = cout; a.ldy = cout;
  a.KH = a.KW = 3; a.SH = a.SW = 1; a.PT = a.PL = 1;
  a.x = dalloc((size_t)M * cin * 4);
  a.w = (const bf16_t*)dalloc((size_t)9 * cin * cout * 2);
  a.y = dalloc((size_t)M * cout * 4);
  float* stats = (float*)dalloc(1 << 20);
  float* gam = (float*)dalloc(1 << 16);
  a.ksplit = 1;
  a.tickets = (unsigned*)dalloc(4 * (17 + 16 * 2 * cout));  // slot copies of the reductions
  a.tickets_n = 17 + 16 * 2 * cout;
  a.stats_slots = a.gsum_slots = 1;
  a.gsum_ld = cout;
  a.out_mode = OUT_BF16;
  if (form == 1) {
    a.pro = BnArgs{stats, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 1, cin, 1, nullptr};
    a.stats_out = stats + 4096; a.stats_ld = cout;
  } else {
    a.bpro.x = (const bf16_t*)dalloc((size_t)M * cin * 2);
    a.bpro.ldx = cin;
    a.bpro.bn = BnArgs{stats, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 0, cin, 1, nullptr};
    a.bpro.gsum = stats + 8192; a.bpro.gsumx = stats + 16384;
    a.bpro.gsum_slots = 1; a.bpro.gsum_ld = cin; a.bpro.inv_n = 1.f / M; a.bpro.mode = 1; a.bpro.unit_alpha = 1;
    a.epi_mode = 1;
    a.mx = (const bf16_t*)dalloc((size_t)M * cout * 2); a.ldmx = cout;
    a.mbn = BnArgs{stats + 32768, gam, gam, nullptr, nullptr, 1.f / M, 1e-3f, 1, 1, cout, 1, nullptr};
    a.gsum = stats + 65536; a.gsumx = stats + 65536 + 1024;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) conv_img(a, form == 2, nullptr);
  hipDeviceSynchronize();
  hipEventRecord(e0, nullptr);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) conv_img(a, form == 2, nullptr);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(4096 * 16);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  printf("%s: %.2f us/launch (err %s)\n  phase median cycles since entry:", name, ms * 1e3 / reps,
         hipGetErrorString(hipGetLastError()));
  for (int k = 1; k < 12; ++k) {
    std::vector<long long> d;
    for (int b = 0; b < N && b < 4096; ++b) d.push_back((long long)(st[b * 16 + k] - st[b * 16]));
    std::sort(d.begin(), d.end());
    printf(" [%d] %lld", k, d[d.size() / 2]);
  }
  // workgroup start / end times (s_memrealtime, 100 MHz, device-wide) relative to the first start
  std::vector<unsigned long long> rt(4096 * 2);
  hipMemcpyFromSymbol(rt.data(), HIP_SYMBOL(g_real), rt.size() * 8);
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < N; ++b) t0 = std::min(t0, rt[b * 2]);
  std::vector<long long> s0, s1;
  for (int b = 0; b < N; ++b) { s0.push_back((long long)(rt[b * 2] - t0)); s1.push_back((long long)(rt[b * 2 + 1] - t0)); }
  std::sort(s0.begin(), s0.end());
  std::sort(s1.begin(), s1.end());
  printf("\n  starts (10 ns ticks): p10 %lld p50 %lld p90 %lld max %lld | ends: p10 %lld p50 %lld max %lld\n",
         s0[N / 10], s0[N / 2], s0[N * 9 / 10], s0.back(), s1[N / 10], s1[N / 2], s1.back());
  int late = 0;
  for (int b = 0; b < N; ++b) late += s0[b] > s1[0];
  printf("  workgroups starting after the first one ended: %d of %d\n", late, N);
}

int main() {
  run("fwd 13x13 128->32", 256, 13, 1);
  run("fwd 6x6 128->32", 256, 6, 1);
  run("dgrad 13x13 32->128", 256, 13, 2);
  run("dgrad 6x6 32->128", 256, 6, 2);
  return 0;
}
