// Event-timed launches of the inference-mode dense block (csrc/kernels/dense_infer.hip) at
// DenseNet-121's stage-1 / stage-2 shapes (bs 256, 50x50), for A/B of kernel variants:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -Icsrc/kernels \
//       -o /tmp/di_time tools/micro/di_time.hip
#include "dense_infer.hip"
#include <cstdio>
#include <vector>

namespace idc {
LaunchGroups& launch_groups() {  // (the plan executor's; one ungrouped launch here)
  static LaunchGroups g{};
  return g;
}
}  // namespace idc
using namespace idc;

template <typename T>
static T* dalloc(size_t n, float scale) {
  std::vector<T> h(n);
  unsigned s = 12345;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float v = ((s >> 8) * (1.f / 16777216.f) - 0.5f) * scale;
    if constexpr (sizeof(T) == 2) {
      const unsigned u = __builtin_bit_cast(unsigned, v);
      h[i] = (T)(u >> 16);
    } else {
      h[i] = (T)v;
    }
  }
  T* p = nullptr;
  hipMalloc(&p, n * sizeof(T));
  hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice);
  return p;
}

static void run(int N, int H, int c0, int L) {
  const int ld = c0 + 32 * L;
  std::vector<DenseLayerDesc> lay(L);
  for (int l = 0; l < L; ++l) {
    const int cin = c0 + 32 * l;
    DenseLayerDesc& d = lay[l];
    d = DenseLayerDesc{};
    d.w1 = dalloc<bf16_t>((size_t)128 * cin, 0.1f);
    d.w2 = dalloc<bf16_t>((size_t)32 * 1152, 0.05f);
    d.g1 = dalloc<float>(cin, 0.5f);
    d.b1 = dalloc<float>(cin, 0.2f);
    d.g2 = dalloc<float>(128, 0.5f);
    d.b2 = dalloc<float>(128, 0.2f);
    d.mm1 = dalloc<float>(cin, 0.1f);
    std::vector<float> one(cin > 128 ? cin : 128, 1.f);
    float* mv1;
    hipMalloc(&mv1, cin * 4);
    hipMemcpy(mv1, one.data(), cin * 4, hipMemcpyHostToDevice);
    d.mv1 = mv1;
    d.mm2 = dalloc<float>(128, 0.1f);
    float* mv2;
    hipMalloc(&mv2, 128 * 4);
    hipMemcpy(mv2, one.data(), 128 * 4, hipMemcpyHostToDevice);
    d.mv2 = mv2;
    d.eps1 = d.eps2 = 1e-3f;
    d.cin = cin;
  }
  DenseLayerDesc* dl;
  hipMalloc(&dl, L * sizeof(DenseLayerDesc));
  hipMemcpy(dl, lay.data(), L * sizeof(DenseLayerDesc), hipMemcpyHostToDevice);
  DenseInferArgs a{};
  a.buf = dalloc<bf16_t>((size_t)N * H * H * ld, 2.f);
  a.ld = ld;
  a.N = N;
  a.H = H;
  a.W = H;
  a.c0 = c0;
  a.L = L;
  a.ipg = 1;
  a.act = 1;
  a.layers = dl;
  for (int i = 0; i < 3; ++i) dense_infer(a, nullptr);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 20;
  hipEventRecord(e0, nullptr);
  for (int i = 0; i < reps; ++i) dense_infer(a, nullptr);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("N=%d H=%d c0=%d L=%d: %.1f us/launch (%s)\n", N, H, c0, L, ms * 1e3 / reps, hipGetErrorString(hipGetLastError()));
}

int main() {
  run(256, 13, 64, 6);
  run(256, 6, 128, 12);
  return 0;
}
