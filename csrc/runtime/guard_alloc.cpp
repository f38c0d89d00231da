// Guard-page device allocator (debugging only: tools/guard_pages.py).
//
// Installed as torch's CURRENT allocator (torch.cuda.memory.change_current_allocator, before the
// first device allocation), so every tensor is its own allocation -- no caching, no splitting.
// Each allocation reserves a virtual range of the mapped size plus one granule, maps physical
// memory over all but that granule, and returns a pointer placed so that the tensor ENDS at the
// last mapped byte (IDC_GUARD_SIDE=end, default) or STARTS at the first mapped byte right after an
// unmapped granule (IDC_GUARD_SIDE=start).  A kernel that reads or writes past the end (or before
// the start) of any tensor then touches an unmapped page and faults at once, in its own dispatch,
// instead of silently reading a neighbour -- which is what only happens to fault when the caching
// allocator has happened to put a tensor at the end of a segment.
//
// Frees synchronise the device first (a pluggable allocator gets no stream ordering from torch).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace {

struct GuardBlock {
  uintptr_t va = 0;  // reserved range base
  size_t reserved = 0;
  size_t mapped = 0;
  uintptr_t map_at = 0;  // first mapped byte
  hipMemGenericAllocationHandle_t handle{};
};

std::mutex g_mu;
std::unordered_map<uintptr_t, GuardBlock> g_blocks;  // user pointer -> block
size_t g_gran = 0;
bool g_start_side = false;
long long g_live = 0, g_total = 0;

size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }

hipMemAllocationProp prop_for(int device) {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof(p));
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

}  // namespace

extern "C" __attribute__((visibility("default"))) void* idc_guard_malloc(size_t size, int device,
                                                                        hipStream_t stream) {
  (void)stream;
  std::lock_guard<std::mutex> l(g_mu);
  hipMemAllocationProp prop = prop_for(device);
  if (!g_gran) {
    if (hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess ||
        !g_gran)
      return nullptr;
    const char* side = std::getenv("IDC_GUARD_SIDE");
    g_start_side = side && std::strcmp(side, "start") == 0;
  }
  const size_t body = round_up(size ? size : 1, 256);  // torch and MIOpen assume >= 256 B alignment
  GuardBlock b;
  b.mapped = round_up(body, g_gran);
  b.reserved = b.mapped + g_gran;
  void* va = nullptr;
  if (hipMemAddressReserve(&va, b.reserved, g_gran, nullptr, 0) != hipSuccess) return nullptr;
  b.va = reinterpret_cast<uintptr_t>(va);
  b.map_at = g_start_side ? b.va + g_gran : b.va;
  if (hipMemCreate(&b.handle, b.mapped, &prop, 0) != hipSuccess) {
    (void)hipMemAddressFree(va, b.reserved);
    return nullptr;
  }
  if (hipMemMap(reinterpret_cast<void*>(b.map_at), b.mapped, 0, b.handle, 0) != hipSuccess) {
    (void)hipMemRelease(b.handle);
    (void)hipMemAddressFree(va, b.reserved);
    return nullptr;
  }
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof(acc));
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = device;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(reinterpret_cast<void*>(b.map_at), b.mapped, &acc, 1) != hipSuccess) {
    (void)hipMemUnmap(reinterpret_cast<void*>(b.map_at), b.mapped);
    (void)hipMemRelease(b.handle);
    (void)hipMemAddressFree(va, b.reserved);
    return nullptr;
  }
  const uintptr_t user = g_start_side ? b.map_at : b.map_at + b.mapped - body;
  g_blocks[user] = b;
  ++g_live;
  ++g_total;
  return reinterpret_cast<void*>(user);
}

extern "C" __attribute__((visibility("default"))) void idc_guard_free(void* ptr, size_t size, int device,
                                                                     hipStream_t stream) {
  (void)size;
  (void)device;
  (void)stream;
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_blocks.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == g_blocks.end()) return;
  const GuardBlock b = it->second;
  g_blocks.erase(it);
  (void)hipDeviceSynchronize();  // work still reading the block must finish before it unmaps
  (void)hipMemUnmap(reinterpret_cast<void*>(b.map_at), b.mapped);
  (void)hipMemRelease(b.handle);
  (void)hipMemAddressFree(reinterpret_cast<void*>(b.va), b.reserved);
  --g_live;
}

// allocation counters for the harness: (live blocks, blocks allocated so far, granule bytes)
extern "C" __attribute__((visibility("default"))) long long idc_guard_stats(int which) {
  std::lock_guard<std::mutex> l(g_mu);
  return which == 0 ? g_live : which == 1 ? g_total : (long long)g_gran;
}
