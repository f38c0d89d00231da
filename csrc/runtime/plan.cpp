// Native execution plan for the idc_models_amd MI355X runtime.
//
// The Python lowering (idc_models_amd/runtime) turns a model + batch shape into a STATIC list of
// kernel launches over preallocated arenas (activations, statistics, gradients, weights).  This
// file owns that list: ops are appended once (argument structs copied in as raw bytes whose
// layout is mirrored by ctypes on the Python side and checked via `struct_sizes()`), then
//
//   * run(begin, end, stream)        issues ops[begin:end] back-to-back from C++ (no Python per
//                                     kernel), used for eager steps and for segment replays;
//   * capture(begin, end, stream)    records ops[begin:end] into a hipGraph (thread-local capture
//                                     mode) and instantiates it -> graph id;
//   * launch(graph, stream)          replays a captured segment: one host call per segment.
//
// A training step is typically 3 graphs (forward, backward, optimizer) or, under data
// parallelism, backward split into bucket-aligned segments so RCCL all-reduces (issued by
// torch.distributed on its own stream) overlap the remaining backward segments.
//
// Lanes: an op tagged lane 1 runs on the plan's SIDE stream, forked from the main stream at its
// position (event record + wait, which become graph edges under capture) and joined back at the
// end of every run/capture range.  Weight-gradient kernels are off the backward critical path
// (nothing but the optimizer consumes them), so the lowering puts them on lane 1 where they fill
// the CUs the small, latency-bound dgrad chain leaves idle.  The lowering guarantees that a
// side-lane op only reads buffers no later main-lane op of the same range overwrites.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <limits>
#include <mutex>
#include <unordered_map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/conv_igemm.h"
#include "../kernels/conv_wgrad.h"
#include "../kernels/dense_stage.h"
#include "../kernels/mb_chain.h"
#include "../kernels/mb_infer.h"
#include "../kernels/dwconv.h"
#include "../kernels/mlp_head.h"
#include "../kernels/nn_kernels.h"
#include "../kernels/secagg.h"
#include "../comm/communicator.h"

namespace py = pybind11;
using namespace idc;

namespace {

enum OpKind : int {
  OP_CONV = 0,
  OP_WGRAD = 1,
  OP_BN_BWD_APPLY = 2,
  OP_BN_BWD_REDUCE = 3,
  OP_MAXPOOL = 4,
  OP_AVGPOOL = 5,
  OP_POOL_BWD = 6,
  OP_BN_MOVING = 7,
  OP_HEAD_FWD = 8,
  OP_HEAD_BWD = 9,
  OP_RMSPROP = 10,
  OP_CAST = 11,
  OP_INPUT = 12,
  OP_MEMSET = 13,
  OP_BN_STATS = 14,
  OP_BN_APPLY = 15,
  OP_DW_FWD = 16,
  OP_DW_BWD_DATA = 17,
  OP_DW_WGRAD = 18,
  OP_COPY = 19,
  OP_FINITE_CHECK = 20,
  OP_MLP_FWD = 21,
  OP_MLP_BWD = 22,
  OP_MLP_STEP = 23,
  OP_COLLAPSE = 24,
  OP_STATS_SHIFT = 25,
  // gradient-bucket all-reduce on the communicator's stream (the "comm lane"): p[0] buffer,
  // l[0] element count, i[0] dtype code, i[1] reduction op (csrc/comm/communicator.h)
  OP_ALLREDUCE = 26,
  // batched weight gradients (conv_wgrad.h): p[0] device WgBatchEntry[n], p[1] device begins
  // (WG_BATCH_MAX ints), i[0] n, i[1] total workgroups, i[2] batch signature, l[0] LDS bytes
  OP_WGRAD_BATCH = 27,
  // persistent dense-stage forward (dense_stage.hip): payload DenseStageArgs, i[0] = grid
  OP_DENSE_STAGE = 28,
  // persistent dense-stage backward (dense_stage_bwd.hip): payload DenseBwdArgs, i[0] = grid
  OP_DENSE_STAGE_BWD = 29,
  // persistent MobileNetV2 block chain (mb_chain.hip): payload MbChainArgs, i[0] = grid,
  // i[1] = dynamic LDS bytes
  OP_MB_CHAIN = 30,
  // one MobileNetV2 block in inference mode (mb_infer.hip): payload MbInferArgs
  OP_MB_INFER = 31,
  // a whole DenseNet dense block in inference mode (dense_infer.hip): payload DenseInferArgs
  OP_DENSE_INFER = 32,
};

struct Op {
  int kind;
  int lane = 0;
  int i[8];
  float f[8];
  long long l[4];
  uintptr_t p[8];
  std::vector<unsigned char> blob;
};

inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
const T& as(const Op& op) {
  if (op.blob.size() != sizeof(T)) throw std::runtime_error("bad op payload size");
  return *reinterpret_cast<const T*>(op.blob.data());
}

class Plan {
 public:
  ~Plan() {
    clear_graphs();
    if (fork_) hipEventDestroy(fork_);
    if (join_) hipEventDestroy(join_);
    if (mark_) hipEventDestroy(mark_);
    if (cfork_) hipEventDestroy(cfork_);
    if (cjoin_) hipEventDestroy(cjoin_);
    if (side_) hipStreamDestroy(side_);
  }

  // attach the communicator whose stream runs this plan's OP_ALLREDUCE ops (kept alive by the
  // Python binding for as long as the plan)
  void set_comm(Communicator* c) { comm_ = c; }
  bool has_comm_ops(int begin, int end) const {
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    for (int k = begin; k < end; ++k)
      if (ops_[k].kind == OP_ALLREDUCE) return true;
    return false;
  }

  int add(int kind, py::bytes payload, std::vector<int> ints, std::vector<float> floats,
          std::vector<long long> longs, std::vector<uintptr_t> ptrs, int lane) {
    Op op;
    op.kind = kind;
    op.lane = lane;
    std::memset(op.i, 0, sizeof(op.i));
    std::memset(op.f, 0, sizeof(op.f));
    std::memset(op.l, 0, sizeof(op.l));
    std::memset(op.p, 0, sizeof(op.p));
    std::string s = payload;
    op.blob.assign(s.begin(), s.end());
    for (size_t k = 0; k < ints.size() && k < 8; ++k) op.i[k] = ints[k];
    for (size_t k = 0; k < floats.size() && k < 8; ++k) op.f[k] = floats[k];
    for (size_t k = 0; k < longs.size() && k < 4; ++k) op.l[k] = longs[k];
    for (size_t k = 0; k < ptrs.size() && k < 8; ++k) op.p[k] = ptrs[k];
    ops_.push_back(std::move(op));
    return (int)ops_.size() - 1;
  }

  uintptr_t get_ptr(int idx, int slot) const { return ops_.at(idx).p[slot & 7]; }
  // per-step operands of a directly issued op (the input stage reads the caller's tensors); an op
  // inside a captured graph keeps the pointers it was captured with
  void set_ptr(int idx, int slot, uintptr_t v) { ops_.at(idx).p[slot & 7] = v; }
  long long get_long(int idx, int slot) const { return ops_.at(idx).l[slot & 3]; }
  void set_float(int idx, int slot, float v) { ops_.at(idx).f[slot] = v; }
  void set_int(int idx, int slot, int v) { ops_.at(idx).i[slot] = v; }
  int get_int(int idx, int slot) const { return ops_.at(idx).i[slot]; }
  int kind(int idx) const { return ops_.at(idx).kind; }
  py::bytes payload(int idx) const {
    const auto& b = ops_.at(idx).blob;
    return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
  }

  int size() const { return (int)ops_.size(); }

  // join=false (direct runs only): the side lane is NOT joined back at the end of the range; a
  // consumer that needs the range's side-lane work (a gradient bucket's all-reduce) waits for it
  // with wait_side() on its own stream, and the main lane keeps going.  The next joined range
  // (or capture) joins everything.
  void run(int begin, int end, uintptr_t stream, bool join) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    issue(begin, end, st, join);
  }

  // Grouped execution (csrc/kernels/common.h GroupArg): every launch of this plan runs `k` copies
  // of the program whose buffers sit `stride` bytes apart (client-batched federated training).
  void set_groups(int k, long long stride) {
    if (k < 1 || (k > 1 && stride <= 0)) throw std::runtime_error("set_groups: bad group count / stride");
    groups_ = k;
    gstride_ = k > 1 ? stride : 0;
  }
  int groups() const { return groups_; }

  // make `stream` wait for every side-lane op issued so far (event record on the side lane)
  void wait_side(uintptr_t stream) {
    if (!side_) return;
    check(hipEventRecord(mark_, side_), "hipEventRecord(mark)");
    check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), mark_, 0), "hipStreamWaitEvent(mark)");
  }

  int lane(int idx) const { return ops_.at(idx).lane; }
  // n main ops between a side batch's first member and its fork; 0: fork at once (the side op
  // starts when the main ops issued before it finish, not one main op later)
  void set_side_flush(int n) { side_flush_ = n < 0 ? 0 : n; }

  int capture(int begin, int end, uintptr_t stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    try {
      issue(begin, end, st);
    } catch (...) {
      hipGraph_t g;
      hipStreamEndCapture(st, &g);
      if (g) hipGraphDestroy(g);
      throw;
    }
    hipGraph_t g = nullptr;
    check(hipStreamEndCapture(st, &g), "hipStreamEndCapture");
    hipGraphExec_t ex = nullptr;
    check(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0), "hipGraphInstantiate");
    graphs_.push_back(g);
    execs_.push_back(ex);
    return (int)execs_.size() - 1;
  }

  void launch(int gid, uintptr_t stream) {
    check(hipGraphLaunch(execs_.at(gid), reinterpret_cast<hipStream_t>(stream)), "hipGraphLaunch");
  }

  // ---- lane-split chunk graphs (the backward) --------------------------------------------
  // A backward chunk [begin, end) becomes TWO plain graphs: its main-lane ops and its side-lane
  // ops (weight gradients), each a straight chain with no event nodes (ROCm replays those fast).
  // The caller launches the main graph on the plan stream, forks the side stream after it
  // (fork_side), launches the side graph there and keeps going with the next chunk's main graph,
  // so chunk i's weight gradients overlap chunk i+1's data gradients.  A side op's producers all
  // precede it in op order, hence sit in main chunks <= its own: ordering after the main graph of
  // its chunk is sufficient, and the lowering guarantees no later main op overwrites its inputs.
  // Returns -1 when the lane has no op in the range.
  int capture_lane(int begin, int end, int lane, uintptr_t stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    bool any = false;
    for (int k = begin; k < end; ++k)
      if (ops_[k].lane == lane && ops_[k].kind != OP_ALLREDUCE) any = true;
    if (!any) return -1;
    GroupScope gscope(groups_, gstride_);
    check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture(lane)");
    try {
      for (int k = begin; k < end; ++k)
        if (ops_[k].lane == lane && ops_[k].kind != OP_ALLREDUCE) exec(ops_[k], st);
    } catch (...) {
      hipGraph_t g = nullptr;
      hipStreamEndCapture(st, &g);
      if (g) hipGraphDestroy(g);
      throw;
    }
    hipGraph_t g = nullptr;
    check(hipStreamEndCapture(st, &g), "hipStreamEndCapture(lane)");
    hipGraphExec_t ex = nullptr;
    check(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0), "hipGraphInstantiate(lane)");
    graphs_.push_back(g);
    execs_.push_back(ex);
    return (int)execs_.size() - 1;
  }

  // the side stream waits for everything issued on `stream` so far
  void fork_side(uintptr_t stream) {
    ensure_side();
    check(hipEventRecord(fork_, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord(fork)");
    check(hipStreamWaitEvent(side_, fork_, 0), "hipStreamWaitEvent(fork)");
    side_open_ = true;
  }
  void launch_side(int gid) {
    ensure_side();
    check(hipGraphLaunch(execs_.at(gid), side_), "hipGraphLaunch(side)");
    side_open_ = true;
  }
  // `stream` waits for every side-lane op issued so far
  void join_side(uintptr_t stream) {
    if (!side_ || !side_open_) return;
    check(hipEventRecord(join_, side_), "hipEventRecord(join)");
    check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), join_, 0), "hipStreamWaitEvent(join)");
    side_open_ = false;
  }
  // the collectives of [begin, end) on the comm stream, after everything issued so far on the
  // side stream (whose last graph followed the main graph of the same chunk) and on `stream`
  void comm_range(int begin, int end, uintptr_t stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    bool first = true;
    for (int k = begin; k < end; ++k) {
      if (ops_[k].kind != OP_ALLREDUCE) continue;
      if (first) {
        issue_comm(ops_[k], st, side_ != nullptr && side_open_);
        first = false;
      } else {
        comm_->all_reduce(reinterpret_cast<void*>(ops_[k].p[0]), ops_[k].l[0], ops_[k].i[0], ops_[k].i[1],
                          comm_->stream());
      }
      comm_open_ = true;
    }
  }
  void join_comm(uintptr_t stream) {
    if (!comm_ || !comm_open_) return;
    check(hipEventRecord(cjoin_, comm_->stream()), "hipEventRecord(comm join)");
    check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), cjoin_, 0), "hipStreamWaitEvent(comm join)");
    comm_open_ = false;
  }
  int count_lane(int begin, int end, int lane) const {
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    int n = 0;
    for (int k = begin; k < end; ++k) n += (ops_[k].lane == lane && ops_[k].kind != OP_ALLREDUCE);
    return n;
  }

  // Two-lane graphs.  A single captured graph with fork/join edges is executed by ROCm without
  // the side lane's concurrency (measured slower than direct issue on the DenseNet backward), and
  // direct issue of ~250 launches leaves the small-kernel backward host-bound (issue gaps).  So a
  // range with side-lane ops becomes TWO graphs: the main lane's ops, with an external event
  // record node at every fork point, and the side lane's batches, each behind an external event
  // wait node on its fork event.  launch_dual() launches the main graph first and then the side
  // graph on the side stream, from this thread: HIP enqueues a graph's nodes during
  // hipGraphLaunch, so every wait node refers to the record of the same launch.
  int capture_dual(int begin, int end, uintptr_t stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    ensure_side();
    if (has_comm_ops(begin, end)) throw std::runtime_error("capture_dual: range holds collectives; use capture()");
    GroupScope gscope(groups_, gstride_);
    Dual d;
    std::vector<std::vector<int>> batches;
    auto abort_capture = [](hipStream_t s) {
      hipGraph_t g = nullptr;
      hipStreamEndCapture(s, &g);
      if (g) hipGraphDestroy(g);
    };
    check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture(main)");
    try {
      std::vector<int> pending;
      int main_since = 0;
      auto flush = [&]() {
        if (pending.empty()) return;
        hipEvent_t e = nullptr;
        check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate(dual)");
        d.evs.push_back(e);
        add_event_node(st, e, /*record=*/true);
        batches.push_back(pending);
        pending.clear();
      };
      for (int k = begin; k < end; ++k) {
        const Op& op = ops_[k];
        if (op.lane == 1) {
          if (pending.empty()) main_since = 0;
          pending.push_back(k);
          if (side_flush_ == 0) flush();
        } else {
          exec(op, st);
          if (!pending.empty() && ++main_since >= side_flush_) flush();
        }
      }
      flush();
    } catch (...) {
      abort_capture(st);
      for (auto e : d.evs) hipEventDestroy(e);
      throw;
    }
    check(hipStreamEndCapture(st, &d.gm), "hipStreamEndCapture(main)");
    check(hipGraphInstantiate(&d.main, d.gm, nullptr, nullptr, 0), "hipGraphInstantiate(main)");
    if (!batches.empty()) {
      check(hipStreamBeginCapture(side_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture(side)");
      try {
        for (size_t b = 0; b < batches.size(); ++b) {
          add_event_node(side_, d.evs[b], /*record=*/false);
          for (int k : batches[b]) exec(ops_[k], side_);
        }
      } catch (...) {
        abort_capture(side_);
        throw;
      }
      check(hipStreamEndCapture(side_, &d.gs), "hipStreamEndCapture(side)");
      check(hipGraphInstantiate(&d.side, d.gs, nullptr, nullptr, 0), "hipGraphInstantiate(side)");
    }
    duals_.push_back(std::move(d));
    return (int)duals_.size() - 1;
  }

  // join=false: the side graph keeps running past the range (see run()); wait_side() orders a
  // consumer after it and the next joined range joins it
  void launch_dual(int id, uintptr_t stream, bool join) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const Dual& d = duals_.at(id);
    check(hipGraphLaunch(d.main, st), "hipGraphLaunch(main)");
    if (d.side) check(hipGraphLaunch(d.side, side_), "hipGraphLaunch(side)");
    if ((d.side || side_open_) && join) {
      check(hipEventRecord(join_, side_), "hipEventRecord(join)");
      check(hipStreamWaitEvent(st, join_, 0), "hipStreamWaitEvent(join)");
      side_open_ = false;
    } else if (d.side) {
      side_open_ = true;
    }
  }

  // Add an event record (leaf) or wait node to the graph `st` is capturing, after the nodes
  // captured so far (hipEventRecordWithFlags(External) is rejected under capture on this ROCm).
  // A wait node becomes the dependency of everything captured after it.
  static void add_event_node(hipStream_t st, hipEvent_t e, bool record) {
    hipStreamCaptureStatus status;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    check(hipStreamGetCaptureInfo_v2(st, &status, &id, &g, &deps, &ndeps), "hipStreamGetCaptureInfo_v2");
    if (status != hipStreamCaptureStatusActive || g == nullptr) throw std::runtime_error("add_event_node: not capturing");
    std::vector<hipGraphNode_t> dv(deps, deps + ndeps);
    hipGraphNode_t n = nullptr;
    if (record) {
      check(hipGraphAddEventRecordNode(&n, g, dv.data(), dv.size(), e), "hipGraphAddEventRecordNode");
    } else {
      check(hipGraphAddEventWaitNode(&n, g, dv.data(), dv.size(), e), "hipGraphAddEventWaitNode");
      check(hipStreamUpdateCaptureDependencies(st, &n, 1, hipStreamSetCaptureDependencies),
            "hipStreamUpdateCaptureDependencies");
    }
  }

  bool has_side(int begin, int end) const {
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    for (int k = begin; k < end; ++k)
      if (ops_[k].lane == 1) return true;
    return false;
  }

  void clear_graphs() {
    for (auto e : execs_) hipGraphExecDestroy(e);
    for (auto g : graphs_) hipGraphDestroy(g);
    execs_.clear();
    graphs_.clear();
    for (auto& d : duals_) {
      if (d.main) hipGraphExecDestroy(d.main);
      if (d.side) hipGraphExecDestroy(d.side);
      if (d.gm) hipGraphDestroy(d.gm);
      if (d.gs) hipGraphDestroy(d.gs);
      for (auto e : d.evs) hipEventDestroy(e);
    }
    duals_.clear();
  }

  std::string describe(int idx) const {
    static const char* names[] = {"conv", "wgrad", "bn_bwd_apply", "bn_bwd_reduce", "maxpool", "avgpool",
                                  "pool_bwd", "bn_moving", "head_fwd", "head_bwd", "rmsprop", "cast",
                                  "input", "memset", "bn_stats", "bn_apply", "dw_fwd", "dw_bwd_data",
                                  "dw_wgrad", "copy", "finite_check", "mlp_fwd", "mlp_bwd", "mlp_step",
                                  "collapse", "stats_shift", "allreduce", "wgrad_batch", "dense_stage",
                                  "dense_stage_bwd", "mb_chain", "mb_infer", "dense_infer"};
    int k = ops_.at(idx).kind;
    return (k >= 0 && k < (int)(sizeof(names) / sizeof(names[0]))) ? names[k] : "?";
  }

 private:
  void ensure_side() {
    if (side_) return;
    // IDC_SIDE_PRIO=low gives the side lane (weight gradients, off the critical path) the lowest
    // stream priority, so the dgrad chain's workgroups dispatch first when both lanes have work
    // queued.  Opt-in: measured neutral on DenseNet-121 (runtime/program.py).
    int least = 0, greatest = 0;
    check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
    const char* sp = std::getenv("IDC_SIDE_PRIO");
    const int prio = (sp && std::strcmp(sp, "low") == 0) ? least : 0;
    // IDC_SIDE_CUS=N: the side lane runs on N of the device's CUs only (a CU-masked queue, bits
    // spread evenly over the CU index space), so weight-gradient workgroups never occupy the
    // CUs the data-gradient chain needs next (measured: runtime/program.py)
    const char* scu = std::getenv("IDC_SIDE_CUS");
    const int ncu_side = scu ? std::atoi(scu) : 0;
    int dev = 0, ncu = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
    if (ncu_side > 0 && ncu_side < ncu) {
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu_side; ++i) {
        const int cu = (int)((long long)i * ncu / ncu_side);
        mask[cu / 32] |= 1u << (cu % 32);
      }
      check(hipExtStreamCreateWithCUMask(&side_, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask(side)");
    } else {
      check(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, prio), "hipStreamCreate(side)");
    }
    check(hipEventCreateWithFlags(&fork_, hipEventDisableTiming), "hipEventCreate(fork)");
    check(hipEventCreateWithFlags(&join_, hipEventDisableTiming), "hipEventCreate(join)");
    check(hipEventCreateWithFlags(&mark_, hipEventDisableTiming), "hipEventCreate(mark)");
  }

  // issue ops[begin:end): lane-0 ops on `st`; lane-1 ops are queued and issued on the side
  // stream in batches — one fork (event record + wait) per batch, placed after the main op that
  // completes `side_flush_` main ops past the batch's first member (every queued op's producers
  // precede the fork, and the lowering guarantees no later main op overwrites a side op's
  // inputs, so deferring is safe) — and one join at the end.  Batching keeps the host API calls
  // per step low: with direct (non-graph) issue the backward is otherwise host-bound.
  // sets the launch-group context of the calling thread for the lifetime of one issue()
  struct GroupScope {
    LaunchGroups saved;
    GroupScope(int k, long long stride) : saved(launch_groups()) {
      launch_groups().k = k;
      launch_groups().stride = stride;
    }
    ~GroupScope() { launch_groups() = saved; }
  };

  void issue(int begin, int end, hipStream_t st, bool join = true) {
    GroupScope gscope(groups_, gstride_);
    bool side_used = false;
    std::vector<int> pending;
    int main_since = 0;
    auto flush = [&]() {
      if (pending.empty()) return;
      ensure_side();
      check(hipEventRecord(fork_, st), "hipEventRecord(fork)");
      check(hipStreamWaitEvent(side_, fork_, 0), "hipStreamWaitEvent(fork)");
      for (int k : pending) exec(ops_[k], side_);
      pending.clear();
      side_used = true;
    };
    bool comm_used = false;
    for (int k = begin; k < end; ++k) {
      const Op& op = ops_[k];
      if (op.kind == OP_ALLREDUCE) {
        // a bucket's gradients are final once every main-lane op so far AND every side-lane op
        // so far (weight gradients) has run: fork any pending side batch, then the comm stream
        // waits on both lanes and enqueues the collective; the main lane runs on
        flush();
        issue_comm(op, st, side_used || side_open_);
        comm_used = true;
        continue;
      }
      if (op.lane == 1) {
        if (pending.empty()) main_since = 0;
        pending.push_back(k);
        if (side_flush_ == 0) flush();
      } else {
        exec(op, st);
        if (!pending.empty() && ++main_since >= side_flush_) flush();
      }
    }
    flush();
    if ((side_used || side_open_) && join) {
      check(hipEventRecord(join_, side_), "hipEventRecord(join)");
      check(hipStreamWaitEvent(st, join_, 0), "hipStreamWaitEvent(join)");
      side_open_ = false;
    } else if (side_used) {
      side_open_ = true;
    }
    if ((comm_used || comm_open_) && join) {
      check(hipEventRecord(cjoin_, comm_->stream()), "hipEventRecord(comm join)");
      check(hipStreamWaitEvent(st, cjoin_, 0), "hipStreamWaitEvent(comm join)");
      comm_open_ = false;
    } else if (comm_used) {
      comm_open_ = true;
    }
  }

  void issue_comm(const Op& op, hipStream_t st, bool side_active) {
    if (!comm_) throw std::runtime_error("plan: OP_ALLREDUCE without a communicator (set_comm)");
    if (groups_ > 1) throw std::runtime_error("plan: collectives inside a grouped plan");
    if (!cfork_) {
      check(hipEventCreateWithFlags(&cfork_, hipEventDisableTiming), "hipEventCreate(comm fork)");
      check(hipEventCreateWithFlags(&cjoin_, hipEventDisableTiming), "hipEventCreate(comm join)");
    }
    hipStream_t cs = comm_->stream();
    check(hipEventRecord(cfork_, st), "hipEventRecord(comm fork)");
    check(hipStreamWaitEvent(cs, cfork_, 0), "hipStreamWaitEvent(comm fork)");
    if (side_active) {
      check(hipEventRecord(mark_, side_), "hipEventRecord(side mark)");
      check(hipStreamWaitEvent(cs, mark_, 0), "hipStreamWaitEvent(side mark)");
    }
    comm_->all_reduce(reinterpret_cast<void*>(op.p[0]), op.l[0], op.i[0], op.i[1], cs);
  }

  // IDC_SYNC_OPS=1 (fault attribution only): every directly issued op is followed by a stream
  // synchronisation, so an asynchronous fault is reported by the op that caused it instead of by
  // whatever API call happens to run next (torch, MIOpen)
  static bool sync_ops() {
    static const bool on = [] {
      const char* e = std::getenv("IDC_SYNC_OPS");
      return e && e[0] == '1';
    }();
    return on;
  }
  void exec(const Op& op, hipStream_t st) {
    exec_op(op, st);
    if (sync_ops()) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(st, &cs);
      if (cs == hipStreamCaptureStatusNone) {
        const hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
          const long idx = (long)(&op - ops_.data());
          throw std::runtime_error("IDC_SYNC_OPS: op " + std::to_string(idx) + " (" + describe((int)idx) +
                                   ") faulted: " + hipGetErrorString(e));
        }
      }
    }
  }
  void exec_op(const Op& op, hipStream_t st) {
    switch (op.kind) {
      case OP_CONV: {
        ConvArgs a = as<ConvArgs>(op);
        a.ksplit = op.i[2] > 1 ? op.i[2] : 1;  // split factor lives in the op (autotuned)
        check(conv_igemm(a, op.i[0], op.i[1] != 0, st), "conv_igemm");
        break;
      }
      case OP_WGRAD: {
        const WgradArgs& a = as<WgradArgs>(op);
        check(conv_wgrad(a, op.i[0], op.i[1] != 0, st, op.i[2]), "conv_wgrad");
        if (a.part) {  // deterministic mode: fixed-order sum of the per-slice partials
          const long long n = (long long)a.KH * a.KW * (a.cin_real ? a.cin_real : a.Cin) * a.Cout;
          check(wgrad_reduce(a.part, a.dw, n, wgrad_effective_splits(a, op.i[0], op.i[2]), st), "wgrad_reduce");
        }
        break;
      }
      case OP_BN_BWD_APPLY: check(bn_bwd_apply(as<BnBwdApplyArgs>(op), st), "bn_bwd_apply"); break;
      case OP_BN_BWD_REDUCE: check(bn_bwd_reduce(as<BnBwdReduceArgs>(op), st), "bn_bwd_reduce"); break;
      case OP_MAXPOOL: check(maxpool_fwd(as<PoolArgs>(op), st), "maxpool_fwd"); break;
      case OP_AVGPOOL: check(avgpool_fwd(as<PoolArgs>(op), st), "avgpool_fwd"); break;
      case OP_POOL_BWD: check(pool_bwd(as<PoolBwdArgs>(op), st), "pool_bwd"); break;
      case OP_BN_MOVING:
        check(bn_update_moving(reinterpret_cast<const BnMovingDesc*>(op.p[0]), op.i[0], op.i[1], st),
              "bn_update_moving");
        break;
      case OP_HEAD_FWD: check(head_fwd(as<HeadArgs>(op), st), "head_fwd"); break;
      case OP_HEAD_BWD: check(head_bwd(as<HeadBwdArgs>(op), st), "head_bwd"); break;
      case OP_RMSPROP:
        check(rmsprop(reinterpret_cast<float*>(op.p[0]), reinterpret_cast<const float*>(op.p[1]),
                      reinterpret_cast<float*>(op.p[2]), op.l[0], op.f[0], op.f[1], op.f[2], op.f[3],
                      reinterpret_cast<const int*>(op.p[3]), reinterpret_cast<int*>(op.p[4]), st),
              "rmsprop");
        break;
      case OP_CAST:
        check(cast_weights(reinterpret_cast<const CastEntry*>(op.p[0]), reinterpret_cast<const int*>(op.p[1]),
                           op.l[0], st),
              "cast_weights");
        break;
      case OP_INPUT:
        check(input_stage(reinterpret_cast<const void*>(op.p[0]), op.i[0], op.i[1], op.i[2], op.i[3], op.i[4],
                          reinterpret_cast<bf16_t*>(op.p[1]), op.i[5], reinterpret_cast<const void*>(op.p[2]),
                          op.i[6], op.i[7], reinterpret_cast<float*>(op.p[3]), st),
              "input_stage");
        break;
      case OP_MEMSET:
        check(zero_fill(reinterpret_cast<void*>(op.p[0]), op.l[0], st), "zero_fill");
        break;
      case OP_BN_STATS:
        check(bn_stats(reinterpret_cast<const bf16_t*>(op.p[0]), op.i[0], op.i[1], op.i[2],
                       reinterpret_cast<float*>(op.p[1]), op.i[3], op.i[4], op.i[5], st),
              "bn_stats");
        break;
      case OP_BN_APPLY: {
        const BnArgs& bn = as<BnArgs>(op);
        check(bn_apply(reinterpret_cast<const bf16_t*>(op.p[0]), op.i[0], bn,
                       reinterpret_cast<const bf16_t*>(op.p[1]), op.i[1], reinterpret_cast<bf16_t*>(op.p[2]),
                       op.i[2], op.i[3], op.i[4], reinterpret_cast<float*>(op.p[3]), op.i[5], op.i[6], st),
              "bn_apply");
        break;
      }
      case OP_DW_FWD: check(dwconv_fwd(as<DwArgs>(op), st), "dwconv_fwd"); break;
      // i[0] 1: data + weight-gradient partials in one pass (dwconv_bwd_fused)
      case OP_DW_BWD_DATA:
        check(op.i[0] == 1 ? dwconv_bwd_fused(as<DwArgs>(op), st) : dwconv_bwd_data(as<DwArgs>(op), st),
              "dwconv_bwd_data");
        break;
      // i[0] 2: only the column sums of a fused backward's partials (dwconv_wgrad_sum)
      case OP_DW_WGRAD:
        check(op.i[0] == 2 ? dwconv_wgrad_sum(as<DwArgs>(op), st) : dwconv_wgrad(as<DwArgs>(op), st), "dwconv_wgrad");
        break;
      case OP_FINITE_CHECK:
        if (op.i[0] == 0)
          check(finite_check(reinterpret_cast<const float*>(op.p[0]), op.l[0], reinterpret_cast<int*>(op.p[1]), st),
                "finite_check");
        else
          check(finite_flag_reset(reinterpret_cast<int*>(op.p[1]), reinterpret_cast<int*>(op.p[2]), st),
                "finite_flag_reset");
        break;
      case OP_MLP_FWD: check(mlp2_fwd(as<Mlp2Args>(op), st), "mlp2_fwd"); break;
      case OP_MLP_BWD: check(mlp2_bwd(as<Mlp2Args>(op), st), "mlp2_bwd"); break;
      case OP_MLP_STEP: check(mlp2_step(reinterpret_cast<unsigned int*>(op.p[0]), st), "mlp2_step"); break;
      case OP_COLLAPSE:
        check(slot_collapse(reinterpret_cast<const float*>(op.p[0]), reinterpret_cast<float*>(op.p[1]),
                            reinterpret_cast<const float*>(op.p[2]), reinterpret_cast<float*>(op.p[3]), op.i[0],
                            op.i[1], op.i[2], st),
              "slot_collapse");
        break;
      case OP_WGRAD_BATCH:
        check(wgrad_batch(reinterpret_cast<const WgBatchEntry*>(op.p[0]), reinterpret_cast<const int*>(op.p[1]),
                          op.i[0], op.i[1], op.i[2], op.l[0], st),
              "wgrad_batch");
        break;
      case OP_DENSE_STAGE: check(dense_stage_fwd(as<DenseStageArgs>(op), op.i[0], st), "dense_stage_fwd"); break;
      case OP_DENSE_STAGE_BWD: check(dense_stage_bwd(as<DenseBwdArgs>(op), op.i[0], st), "dense_stage_bwd"); break;
      case OP_MB_CHAIN: check(mb_chain(as<MbChainArgs>(op), op.i[0], op.i[1], st), "mb_chain"); break;
      case OP_MB_INFER: check(mb_infer(as<MbInferArgs>(op), st), "mb_infer"); break;
      case OP_DENSE_INFER: check(dense_infer(as<DenseInferArgs>(op), st), "dense_infer"); break;
      case OP_STATS_SHIFT:
        check(stats_shift(reinterpret_cast<const ShiftDesc*>(op.p[0]), op.i[0], op.i[1], st), "stats_shift");
        break;
      case OP_COPY:
        for (int g = 0; g < groups_; ++g)  // a copy engine transfer per program copy
          check(hipMemcpyAsync(reinterpret_cast<void*>(op.p[0] + g * gstride_),
                               reinterpret_cast<const void*>(op.p[1] + g * gstride_), (size_t)op.l[0],
                               hipMemcpyDeviceToDevice, st),
                "copy");
        break;
      case OP_ALLREDUCE: throw std::runtime_error("OP_ALLREDUCE outside issue()");
      default: throw std::runtime_error("unknown op kind");
    }
  }

  std::vector<Op> ops_;
  hipStream_t side_ = nullptr;
  int side_flush_ = 1;
  hipEvent_t fork_ = nullptr, join_ = nullptr, mark_ = nullptr;
  bool side_open_ = false;  // side-lane work issued by a join=false run, not yet joined
  Communicator* comm_ = nullptr;
  int groups_ = 1;
  long long gstride_ = 0;
  hipEvent_t cfork_ = nullptr, cjoin_ = nullptr;
  bool comm_open_ = false;  // collectives issued by a join=false run, not yet joined
  std::vector<hipGraph_t> graphs_;
  std::vector<hipGraphExec_t> execs_;
  struct Dual {
    hipGraph_t gm = nullptr, gs = nullptr;
    hipGraphExec_t main = nullptr, side = nullptr;
    std::vector<hipEvent_t> evs;  // one external fork event per side batch
  };
  std::vector<Dual> duals_;
};

// ---- grouped-program region allocator -------------------------------------------------------
// A grouped program (csrc/kernels/common.h GroupArg) must have ALL its buffers inside copy 0 of
// its region so that copy g is copy 0 + g * stride.  The runtime (runtime/grouped.py) routes every
// torch allocation made while it builds the model and its program into a torch.cuda.MemPool
// whose pluggable allocator is this bump allocator over the active region.  Frees are no-ops: a
// region is released as a whole with its slab.
struct RegionState {
  uintptr_t base = 0;
  size_t cap = 0, used = 0;
};
std::mutex g_region_mu;
std::unordered_map<uintptr_t, RegionState> g_regions;
thread_local uintptr_t g_region_active = 0;  // per thread, as allocating() routes per thread

void region_activate(uintptr_t base, long long cap) {
  std::lock_guard<std::mutex> l(g_region_mu);
  RegionState& r = g_regions[base];
  r.base = base;
  r.cap = (size_t)cap;
  g_region_active = base;
}
long long region_used(uintptr_t base) {
  std::lock_guard<std::mutex> l(g_region_mu);
  auto it = g_regions.find(base);
  return it == g_regions.end() ? 0 : (long long)it->second.used;
}
void region_forget(uintptr_t base) {
  std::lock_guard<std::mutex> l(g_region_mu);
  g_regions.erase(base);
  if (g_region_active == base) g_region_active = 0;
}

// direct (non-plan) entry points, used by the op-level python API and tests
void py_conv(py::bytes payload, int tile, int a_f32, uintptr_t stream) {
  std::string s = payload;
  if (s.size() != sizeof(ConvArgs)) throw std::runtime_error("ConvArgs size mismatch");
  ConvArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  if (tile < 0) tile = conv_pick_tile(a.N * a.Ho * a.Wo, a.Cout);
  check(conv_igemm(a, tile, a_f32 != 0, reinterpret_cast<hipStream_t>(stream)), "conv_igemm");
}

void py_wgrad(py::bytes payload, int splits, int g_f32, uintptr_t stream, int variant) {
  std::string s = payload;
  if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
  WgradArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  if (splits <= 0) splits = wgrad_pick_splits(a.N * a.Ho * a.Wo, a.KH * a.KW * a.Cin, a.Cout);
  if (splits <= 0 && variant > 0) splits = wgrad_big_pick_splits(a.N * a.Ho * a.Wo, a.KH * a.KW * a.Cin, a.Cout, variant);
  check(conv_wgrad(a, splits, g_f32 != 0, reinterpret_cast<hipStream_t>(stream), variant), "conv_wgrad");
}

bool py_wgrad_big_ok(py::bytes payload, int g_f32, int variant) {
  std::string s = payload;
  if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
  WgradArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  return wgrad_big_ok(a, g_f32 != 0, variant);
}

py::dict struct_sizes() {
  py::dict d;
  d["BnArgs"] = sizeof(BnArgs);
  d["ConvArgs"] = sizeof(ConvArgs);
  d["WgradArgs"] = sizeof(WgradArgs);
  d["WgBatchEntry"] = sizeof(WgBatchEntry);
  d["BnBwdApplyArgs"] = sizeof(BnBwdApplyArgs);
  d["BnBwdReduceArgs"] = sizeof(BnBwdReduceArgs);
  d["PoolArgs"] = sizeof(PoolArgs);
  d["PoolBwdArgs"] = sizeof(PoolBwdArgs);
  d["BnMovingDesc"] = sizeof(BnMovingDesc);
  d["ShiftDesc"] = sizeof(ShiftDesc);
  d["DenseStageArgs"] = sizeof(DenseStageArgs);
  d["DenseLayerDesc"] = sizeof(DenseLayerDesc);
  d["DenseBwdArgs"] = sizeof(DenseBwdArgs);
  d["DenseBwdLayerDesc"] = sizeof(DenseBwdLayerDesc);
  d["DenseBwdPhase"] = sizeof(DenseBwdPhase);
  d["MbPhaseDesc"] = sizeof(MbPhaseDesc);
  d["MbInferArgs"] = sizeof(MbInferArgs);
  d["DenseInferArgs"] = sizeof(DenseInferArgs);
  d["MbChainArgs"] = sizeof(MbChainArgs);
  d["MbPhaseDesc.pre"] = offsetof(MbPhaseDesc, pre);
  d["BnArgs.shift"] = offsetof(BnArgs, shift);
  d["ConvArgs.stats_shift"] = offsetof(ConvArgs, stats_shift);
  d["PoolArgs.stats_shift"] = offsetof(PoolArgs, stats_shift);
  d["DwArgs.stats_shift"] = offsetof(DwArgs, stats_shift);
  d["BnMovingDesc.shift"] = offsetof(BnMovingDesc, shift);
  d["HeadArgs"] = sizeof(HeadArgs);
  d["HeadBwdArgs"] = sizeof(HeadBwdArgs);
  d["CastEntry"] = sizeof(CastEntry);
  d["DwArgs"] = sizeof(DwArgs);
  d["Mlp2Args"] = sizeof(Mlp2Args);
  d["ConvArgs.mbn"] = offsetof(ConvArgs, mbn);
  d["ConvArgs.gsumx"] = offsetof(ConvArgs, gsumx);
  d["ConvArgs.ksplit"] = offsetof(ConvArgs, ksplit);
  d["WgradArgs.pix_per_split"] = offsetof(WgradArgs, pix_per_split);
  d["HeadArgs.training"] = offsetof(HeadArgs, training);
  d["PoolBwdArgs.is_avg"] = offsetof(PoolBwdArgs, is_avg);
  d["ConvArgs.gsum_ld"] = offsetof(ConvArgs, gsum_ld);
  d["BnArgs.slots"] = offsetof(BnArgs, slots);
  d["DwArgs.gsum_ld"] = offsetof(DwArgs, gsum_ld);
  d["BwdAff"] = sizeof(BwdAff);
  d["ConvArgs.bepi"] = offsetof(ConvArgs, bepi);
  d["WgradArgs.gpro"] = offsetof(WgradArgs, gpro);
  d["PoolBwdArgs.dx_f32"] = offsetof(PoolBwdArgs, dx_f32);
  d["BwdAff.fold_sumx"] = offsetof(BwdAff, fold_sumx);
  d["ConvArgs.aout"] = offsetof(ConvArgs, aout);
  d["WgradArgs.part_floats"] = offsetof(WgradArgs, part_floats);
  d["HeadBwdArgs.det"] = offsetof(HeadBwdArgs, det);
  d["DwArgs.dyaff"] = offsetof(DwArgs, dyaff);
  return d;
}

int py_pick_tile(int M, int Cout) { return conv_pick_tile(M, Cout); }

bool py_big_ok(py::bytes payload, int a_f32) {
  std::string s = payload;
  if (s.size() != sizeof(ConvArgs)) throw std::runtime_error("ConvArgs size mismatch");
  ConvArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  return conv_big_ok(a, a_f32 != 0);
}
int py_pick_splits(int M, int K, int Cout) { return wgrad_pick_splits(M, K, Cout); }

int py_effective_splits(py::bytes payload, int splits) {
  std::string s = payload;
  if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
  WgradArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  return wgrad_effective_splits(a, splits);
}

int py_wgrad_batch_sig(py::bytes payload, int g_f32, int variant) {
  std::string s = payload;
  if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
  WgradArgs a;
  std::memcpy(&a, s.data(), sizeof(a));
  return wgrad_batch_sig(a, g_f32 != 0, variant);
}

// members' WgradArgs payloads + split factors -> (WgBatchEntry table bytes, begins padded to
// WG_BATCH_MAX, total workgroups, LDS bytes)
py::tuple py_wgrad_batch_pack(py::list payloads, py::list splits) {
  const int n = (int)py::len(payloads);
  if (n < 1 || n > WG_BATCH_MAX || (int)py::len(splits) != n) throw std::runtime_error("wgrad_batch_pack: bad member count");
  std::vector<WgBatchEntry> ents(n);
  std::vector<int> begins(WG_BATCH_MAX, std::numeric_limits<int>::max());
  long long total = 0, smem = 0;
  int sig = -2;
  for (int i = 0; i < n; ++i) {
    std::string s = payloads[i].cast<py::bytes>();
    if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
    WgradArgs a;
    std::memcpy(&a, s.data(), sizeof(a));
    const int si = wgrad_batch_sig(a, false, 0);
    if (si < 0 || (sig != -2 && si != sig)) throw std::runtime_error("wgrad_batch_pack: members differ in kernel shape");
    sig = si;
    long long sm = 0;
    begins[i] = (int)total;
    total += wgrad_batch_entry(a, splits[i].cast<int>(), ents[i], sm);
    smem = std::max(smem, sm);
  }
  if (total > (1LL << 30)) throw std::runtime_error("wgrad_batch_pack: grid too large");
  py::bytes tab(reinterpret_cast<const char*>(ents.data()), ents.size() * sizeof(WgBatchEntry));
  py::list bl;
  for (int b : begins) bl.append(b);
  return py::make_tuple(tab, bl, total, smem, sig);
}

void py_secagg_mask(uintptr_t x, uintptr_t out, long long n, uintptr_t seg_scale, uintptr_t seg_end, int nseg,
                    float clip, int nclients, int rank, uintptr_t keys, unsigned long long round_,
                    unsigned long long alive, uintptr_t stream, int accumulate) {
  check(secagg_quantize_mask(reinterpret_cast<const float*>(x), reinterpret_cast<uint32_t*>(out), n,
                             reinterpret_cast<const float*>(seg_scale), reinterpret_cast<const long long*>(seg_end),
                             nseg, clip, nclients, rank, reinterpret_cast<const uint32_t*>(keys), round_, alive,
                             reinterpret_cast<hipStream_t>(stream), accumulate),
        "secagg_quantize_mask");
}

void py_group_metrics(uintptr_t loss, uintptr_t logits, uintptr_t labels, long long stride, int K, int B, float thr,
                      uintptr_t acc, uintptr_t stream) {
  check(group_metrics(reinterpret_cast<const float*>(loss), reinterpret_cast<const float*>(logits),
                      reinterpret_cast<const float*>(labels), stride, K, B, thr, reinterpret_cast<double*>(acc),
                      reinterpret_cast<hipStream_t>(stream)),
        "group_metrics");
}

void py_secagg_absmax(uintptr_t x, long long n, uintptr_t seg_end, int nseg, uintptr_t out, uintptr_t stream) {
  check(secagg_absmax(reinterpret_cast<const float*>(x), n, reinterpret_cast<const long long*>(seg_end), nseg,
                      reinterpret_cast<unsigned*>(out), reinterpret_cast<hipStream_t>(stream)),
        "secagg_absmax");
}

void py_secagg_unmask(uintptr_t sum, uintptr_t out, long long n, uintptr_t seg_scale, uintptr_t seg_end, int nseg,
                      float divisor, uintptr_t stream) {
  check(secagg_dequantize(reinterpret_cast<const uint32_t*>(sum), reinterpret_cast<float*>(out), n,
                          reinterpret_cast<const float*>(seg_scale), reinterpret_cast<const long long*>(seg_end),
                          nseg, divisor, reinterpret_cast<hipStream_t>(stream)),
        "secagg_dequantize");
}

void py_rmsprop(uintptr_t w, uintptr_t g, uintptr_t ms, long long n, float lr, float rho, float eps, float gs,
                uintptr_t stream) {
  check(rmsprop(reinterpret_cast<float*>(w), reinterpret_cast<const float*>(g), reinterpret_cast<float*>(ms), n,
                lr, rho, eps, gs, nullptr, nullptr, reinterpret_cast<hipStream_t>(stream)),
        "rmsprop");
}

// Pinned host words the device writes and the host polls without a synchronisation (the
// persistent launches' give-up flag, DenseStageArgs::hostflag).  hipHostMalloc memory is mapped
// into the device address space under the same pointer.
uintptr_t py_host_alloc(long long bytes) {
  void* p = nullptr;
  check(hipHostMalloc(&p, (size_t)bytes, hipHostMallocMapped), "hipHostMalloc");
  std::memset(p, 0, (size_t)bytes);
  return reinterpret_cast<uintptr_t>(p);
}
void py_host_free(uintptr_t p) {
  if (p) (void)hipHostFree(reinterpret_cast<void*>(p));
}

}  // namespace

// torch.cuda.memory.CUDAPluggableAllocator entry points (looked up by name with dlsym)
extern "C" __attribute__((visibility("default"))) void* idc_region_malloc(size_t size, int device,
                                                                         hipStream_t stream) {
  (void)device;
  (void)stream;
  std::lock_guard<std::mutex> l(g_region_mu);
  auto it = g_regions.find(g_region_active);
  if (it == g_regions.end()) return nullptr;
  RegionState& r = it->second;
  const size_t sz = (size + 511) & ~(size_t)511;
  if (r.used + sz > r.cap) return nullptr;  // torch reports an out-of-memory error
  void* p = reinterpret_cast<void*>(r.base + r.used);
  r.used += sz;
  return p;
}
extern "C" __attribute__((visibility("default"))) void idc_region_free(void* ptr, size_t size, int device,
                                                                      hipStream_t stream) {
  (void)ptr;
  (void)size;
  (void)device;
  (void)stream;
}

PYBIND11_MODULE(_idc_native, m) {
  m.doc() = "idc_models_amd native MI355X (gfx950) kernels and plan executor";
  py::class_<Communicator>(m, "Communicator")
      .def(py::init([](int rank, int world, py::bytes uid, int device, double init_timeout_s) {
             std::string u = uid;
             py::gil_scoped_release nogil;  // a non-blocking init polls for its peers
             return new Communicator(rank, world, u, device, init_timeout_s);
           }),
           py::arg("rank"), py::arg("world"), py::arg("unique_id"), py::arg("device"),
           py::arg("init_timeout_s") = 0.0)
      .def("mark", &Communicator::mark)
      .def("mark_age", &Communicator::mark_age)
      .def_static("make_unique_id", []() { return py::bytes(Communicator::make_unique_id()); })
      .def("all_reduce", [](Communicator& c, uintptr_t buf, long long n, int dt, int op, uintptr_t st) {
             c.all_reduce(reinterpret_cast<void*>(buf), n, dt, op, reinterpret_cast<hipStream_t>(st));
           }, py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("stream") = 0)
      .def("reduce", [](Communicator& c, uintptr_t buf, long long n, int dt, int op, int root, uintptr_t st) {
             c.reduce(reinterpret_cast<void*>(buf), n, dt, op, root, reinterpret_cast<hipStream_t>(st));
           }, py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("root"),
           py::arg("stream") = 0)
      .def("broadcast", [](Communicator& c, uintptr_t buf, long long n, int dt, int root, uintptr_t st) {
             c.broadcast(reinterpret_cast<void*>(buf), n, dt, root, reinterpret_cast<hipStream_t>(st));
           }, py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("root"), py::arg("stream") = 0)
      .def("all_gather", [](Communicator& c, uintptr_t send, uintptr_t recv, long long n, int dt, uintptr_t st) {
             c.all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt,
                          reinterpret_cast<hipStream_t>(st));
           }, py::arg("send"), py::arg("recv"), py::arg("count_per_rank"), py::arg("dtype"), py::arg("stream") = 0)
      .def("group_start", &Communicator::group_start)
      .def("group_end", &Communicator::group_end)
      .def("check_async", &Communicator::check_async)
      .def("abort", &Communicator::abort)
      .def("close", &Communicator::close)
      .def_property_readonly("stream", [](const Communicator& c) { return reinterpret_cast<uintptr_t>(c.stream()); })
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def_property_readonly("device", &Communicator::device)
      .def_property_readonly("is_open", &Communicator::open)
      .def_property_readonly("collectives", &Communicator::collectives);
  m.def("rccl_version", &rccl_version);
  m.def("region_activate", &region_activate);
  m.def("region_used", &region_used);
  m.def("region_forget", &region_forget);
  m.attr("OP_ALLREDUCE") = (int)OP_ALLREDUCE;
  py::class_<Plan>(m, "Plan")
      .def(py::init<>())
      .def("set_comm", &Plan::set_comm, py::keep_alive<1, 2>())
      .def("set_groups", &Plan::set_groups)
      .def("get_ptr", &Plan::get_ptr)
      .def("set_ptr", &Plan::set_ptr)
      .def("get_long", &Plan::get_long)
      .def("groups", &Plan::groups)
      .def("has_comm_ops", &Plan::has_comm_ops)
      .def("add", &Plan::add, py::arg("kind"), py::arg("payload"), py::arg("ints"), py::arg("floats"),
           py::arg("longs"), py::arg("ptrs"), py::arg("lane") = 0)
      .def("lane", &Plan::lane)
      .def("set_side_flush", &Plan::set_side_flush)
      .def("set_float", &Plan::set_float)
      .def("set_int", &Plan::set_int)
      .def("get_int", &Plan::get_int)
      .def("kind", &Plan::kind)
      .def("payload", &Plan::payload)
      .def("size", &Plan::size)
      .def("run", &Plan::run, py::arg("begin"), py::arg("end"), py::arg("stream"), py::arg("join") = true)
      .def("wait_side", &Plan::wait_side)
      .def("capture", &Plan::capture)
      .def("launch", &Plan::launch)
      .def("capture_dual", &Plan::capture_dual)
      .def("capture_lane", &Plan::capture_lane)
      .def("fork_side", &Plan::fork_side)
      .def("launch_side", &Plan::launch_side)
      .def("join_side", &Plan::join_side)
      .def("comm_range", &Plan::comm_range)
      .def("join_comm", &Plan::join_comm)
      .def("count_lane", &Plan::count_lane)
      .def("launch_dual", &Plan::launch_dual)
      .def("has_side", &Plan::has_side)
      .def("clear_graphs", &Plan::clear_graphs)
      .def("describe", &Plan::describe);
  m.def("conv", &py_conv);
  m.def("wgrad", &py_wgrad, py::arg("payload"), py::arg("splits"), py::arg("g_f32"), py::arg("stream"),
        py::arg("variant") = 0);
  m.def("wgrad_big_ok", &py_wgrad_big_ok);
  m.def("wgrad_stem_ok", [](py::bytes payload, int g_f32) {
    std::string s = payload;
    if (s.size() != sizeof(WgradArgs)) throw std::runtime_error("WgradArgs size mismatch");
    WgradArgs a;
    std::memcpy(&a, s.data(), sizeof(a));
    return wgrad_stem_ok(a, g_f32 != 0);
  });
  m.def("wgrad_big_pick_splits", &wgrad_big_pick_splits);
  m.def("wgrad_num_variants", &wgrad_num_variants);
  m.def("struct_sizes", &struct_sizes);
  m.def("pick_tile", &py_pick_tile);
  m.def("dw_wgrad_ws_floats", &dwconv_wgrad_ws_floats);
  m.def("big_ok", &py_big_ok);
  m.attr("TILE_BIG128") = TILE_BIG128;
  m.attr("TILE_BIG256") = TILE_BIG256;
  m.attr("TILE_BIG64") = TILE_BIG64;
  m.attr("TILE_BIG128D") = TILE_BIG128D;
  m.attr("TILE_IMG") = TILE_IMG;
  m.attr("TILE_STEM") = TILE_STEM;
  m.def("img_ok", [](py::bytes payload, int a_f32) {
    std::string s = payload;
    if (s.size() != sizeof(ConvArgs)) throw std::runtime_error("ConvArgs size mismatch");
    ConvArgs a;
    std::memcpy(&a, s.data(), sizeof(a));
    return conv_img_ok(a, a_f32 != 0);
  });
  m.def("stem_ok", [](py::bytes payload, int a_f32) {
    std::string s = payload;
    if (s.size() != sizeof(ConvArgs)) throw std::runtime_error("ConvArgs size mismatch");
    ConvArgs a;
    std::memcpy(&a, s.data(), sizeof(a));
    return conv_stem_ok(a, a_f32 != 0);
  });
  m.def("pick_splits", &py_pick_splits);
  m.def("effective_splits", &py_effective_splits);
  m.def("wgrad_batch_sig", &py_wgrad_batch_sig);
  m.def("wgrad_batch_pack", &py_wgrad_batch_pack);
  m.attr("WG_BATCH_MAX") = WG_BATCH_MAX;
  m.def("rows_grid", &rows_grid);
  m.def("pool_rows_grid", &pool_rows_grid);
  m.def("num_tiles", &conv_num_tiles);
  m.def("tile_bm", &conv_tile_bm);
  m.def("tile_bn", &conv_tile_bn);
  m.def("tile_bk", &conv_tile_bk);
  m.def("rmsprop", &py_rmsprop);
  m.def("host_alloc", &py_host_alloc);
  m.def("host_free", &py_host_free);
  m.def("secagg_mask", &py_secagg_mask, py::arg("x"), py::arg("out"), py::arg("n"), py::arg("seg_scale"),
        py::arg("seg_end"), py::arg("nseg"), py::arg("clip"), py::arg("nclients"), py::arg("rank"), py::arg("keys"),
        py::arg("round_"), py::arg("alive"), py::arg("stream"), py::arg("accumulate") = 0);
  m.def("secagg_unmask", &py_secagg_unmask);
  m.def("secagg_absmax", &py_secagg_absmax);
  m.def("group_metrics", &py_group_metrics);
  m.attr("OP_CONV") = (int)OP_CONV;
  m.attr("OP_DENSE_STAGE") = (int)OP_DENSE_STAGE;
  m.attr("OP_DENSE_STAGE_BWD") = (int)OP_DENSE_STAGE_BWD;
  m.attr("DSB_KG") = DSB_KG;
  m.attr("DSB_MAX_CG") = DSB_MAX_CG;
  m.def("dsb_sync_words", &dsb_sync_words);
  m.attr("DS_SLOTS") = DS_SLOTS;
  m.def("dense_stage_tasks", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(DenseStageArgs)) throw std::runtime_error("dense_stage_tasks: bad payload");
    return dense_stage_tasks(*reinterpret_cast<const DenseStageArgs*>(s.data()));
  });
  m.def("dense_stage_phase_tiles", [](int M, int ksplit) {
    int nA, nB;
    dense_stage_phase_tiles(M, ksplit, nA, nB);
    return py::make_tuple(nA, nB);
  }, py::arg("M"), py::arg("ksplit") = 1);
  m.def("dense_stage_sync_words", &dense_stage_sync_words);
  m.def("dense_rows_bwd_part_floats", &dense_rows_bwd_part_floats);
  m.def("dense_rows_bwd_geometry", [](int N, int H, int W, int ld, int nlayers) {
    int ipg = 0, grid = 0;
    const bool ok = dense_rows_bwd_geometry(N, H, W, ld, nlayers, ipg, grid);
    return py::make_tuple(ok, ipg, grid);
  });
  m.def("dense_rows_geometry", [](int N, int H, int W, int ld, int max_cin) {
    int rb = 0, ipg = 0, grid = 0;
    const bool ok = dense_rows_geometry(N, H, W, ld, max_cin, rb, ipg, grid);
    return py::make_tuple(ok, rb, ipg, grid);
  });
  m.def("dense_stage_partial_floats", &dense_stage_partial_floats);
  m.def("dense_stage_default_ksplit", &dense_stage_default_ksplit);
  m.attr("DS_MAX_KSPLIT") = DS_MAX_KSPLIT;
  m.def("dense_stage_shape_ok", &dense_stage_shape_ok);
  m.attr("DS_SCRATCH_PER_LAYER") = DS_SCRATCH_PER_LAYER;
  m.attr("DS_MAX_CIN") = DS_MAX_CIN;
  m.attr("OP_MB_CHAIN") = (int)OP_MB_CHAIN;
  m.attr("OP_MB_INFER") = (int)OP_MB_INFER;
  m.attr("OP_DENSE_INFER") = (int)OP_DENSE_INFER;
  m.def("dense_infer_smem", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(DenseInferArgs)) throw std::runtime_error("dense_infer_smem: bad payload");
    return dense_infer_smem(*reinterpret_cast<const DenseInferArgs*>(s.data()));
  });
  m.def("dense_img_ok", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(DenseStageArgs)) throw std::runtime_error("dense_img_ok: bad payload");
    return dense_img_ok(*reinterpret_cast<const DenseStageArgs*>(s.data()));
  });
  m.def("dw_bwd_fused_ok", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(DwArgs)) throw std::runtime_error("dw_bwd_fused_ok: bad payload");
    return dwconv_bwd_fused_ok(*reinterpret_cast<const DwArgs*>(s.data()));
  });
  m.def("mb_infer_smem", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(MbInferArgs)) throw std::runtime_error("mb_infer_smem: bad payload");
    return mb_infer_smem(*reinterpret_cast<const MbInferArgs*>(s.data()));
  });
  m.def("mb_infer_slab_floats", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(MbInferArgs)) throw std::runtime_error("mb_infer_slab_floats: bad payload");
    return mb_infer_slab_floats(*reinterpret_cast<const MbInferArgs*>(s.data()));
  });
  m.attr("MBI_MAX_ACC") = MBI_MAX_ACC;
  m.def("mb_phase_ok", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(MbPhaseDesc)) throw std::runtime_error("mb_phase_ok: bad payload");
    return mb_phase_ok(*reinterpret_cast<const MbPhaseDesc*>(s.data()));
  });
  m.def("mb_phase_smem", [](py::bytes payload) {
    std::string s = payload;
    if (s.size() != sizeof(MbPhaseDesc)) throw std::runtime_error("mb_phase_smem: bad payload");
    return mb_phase_smem(*reinterpret_cast<const MbPhaseDesc*>(s.data()));
  });
  m.attr("MB_SMEM_LIMIT") = mb_smem_limit();
  m.attr("MB_MAX_PHASES") = MB_MAX_PHASES;
}
