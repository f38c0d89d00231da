// Native RCCL communicator for the idc_models_amd MI355X runtime (SURVEY §5 "distributed comm
// backend", §2.5 C1/C2/C5/C6/C9).
//
// One process per GPU.  A Communicator owns
//   * an RCCL communicator (ncclComm_t) bootstrapped from a unique id that rank 0 creates and the
//     Python side hands to every rank through the torch.distributed TCPStore, and
//   * its own non-blocking HIP stream, on which every collective it issues runs.
//
// Ordering against compute is by HIP events only (no host synchronisation): the plan executor
// (csrc/runtime/plan.cpp, op kind OP_ALLREDUCE) records an event on the main lane (and on the
// weight-gradient side lane) at a bucket boundary, makes the comm stream wait for it, enqueues
// ncclAllReduce on the comm stream and joins the comm stream back into the main lane at the end of
// the backward range.  All of that is plain stream work, so it is also legal inside a HIP-graph
// capture.
//
// The reference reaches the same collective implicitly, through MirroredStrategy's NCCL all-reduce
// (/root/reference/dist_model_tf_vgg.py:115, dist_model_tf_dense.py:20-24).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

namespace idc {

// dtype / op codes shared with idc_models_amd/parallel/native_comm.py
enum CommDtype : int { CD_F32 = 0, CD_BF16 = 1, CD_I32 = 2, CD_F64 = 3, CD_U32 = 4, CD_I64 = 5, CD_U8 = 6 };
enum CommOp : int { CO_SUM = 0, CO_MAX = 1, CO_MIN = 2, CO_AVG = 3 };

class Communicator {
 public:
  // init_timeout_s > 0: the communicator is created non-blocking (ncclCommInitRankConfig,
  // blocking = 0) and the constructor polls its state, aborting and throwing after that many
  // seconds (a peer that never joins); 0: blocking ncclCommInitRank
  Communicator(int rank, int world, const std::string& unique_id, int device, double init_timeout_s = 0.0);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  static std::string make_unique_id();

  // every collective is enqueued on `st` (nullptr: the communicator's own stream)
  void all_reduce(void* buf, long long count, int dtype, int op, hipStream_t st);
  void reduce(void* buf, long long count, int dtype, int op, int root, hipStream_t st);
  void broadcast(void* buf, long long count, int dtype, int root, hipStream_t st);
  void all_gather(const void* send, void* recv, long long count_per_rank, int dtype, hipStream_t st);
  void group_start();
  void group_end();

  // raises if RCCL reported an asynchronous error (peer failure, timeout in the proxy, ...)
  void check_async() const;
  void abort();
  void close();

  // Progress marks for the host watchdog (parallel/watchdog.py): mark() records an event on the
  // comm stream after the collectives enqueued so far, unless the previous mark is still
  // outstanding (so the age below is that of the OLDEST unfinished mark); mark_age() is the
  // seconds since that mark was recorded while it has not completed, 0 when none is pending.
  void mark();
  double mark_age();

  hipStream_t stream() const { return stream_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  bool open() const { return comm_ != nullptr; }
  long long collectives() const { return ncoll_; }

 private:
  void require_open() const;
  void settle(ncclResult_t r, const char* what);  // non-blocking comms: wait out ncclInProgress
  ncclComm_t comm_ = nullptr;
  bool nonblocking_ = false;
  double settle_timeout_s_ = 0.0;
  hipEvent_t mark_ev_ = nullptr;
  bool mark_pending_ = false;
  double mark_t_ = 0.0;
  hipStream_t stream_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
  long long ncoll_ = 0;
};

int rccl_version();

}  // namespace idc
