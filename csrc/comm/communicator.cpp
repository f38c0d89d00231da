// Native RCCL communicator (see communicator.h).
#include "communicator.h"

#include <chrono>
#include <thread>

#include <cstring>
#include <stdexcept>

namespace idc {

namespace {

inline void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case CD_F32: return ncclFloat32;
    case CD_BF16: return ncclBfloat16;
    case CD_I32: return ncclInt32;
    case CD_F64: return ncclFloat64;
    case CD_U32: return ncclUint32;
    case CD_I64: return ncclInt64;
    case CD_U8: return ncclUint8;
    default: throw std::runtime_error("Communicator: unknown dtype code");
  }
}

ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case CO_SUM: return ncclSum;
    case CO_MAX: return ncclMax;
    case CO_MIN: return ncclMin;
    case CO_AVG: return ncclAvg;
    default: throw std::runtime_error("Communicator: unknown reduction op");
  }
}

}  // namespace

std::string Communicator::make_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

Communicator::Communicator(int rank, int world, const std::string& unique_id, int device, double init_timeout_s)
    : rank_(rank), world_(world), device_(device) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("Communicator: bad rank/world");
  if (unique_id.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("Communicator: unique id must be 128 bytes");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), NCCL_UNIQUE_ID_BYTES);
  hip_check(hipSetDevice(device), "hipSetDevice");
  // the collectives' own lane: non-blocking, so it never serialises against the legacy stream
  hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate(comm)");
  ncclResult_t r;
  if (init_timeout_s > 0.0) {
    // non-blocking creation: a rank whose peers never arrive gives up after init_timeout_s
    // instead of blocking forever inside ncclCommInitRank
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    nonblocking_ = true;
    settle_timeout_s_ = init_timeout_s;
    r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
    if (r == ncclInProgress || r == ncclSuccess) {
      const double t0 = now_s();
      ncclResult_t st = ncclInProgress;
      while (comm_ != nullptr) {
        if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) { st = ncclSystemError; break; }
        if (st != ncclInProgress) break;
        if (now_s() - t0 > init_timeout_s) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (st != ncclSuccess) {
        if (comm_) ncclCommAbort(comm_);
        comm_ = nullptr;
        hipStreamDestroy(stream_);
        stream_ = nullptr;
        if (st == ncclInProgress)
          throw std::runtime_error("ncclCommInitRankConfig: peers did not join within the init timeout");
        nccl_check(st, "ncclCommInitRankConfig");
      }
      r = ncclSuccess;
    }
  } else {
    r = ncclCommInitRank(&comm_, world, id, rank);
  }
  if (r != ncclSuccess) {
    hipStreamDestroy(stream_);
    stream_ = nullptr;
    comm_ = nullptr;
    nccl_check(r, "ncclCommInitRank");
  }
  hip_check(hipEventCreateWithFlags(&mark_ev_, hipEventDisableTiming), "hipEventCreate(mark)");
}

void Communicator::settle(ncclResult_t r, const char* what) {
  if (r == ncclInProgress && nonblocking_) {
    // a non-blocking communicator may still be setting the call up: wait for it (bounded)
    const double t0 = now_s();
    ncclResult_t st = ncclInProgress;
    while (st == ncclInProgress) {
      nccl_check(ncclCommGetAsyncError(comm_, &st), "ncclCommGetAsyncError");
      if (st == ncclInProgress && now_s() - t0 > settle_timeout_s_)
        throw std::runtime_error(std::string(what) + ": still in progress after the timeout");
    }
    r = st;
  }
  nccl_check(r, what);
}

void Communicator::mark() {
  require_open();
  if (mark_pending_ && hipEventQuery(mark_ev_) == hipErrorNotReady) return;  // oldest one stays
  hip_check(hipEventRecord(mark_ev_, stream_), "hipEventRecord(mark)");
  mark_pending_ = true;
  mark_t_ = now_s();
}

double Communicator::mark_age() {
  if (!mark_pending_ || !mark_ev_) return 0.0;
  if (hipEventQuery(mark_ev_) != hipErrorNotReady) {
    mark_pending_ = false;
    return 0.0;
  }
  return now_s() - mark_t_;
}

Communicator::~Communicator() {
  try {
    close();
  } catch (...) {
  }
}

void Communicator::close() {
  if (mark_ev_) {
    hipEventDestroy(mark_ev_);
    mark_ev_ = nullptr;
  }
  if (comm_) {
    if (stream_) hipStreamSynchronize(stream_);
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  if (stream_) {
    hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
}

void Communicator::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void Communicator::require_open() const {
  if (!comm_) throw std::runtime_error("Communicator: closed");
}

void Communicator::check_async() const {
  require_open();
  ncclResult_t ar = ncclSuccess;
  nccl_check(ncclCommGetAsyncError(comm_, &ar), "ncclCommGetAsyncError");
  nccl_check(ar, "RCCL asynchronous error");
}

void Communicator::all_reduce(void* buf, long long count, int dtype, int op, hipStream_t st) {
  require_open();
  if (count <= 0) return;
  settle(ncclAllReduce(buf, buf, (size_t)count, to_nccl(dtype), to_nccl_op(op), comm_, st ? st : stream_),
         "ncclAllReduce");
  ++ncoll_;
}

void Communicator::reduce(void* buf, long long count, int dtype, int op, int root, hipStream_t st) {
  require_open();
  if (count <= 0) return;
  settle(ncclReduce(buf, buf, (size_t)count, to_nccl(dtype), to_nccl_op(op), root, comm_, st ? st : stream_),
         "ncclReduce");
  ++ncoll_;
}

void Communicator::broadcast(void* buf, long long count, int dtype, int root, hipStream_t st) {
  require_open();
  if (count <= 0) return;
  settle(ncclBroadcast(buf, buf, (size_t)count, to_nccl(dtype), root, comm_, st ? st : stream_),
         "ncclBroadcast");
  ++ncoll_;
}

void Communicator::all_gather(const void* send, void* recv, long long count_per_rank, int dtype, hipStream_t st) {
  require_open();
  if (count_per_rank <= 0) return;
  settle(ncclAllGather(send, recv, (size_t)count_per_rank, to_nccl(dtype), comm_, st ? st : stream_),
         "ncclAllGather");
  ++ncoll_;
}

void Communicator::group_start() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
void Communicator::group_end() {
  const ncclResult_t r = ncclGroupEnd();
  if (comm_) settle(r, "ncclGroupEnd");
  else nccl_check(r, "ncclGroupEnd");
}

int rccl_version() {
  int v = 0;
  nccl_check(ncclGetVersion(&v), "ncclGetVersion");
  return v;
}

}  // namespace idc
