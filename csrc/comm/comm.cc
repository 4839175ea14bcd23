#include "comm.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>

namespace mvcomm {

#define MV_NCCL(call)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (call);                                                           \
    if (r_ != ncclSuccess && r_ != ncclInProgress) {                                    \
      const char* last_ = ncclGetLastError(nullptr);                                    \
      throw std::runtime_error(std::string("mivod RCCL: ") + #call + ": " +             \
                               ncclGetErrorString(r_) + (last_ && *last_ ? " (" : "") + \
                               (last_ && *last_ ? last_ : "") +                         \
                               (last_ && *last_ ? ")" : ""));                           \
    }                                                                                   \
  } while (0)

#define MV_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw std::runtime_error(std::string("mivod HIP: ") + #call + ": " +             \
                               hipGetErrorString(e_));                                 \
  } while (0)

std::string unique_id() {
  ncclUniqueId id;
  MV_NCCL(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int rccl_version() {
  int v = 0;
  MV_NCCL(ncclGetVersion(&v));
  return v;
}

// NCCL_VERSION(X,Y,Z) codes are X*10000 + Y*100 + Z from 2.9 on
static int major_minor(int code) { return code / 100; }

std::string version_note() {
  const int rt = rccl_version();
  if (major_minor(rt) == major_minor(NCCL_VERSION_CODE)) return "";
  return "RCCL run-time library " + std::to_string(rt) + " != header " +
         std::to_string(NCCL_VERSION_CODE) +
         " (mivod links the librccl PyTorch loads; version-dependent features are gated on "
         "the run-time version)";
}

bool runtime_has_ctas_config() { return rccl_version() >= 21700; }
bool runtime_has_fp8() { return rccl_version() >= 22400; }

int Comm::count() const {
  int n = 0;
  MV_NCCL(ncclCommCount(comm_, &n));
  return n;
}

size_t Comm::dtype_size(int dtype) {
  switch (dtype) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat8e4m3: case ncclFloat8e5m2:
      // the enum codes of the header; an older run-time library reads them as
      // something else (or rejects them)
      if (!runtime_has_fp8())
        throw std::invalid_argument("mivod RCCL: fp8 needs RCCL >= 2.24 at run time (have " +
                                    std::to_string(rccl_version()) + ")");
      return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
  }
  throw std::invalid_argument("mivod RCCL: unsupported dtype code " + std::to_string(dtype));
}

Comm::Comm(const std::string& uid, int rank, int size, int device, double timeout_s,
           bool exit_on_abort, int min_ctas, int max_ctas)
    : rank_(rank), size_(size), device_(device), min_ctas_(min_ctas), max_ctas_(max_ctas),
      timeout_s_(timeout_s), exit_on_abort_(exit_on_abort) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES)
    throw std::invalid_argument("mivod RCCL: unique id must be 128 bytes");
  if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("mivod RCCL: bad rank");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  MV_HIP(hipSetDevice(device));
  if ((min_ctas > 0 || max_ctas > 0) && !runtime_has_ctas_config()) {
    fprintf(stderr, "[mivod] RCCL %d has no ncclConfig_t CTA range; using the default\n",
            rccl_version());
    min_ctas = max_ctas = min_ctas_ = max_ctas_ = 0;
  }
  if (min_ctas > 0 || max_ctas > 0) {
    // CTA (= channel) range of this communicator: how many xGMI rings a collective
    // spreads over (the RCCL autotune in mivod/parallel/autotune.py sweeps it)
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    if (min_ctas > 0) cfg.minCTAs = min_ctas;
    if (max_ctas > 0) cfg.maxCTAs = max_ctas;
    MV_NCCL(ncclCommInitRankConfig(&comm_, size, id, rank, &cfg));
  } else {
    MV_NCCL(ncclCommInitRank(&comm_, size, id, rank));
  }
  start_watchdog();
}

Comm::~Comm() {
  try {
    destroy();
  } catch (...) {
  }
}

void Comm::start_watchdog() {
  stop_ = false;
  watchdog_ = std::thread([this] { watchdog_loop(); });
}

void Comm::destroy() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  std::lock_guard<std::mutex> g(mu_);
  if (comm_ != nullptr) {
    if (!aborted_) {
      for (auto& p : pending_) hipEventSynchronize(p.ev);
      ncclCommDestroy(comm_);
    }
    comm_ = nullptr;
  }
  for (auto& p : pending_) hipEventDestroy(p.ev);
  pending_.clear();
  for (auto e : free_events_) hipEventDestroy(e);
  free_events_.clear();
}

void Comm::check() const {
  if (aborted_) {
    std::lock_guard<std::mutex> g(mu_);
    throw std::runtime_error("mivod RCCL communicator aborted: " + error_);
  }
}

std::string Comm::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

CommStats Comm::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return stats_;
}

int Comm::outstanding() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int)pending_.size();
}

void Comm::track(hipStream_t s, size_t bytes, const char* what) {
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> g(mu_);
    stats_.calls++;
    stats_.bytes += (int64_t)bytes;
    if (!free_events_.empty()) {
      ev = free_events_.back();
      free_events_.pop_back();
    } else {
      ev = nullptr;
    }
  }
  if (ev == nullptr) MV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  MV_HIP(hipEventRecord(ev, s));
  std::lock_guard<std::mutex> g(mu_);
  pending_.push_back({ev, std::chrono::steady_clock::now(), what});
}

void Comm::abort(const std::string& why) {
  bool expected = false;
  if (!aborted_.compare_exchange_strong(expected, true)) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    error_ = why;
  }
  fprintf(stderr, "[mivod] rank %d: RCCL watchdog: %s; aborting the communicator\n", rank_,
          why.c_str());
  fflush(stderr);
  if (comm_ != nullptr) ncclCommAbort(comm_);
  if (exit_on_abort_) {
    fprintf(stderr, "[mivod] rank %d: exiting (HOROVOD_STALL_SHUTDOWN_TIME_SECONDS)\n", rank_);
    fflush(stderr);
    std::_Exit(1);
  }
}

void Comm::watchdog_loop() {
  hipSetDevice(device_);
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::milliseconds(50));
    if (stop_ || aborted_) break;
    // retire completed collectives in issue order
    while (!pending_.empty()) {
      hipError_t q = hipEventQuery(pending_.front().ev);
      if (q == hipErrorNotReady) break;
      free_events_.push_back(pending_.front().ev);
      pending_.pop_front();
      stats_.completed++;
    }
    std::string why;
    if (!pending_.empty() && timeout_s_ > 0) {
      double age = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                 pending_.front().t).count();
      if (age > timeout_s_)
        why = std::string(pending_.front().what) + " did not complete within " +
              std::to_string((int)timeout_s_) + " s (a peer rank is dead or stalled)";
    }
    ncclComm_t c = comm_;
    lk.unlock();
    if (why.empty() && c != nullptr) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess &&
          ae != ncclInProgress)
        why = std::string("asynchronous RCCL error: ") + ncclGetErrorString(ae);
    }
    if (!why.empty()) {
      abort(why);
      lk.lock();
      break;
    }
    lk.lock();
  }
}

static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void Comm::allreduce(const void* in, void* out, size_t count, int dtype, int op,
                     uintptr_t stream) {
  check();
  MV_NCCL(ncclAllReduce(in, out, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, comm_,
                        S(stream)));
  track(S(stream), count * dtype_size(dtype), "ncclAllReduce");
}

void Comm::allreduce_premul(const void* in, void* out, size_t count, int dtype, double scale,
                            uintptr_t stream) {
  check();
  // scalar in the reduction dtype, host-immediate (read at enqueue time)
  union {
    double d;
    float f;
    _Float16 h;
    uint16_t b;
    char raw[8];
  } s;
  std::memset(s.raw, 0, sizeof(s.raw));
  switch (dtype) {
    case ncclFloat64: s.d = scale; break;
    case ncclFloat32: s.f = (float)scale; break;
    case ncclFloat16: s.h = (_Float16)scale; break;
    case ncclBfloat16: {
      float f = (float)scale;
      uint32_t u;
      std::memcpy(&u, &f, 4);
      u += 0x7FFFu + ((u >> 16) & 1u);   // round to nearest even
      s.b = (uint16_t)(u >> 16);
      break;
    }
    default: throw std::invalid_argument("mivod RCCL: premul needs a floating dtype");
  }
  ncclRedOp_t op;
  MV_NCCL(ncclRedOpCreatePreMulSum(&op, s.raw, (ncclDataType_t)dtype, ncclScalarHostImmediate,
                                   comm_));
  ncclResult_t r = ncclAllReduce(in, out, count, (ncclDataType_t)dtype, op, comm_, S(stream));
  ncclRedOpDestroy(op, comm_);
  MV_NCCL(r);
  track(S(stream), count * dtype_size(dtype), "ncclAllReduce(PreMulSum)");
}

void Comm::reduce_scatter(const void* in, void* out, size_t recvcount, int dtype, int op,
                          uintptr_t stream) {
  check();
  MV_NCCL(ncclReduceScatter(in, out, recvcount, (ncclDataType_t)dtype, (ncclRedOp_t)op, comm_,
                            S(stream)));
  track(S(stream), recvcount * size_ * dtype_size(dtype), "ncclReduceScatter");
}

void Comm::allgather(const void* in, void* out, size_t sendcount, int dtype, uintptr_t stream) {
  check();
  MV_NCCL(ncclAllGather(in, out, sendcount, (ncclDataType_t)dtype, comm_, S(stream)));
  track(S(stream), sendcount * size_ * dtype_size(dtype), "ncclAllGather");
}

void Comm::broadcast(const void* in, void* out, size_t count, int dtype, int root,
                     uintptr_t stream) {
  check();
  MV_NCCL(ncclBroadcast(in, out, count, (ncclDataType_t)dtype, root, comm_, S(stream)));
  track(S(stream), count * dtype_size(dtype), "ncclBroadcast");
}

void Comm::sendrecv(const void* sbuf, size_t scount, void* rbuf, size_t rcount, int dtype,
                    int peer, uintptr_t stream) {
  check();
  if (scount == 0 && rcount == 0) return;   // partners agree: my send == their recv
  MV_NCCL(ncclGroupStart());
  ncclResult_t r1 = ncclSuccess, r2 = ncclSuccess;
  if (scount) r1 = ncclSend(sbuf, scount, (ncclDataType_t)dtype, peer, comm_, S(stream));
  if (rcount) r2 = ncclRecv(rbuf, rcount, (ncclDataType_t)dtype, peer, comm_, S(stream));
  MV_NCCL(ncclGroupEnd());
  MV_NCCL(r1);
  MV_NCCL(r2);
  track(S(stream), scount * dtype_size(dtype), "ncclSend/ncclRecv");
}

void Comm::alltoallv(const void* sbuf, const std::vector<size_t>& scounts,
                     const std::vector<size_t>& sdispls, void* rbuf,
                     const std::vector<size_t>& rcounts, const std::vector<size_t>& rdispls,
                     int dtype, uintptr_t stream) {
  check();
  if ((int)scounts.size() != size_ || (int)rcounts.size() != size_ ||
      (int)sdispls.size() != size_ || (int)rdispls.size() != size_)
    throw std::invalid_argument("mivod RCCL alltoallv: one count/displacement per rank");
  size_t es = dtype_size(dtype);
  size_t total = 0;
  MV_NCCL(ncclGroupStart());
  for (int p = 0; p < size_; ++p) {
    const char* s = static_cast<const char*>(sbuf) + sdispls[p] * es;
    char* r = static_cast<char*>(rbuf) + rdispls[p] * es;
    if (scounts[p]) ncclSend(s, scounts[p], (ncclDataType_t)dtype, p, comm_, S(stream));
    if (rcounts[p]) ncclRecv(r, rcounts[p], (ncclDataType_t)dtype, p, comm_, S(stream));
    total += scounts[p] + rcounts[p];
  }
  MV_NCCL(ncclGroupEnd());
  track(S(stream), total * es, "ncclAllToAllv");
}

std::unique_ptr<Comm> Comm::split(int color, int key) {
  check();
  std::unique_ptr<Comm> c(new Comm());
  c->device_ = device_;
  c->timeout_s_ = timeout_s_;
  c->exit_on_abort_ = exit_on_abort_;
  c->min_ctas_ = min_ctas_;        // a split child inherits the parent's config
  c->max_ctas_ = max_ctas_;
  MV_NCCL(ncclCommSplit(comm_, color, key, &c->comm_, nullptr));
  if (c->comm_ == nullptr) return nullptr;     // color == NCCL_SPLIT_NOCOLOR
  MV_NCCL(ncclCommCount(c->comm_, &c->size_));
  MV_NCCL(ncclCommUserRank(c->comm_, &c->rank_));
  c->start_watchdog();
  return c;
}

}  // namespace mvcomm
