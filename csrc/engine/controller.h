// mivod coordinator: cross-rank negotiation of named collectives.
//
// Parity: horovod 0.18.1 common/operations.cc RunLoopOnce + controller /
// mpi_controller, re-designed without MPI: rank 0
// owns a TCP star (one persistent socket per worker).  Every cycle each rank
// sends the requests it enqueued since the last cycle; rank 0 records them in
// its message table, and once a name has been submitted by all `size` ranks it
// validates them (kind / dtype / shape / root / op must agree, otherwise an
// error response is sent to all ranks instead of a hang), orders the ready
// names by first arrival, fuses compatible allreduces up to the fusion
// threshold, and broadcasts the response list.  The stall inspector runs on
// rank 0 inside the same loop.
//
// Response cache (HOROVOD_CACHE_CAPACITY, default 1024; 0 disables it):
// requests already negotiated are shipped as a slot id instead of the full
// record, and a cycle whose requests are all cached ships one bit vector of
// capacity/8 bytes when that is smaller (horovod's cache-hit bit vectors).
// Each submitting rank owns its slot assignment (FIFO eviction when full); the
// coordinator mirrors it per rank, so the two sides never need a global
// agreement.
//
// Issue order: every cycle each rank also reports how many GPU collectives it
// has issued (``position``); the coordinator answers with exec_at = max over
// ranks, the point in every rank's collective sequence at which this cycle's
// GPU responses run (mivod/parallel/order.py).
#pragma once
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "timeline.h"
#include "wire.h"

namespace mvcore {

struct ControllerConfig {
  int rank = 0;
  int size = 1;
  std::string host = "127.0.0.1";
  int port = 0;                       // rank 0: 0 => ephemeral
  int64_t fusion_threshold = 64 << 20;
  double stall_check_s = 60.0;
  double stall_shutdown_s = 0.0;      // 0 => never
  bool stall_check = true;
  double connect_timeout_s = 300.0;
  int cache_capacity = 1024;          // HOROVOD_CACHE_CAPACITY; 0 = no response cache
};

struct StallReport {
  std::string name;
  std::vector<int> missing_ranks;
  double age_s;
};

class Controller {
 public:
  explicit Controller(const ControllerConfig& cfg);
  ~Controller();

  // rank 0: start listening, returns the bound port (publish it to workers)
  int listen();
  // rank 0: accept size-1 workers.  workers: connect to host:port.
  void connect(const std::string& host, int port);

  // One negotiation cycle.  Returns responses; sets *all_shutdown when every
  // rank has requested shutdown.
  std::vector<Response> negotiate(const std::vector<Request>& reqs, bool shutdown,
                                  bool* all_shutdown, int64_t position = 0,
                                  int64_t* exec_at = nullptr);

  void set_timeline(std::shared_ptr<Timeline> tl) { tl_ = std::move(tl); }
  void close();

  // observability / tests
  std::vector<StallReport> last_stalls() const;
  int64_t cycles() const { return cycles_; }
  int64_t cache_hits() const { return cache_hits_; }
  int64_t bitvector_cycles() const { return bitvector_cycles_; }
  int cache_size() const { return (int)cache_req_.size(); }
  std::vector<Response> coordinate_for_test(const std::vector<std::vector<Request>>& per_rank);

 private:
  struct Entry {
    std::vector<Request> reqs;  // one per rank (by rank index), empty name = not yet
    int count = 0;
    int64_t order = 0;
    std::chrono::steady_clock::time_point first_seen;
    bool warned = false;
  };
  std::vector<Response> coordinate(std::vector<std::vector<Request>>& per_rank);
  std::string validate(const Entry& e) const;
  std::vector<Response> fuse(std::vector<Response> ready) const;
  void stall_check(std::vector<Response>* errs);
  std::string encode_cached(const std::vector<Request>& reqs, bool shutdown, int64_t position);
  std::vector<Request> decode_cached(const std::string& msg, int from_rank, bool* shutdown,
                                     int64_t* position);

  ControllerConfig cfg_;
  int lfd_ = -1;
  int fd_ = -1;                 // worker -> coordinator
  std::vector<int> peers_;      // coordinator: fd per rank (peers_[0] unused)
  std::map<std::string, Entry> table_;
  int64_t order_ = 0;
  int64_t cycles_ = 0;
  int64_t cache_hits_ = 0;
  int64_t bitvector_cycles_ = 0;
  std::chrono::steady_clock::time_point last_stall_check_;
  std::vector<StallReport> last_stalls_;
  std::shared_ptr<Timeline> tl_;
  mutable std::mutex mu_;
  // response cache: name -> slot (this rank's assignment); mirrored per rank on
  // the coordinator.  FIFO eviction once cache_capacity slots are in use.
  std::unordered_map<std::string, uint32_t> cache_id_;
  std::vector<Request> cache_req_;                // slot -> request
  uint32_t next_evict_ = 0;
  std::vector<std::vector<Request>> peer_cache_;  // coordinator: per-rank slot -> request
};

}  // namespace mvcore
