#include "controller.h"

#include <algorithm>
#include <cstdio>
#include <sstream>
#include <stdexcept>

namespace mvcore {

static const char* kind_name(uint8_t k) {
  switch (k) {
    case ALLREDUCE: return "allreduce";
    case ALLGATHER: return "allgather";
    case BROADCAST: return "broadcast";
    case ALLTOALL: return "alltoall";
  }
  return "collective";
}

static std::string shape_str(const std::vector<int64_t>& s) {
  std::ostringstream o;
  o << "[";
  for (size_t i = 0; i < s.size(); ++i) o << (i ? ", " : "") << s[i];
  o << "]";
  return o.str();
}

static bool same_sig(const Request& a, const Request& b) {
  return a.kind == b.kind && a.dtype == b.dtype && a.shape == b.shape && a.root == b.root &&
         a.op == b.op && a.device == b.device && a.nbytes == b.nbytes &&
         a.prescale == b.prescale && a.postscale == b.postscale;
}

Controller::Controller(const ControllerConfig& cfg) : cfg_(cfg) {
  if (cfg_.size < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.size)
    throw std::invalid_argument("mivod controller: bad rank/size");
  last_stall_check_ = std::chrono::steady_clock::now();
  peer_cache_.resize(cfg_.size);
}

Controller::~Controller() { close(); }

int Controller::listen() {
  if (cfg_.rank != 0) throw std::logic_error("only rank 0 listens");
  int port = cfg_.port;
  lfd_ = tcp_listen("0.0.0.0", &port);
  cfg_.port = port;
  return port;
}

void Controller::connect(const std::string& host, int port) {
  if (cfg_.size == 1) return;
  if (cfg_.rank == 0) {
    if (lfd_ < 0) listen();
    peers_.assign(cfg_.size, -1);
    for (int i = 1; i < cfg_.size; ++i) {
      int fd = tcp_accept(lfd_, cfg_.connect_timeout_s);
      std::string hello = recv_msg(fd);
      Reader r(hello);
      int rk = r.i32();
      if (rk <= 0 || rk >= cfg_.size || peers_[rk] != -1) {
        close_fd(fd);
        throw std::runtime_error("mivod controller: bad hello from a worker");
      }
      peers_[rk] = fd;
    }
    close_fd(lfd_);
    lfd_ = -1;
  } else {
    fd_ = tcp_connect(host, port, cfg_.connect_timeout_s);
    Writer w;
    w.i32(cfg_.rank);
    send_msg(fd_, w.buf);
  }
}

void Controller::close() {
  close_fd(fd_);
  fd_ = -1;
  for (int& f : peers_) {
    close_fd(f);
    f = -1;
  }
  close_fd(lfd_);
  lfd_ = -1;
}

// ---- response-cache aware request encoding --------------------------------
// Message: [u8 shutdown][i64 position][u8 mode]
//   mode 0: [u32 n] n x ( [u8 0][u32 slot][record]  new, stored in `slot`
//                       | [u8 1][u32 slot]          cached
//                       | [u8 2][record] )          uncached (capacity 0)
//   mode 1: [u32 capacity][capacity/8 bytes: cached-slot bit vector]   (every
//           request of the cycle was a cache hit and the bit vector is smaller)
std::string Controller::encode_cached(const std::vector<Request>& reqs, bool shutdown,
                                      int64_t position) {
  Writer w;
  w.u8(shutdown ? 1 : 0);
  w.i64(position);
  const uint32_t cap = (uint32_t)std::max(0, cfg_.cache_capacity);
  std::vector<uint32_t> hit(reqs.size(), UINT32_MAX);
  bool all_hit = cap > 0 && !reqs.empty();
  for (size_t i = 0; i < reqs.size(); ++i) {
    auto it = cap ? cache_id_.find(reqs[i].name) : cache_id_.end();
    if (it != cache_id_.end() && same_sig(cache_req_[it->second], reqs[i])) hit[i] = it->second;
    else all_hit = false;
  }
  if (all_hit && (size_t)(cap + 7) / 8 + 4 < reqs.size() * 5) {
    std::string bits((cap + 7) / 8, '\0');
    for (uint32_t id : hit) bits[id / 8] |= (char)(1u << (id % 8));
    w.u8(1);
    w.u32(cap);
    w.buf.append(bits);
    return w.buf;
  }
  // sequential encoding, mirrored by the coordinator's sequential decode: a slot
  // evicted by an earlier request of this message is simply a miss later on
  w.u8(0);
  w.u32((uint32_t)reqs.size());
  for (size_t i = 0; i < reqs.size(); ++i) {
    const Request& r = reqs[i];
    auto hit_it = cap ? cache_id_.find(r.name) : cache_id_.end();
    if (hit_it != cache_id_.end() && same_sig(cache_req_[hit_it->second], r)) {
      w.u8(1);
      w.u32(hit_it->second);
      continue;
    }
    std::vector<Request> one{r};
    Writer tmp;
    encode_requests(tmp, one, false);
    if (cap == 0) {
      w.u8(2);
      w.str(tmp.buf);
      continue;
    }
    uint32_t slot;
    if (hit_it != cache_id_.end()) {
      slot = hit_it->second;                   // same name, new signature: overwrite
    } else if (cache_req_.size() < cap) {
      slot = (uint32_t)cache_req_.size();
      cache_req_.push_back(r);
    } else {
      slot = next_evict_;                      // FIFO eviction
      next_evict_ = (next_evict_ + 1) % cap;
      cache_id_.erase(cache_req_[slot].name);
    }
    cache_req_[slot] = r;
    cache_id_[r.name] = slot;
    w.u8(0);
    w.u32(slot);
    w.str(tmp.buf);
  }
  return w.buf;
}

std::vector<Request> Controller::decode_cached(const std::string& msg, int from_rank,
                                               bool* shutdown, int64_t* position) {
  Reader rd(msg);
  *shutdown = rd.u8() != 0;
  *position = rd.i64();
  const uint8_t mode = rd.u8();
  auto& pc = peer_cache_[from_rank];
  std::vector<Request> out;
  if (mode == 1) {
    uint32_t cap = rd.u32();
    std::string bits;
    for (uint32_t i = 0; i < (cap + 7) / 8; ++i) bits.push_back((char)rd.u8());
    for (uint32_t id = 0; id < cap; ++id)
      if (bits[id / 8] & (1u << (id % 8))) {
        if (id >= pc.size() || pc[id].name.empty())
          throw std::runtime_error("mivod controller: unknown cache slot");
        out.push_back(pc[id]);
        ++cache_hits_;
      }
    ++bitvector_cycles_;
    return out;
  }
  uint32_t n = rd.u32();
  out.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t tag = rd.u8();
    if (tag == 1) {
      uint32_t id = rd.u32();
      if (id >= pc.size() || pc[id].name.empty())
        throw std::runtime_error("mivod controller: unknown cache slot");
      out.push_back(pc[id]);
      ++cache_hits_;
      continue;
    }
    uint32_t slot = tag == 0 ? rd.u32() : 0;
    std::string rec = rd.str();
    Reader r2(rec);
    bool dummy;
    auto v = decode_requests(r2, &dummy);
    if (v.size() != 1) throw std::runtime_error("mivod controller: bad request record");
    if (tag == 0) {
      if (slot >= pc.size()) pc.resize(slot + 1);
      pc[slot] = v[0];
    }
    out.push_back(v[0]);
  }
  return out;
}

std::vector<Response> Controller::negotiate(const std::vector<Request>& reqs, bool shutdown,
                                            bool* all_shutdown, int64_t position,
                                            int64_t* exec_at) {
  std::lock_guard<std::mutex> g(mu_);
  ++cycles_;
  if (tl_) tl_->mark_cycle();
  *all_shutdown = false;
  if (exec_at) *exec_at = position;
  if (cfg_.size == 1) {
    std::vector<std::vector<Request>> pr{reqs};
    *all_shutdown = shutdown;
    return coordinate(pr);
  }
  if (cfg_.rank != 0) {
    send_msg(fd_, encode_cached(reqs, shutdown, position));
    std::string m = recv_msg(fd_);
    Reader rd(m);
    bool sd = false;
    auto resp = decode_responses(rd, &sd);
    int64_t e = rd.i64();
    if (exec_at) *exec_at = e;
    *all_shutdown = sd;
    return resp;
  }
  // coordinator: gather (own requests go through the same cache path)
  std::vector<std::vector<Request>> per_rank(cfg_.size);
  int n_shutdown = 0;
  int64_t emax = position;
  {
    std::string own = encode_cached(reqs, shutdown, position);
    bool sd;
    int64_t pos;
    per_rank[0] = decode_cached(own, 0, &sd, &pos);
    n_shutdown += sd ? 1 : 0;
  }
  for (int r = 1; r < cfg_.size; ++r) {
    std::string m = recv_msg(peers_[r]);
    bool sd;
    int64_t pos;
    per_rank[r] = decode_cached(m, r, &sd, &pos);
    n_shutdown += sd ? 1 : 0;
    emax = std::max(emax, pos);
  }
  auto resp = coordinate(per_rank);
  bool done = n_shutdown == cfg_.size;
  Writer w;
  encode_responses(w, resp, done);
  w.i64(emax);
  for (int r = 1; r < cfg_.size; ++r) send_msg(peers_[r], w.buf);
  *all_shutdown = done;
  if (exec_at) *exec_at = emax;
  return resp;
}

std::string Controller::validate(const Entry& e) const {
  const Request& a = e.reqs[0];
  for (int r = 1; r < cfg_.size; ++r) {
    const Request& b = e.reqs[r];
    std::ostringstream o;
    if (a.kind != b.kind) {
      o << "Mismatched collective operations: One rank did an " << kind_name(a.kind)
        << ", but another rank did an " << kind_name(b.kind) << ".";
      return o.str();
    }
    if (a.dtype != b.dtype) {
      o << "Mismatched data types: One rank had type " << a.dtype << ", but another rank had type "
        << b.dtype << ".";
      return o.str();
    }
    if ((a.device < 0) != (b.device < 0)) {
      o << "Mismatched " << kind_name(a.kind)
        << " CPU/GPU device selection: One rank specified device CPU, but another rank specified "
           "device GPU.";
      return o.str();
    }
    if (a.kind == ALLREDUCE || a.kind == BROADCAST) {
      if (a.shape != b.shape) {
        o << "Mismatched " << kind_name(a.kind) << " tensor shapes: One rank sent a tensor of shape "
          << shape_str(a.shape) << ", but another rank sent a tensor of shape " << shape_str(b.shape)
          << ".";
        return o.str();
      }
    }
    if (a.kind == ALLREDUCE && a.op != b.op) {
      o << "Mismatched allreduce reduction ops: " << a.op << " vs " << b.op << ".";
      return o.str();
    }
    if (a.kind == ALLREDUCE && (a.prescale != b.prescale || a.postscale != b.postscale)) {
      o << "Mismatched allreduce prescale/postscale factors: (" << a.prescale << ", "
        << a.postscale << ") vs (" << b.prescale << ", " << b.postscale << ").";
      return o.str();
    }
    if (a.kind == BROADCAST && a.root != b.root) {
      o << "Mismatched broadcast root ranks: One rank specified root rank " << a.root
        << ", but another rank specified root rank " << b.root << ".";
      return o.str();
    }
    if (a.kind == ALLGATHER || a.kind == ALLTOALL) {
      if (a.shape.size() != b.shape.size()) {
        o << "Mismatched " << kind_name(a.kind) << " tensor ranks: " << a.shape.size() << " vs "
          << b.shape.size() << ".";
        return o.str();
      }
      for (size_t d = 1; d < a.shape.size(); ++d)
        if (a.shape[d] != b.shape[d]) {
          o << "Mismatched " << kind_name(a.kind)
            << " tensor shapes: dimension " << d << " differs (" << shape_str(a.shape) << " vs "
            << shape_str(b.shape) << ").";
          return o.str();
        }
    }
  }
  if (a.kind == BROADCAST && (a.root < 0 || a.root >= cfg_.size))
    return "Invalid broadcast root rank " + std::to_string(a.root) + ".";
  return "";
}

std::vector<Response> Controller::fuse(std::vector<Response> ready) const {
  // Horovod-style look-ahead fusion: an allreduce absorbs later compatible
  // allreduces (same wire dtype / op / pre- and postscale / CPU-vs-GPU) while the fused byte count stays
  // under the threshold.  Adasum (op 2) tensors are never fused across names.
  std::vector<Response> out;
  std::vector<bool> used(ready.size(), false);
  auto req0 = [&](const Response& r) -> const Request& { return table_.at(r.names[0]).reqs[0]; };
  for (size_t i = 0; i < ready.size(); ++i) {
    if (used[i]) continue;
    Response cur = ready[i];
    used[i] = true;
    if (cur.kind == ALLREDUCE && cur.error.empty()) {
      const Request& a = req0(cur);
      int64_t bytes = a.nbytes;
      if (a.op != 2) {
        for (size_t j = i + 1; j < ready.size(); ++j) {
          if (used[j] || ready[j].kind != ALLREDUCE || !ready[j].error.empty()) continue;
          const Request& b = req0(ready[j]);
          if (b.dtype != a.dtype || b.op != a.op || (b.device < 0) != (a.device < 0)) continue;
          if (b.prescale != a.prescale || b.postscale != a.postscale) continue;
          if (bytes + b.nbytes > cfg_.fusion_threshold) continue;
          bytes += b.nbytes;
          cur.names.push_back(ready[j].names[0]);
          used[j] = true;
        }
      }
    }
    out.push_back(std::move(cur));
  }
  return out;
}

void Controller::stall_check(std::vector<Response>* errs) {
  auto now = std::chrono::steady_clock::now();
  if (!cfg_.stall_check) return;
  double since = std::chrono::duration<double>(now - last_stall_check_).count();
  if (since < std::min(cfg_.stall_check_s, 1.0) && cfg_.stall_shutdown_s <= 0) return;
  last_stall_check_ = now;
  std::vector<StallReport> reps;
  std::vector<std::string> kill;
  for (auto& kv : table_) {
    Entry& e = kv.second;
    double age = std::chrono::duration<double>(now - e.first_seen).count();
    if (age < cfg_.stall_check_s) continue;
    StallReport sr{kv.first, {}, age};
    for (int r = 0; r < cfg_.size; ++r)
      if (e.reqs[r].name.empty()) sr.missing_ranks.push_back(r);
    reps.push_back(sr);
    if (cfg_.stall_shutdown_s > 0 && age >= cfg_.stall_shutdown_s) kill.push_back(kv.first);
    if (!e.warned) {
      e.warned = true;
      std::ostringstream o;
      o << "[mivod] WARNING: One or more tensors were submitted to be reduced, gathered or "
           "broadcasted by subset of ranks and are waiting for remainder of ranks for more than "
        << (int)cfg_.stall_check_s
        << " seconds. This may indicate that different ranks are trying to submit different "
           "tensors or that only subset of ranks is submitting tensors, which will cause "
           "deadlock.\nStalled tensor: "
        << kv.first << " missing ranks:";
      for (int r : sr.missing_ranks) o << " " << r;
      fprintf(stderr, "%s\n", o.str().c_str());
      fflush(stderr);
    }
  }
  last_stalls_ = reps;
  for (const auto& name : kill) {
    Response r;
    r.kind = table_[name].reqs[0].name.empty() ? ALLREDUCE : table_[name].reqs[0].kind;
    r.error = "mivod stall shutdown: tensor " + name + " was not submitted by all ranks within " +
              std::to_string((int)cfg_.stall_shutdown_s) + " s";
    r.names = {name};
    errs->push_back(r);
    table_.erase(name);
  }
}

std::vector<Response> Controller::coordinate(std::vector<std::vector<Request>>& per_rank) {
  auto now = std::chrono::steady_clock::now();
  std::vector<std::pair<int64_t, std::string>> became_ready;
  for (int r = 0; r < (int)per_rank.size(); ++r) {
    for (auto& q : per_rank[r]) {
      q.rank = r;
      auto it = table_.find(q.name);
      if (it == table_.end()) {
        Entry e;
        e.reqs.resize(cfg_.size);
        e.order = order_++;
        e.first_seen = now;
        it = table_.emplace(q.name, std::move(e)).first;
        if (tl_) tl_->start(q.name, std::string("NEGOTIATE_") + kind_name(q.kind));
      }
      Entry& e = it->second;
      if (!e.reqs[r].name.empty()) continue;  // duplicate submission from one rank
      e.reqs[r] = q;
      e.count++;
      if (tl_) tl_->instant(q.name, std::to_string(r));
      if (e.count == cfg_.size) became_ready.emplace_back(e.order, q.name);
    }
  }
  std::sort(became_ready.begin(), became_ready.end());
  std::vector<Response> ready, errors;
  for (auto& br : became_ready) {
    Entry& e = table_[br.second];
    Response resp;
    resp.kind = e.reqs[0].kind;
    resp.names = {br.second};
    resp.error = validate(e);
    if (tl_) tl_->end(br.second);
    if (!resp.error.empty()) errors.push_back(resp);
    else ready.push_back(resp);
  }
  auto out = fuse(ready);
  for (auto& br : became_ready) table_.erase(br.second);
  for (auto& e : errors) out.push_back(e);
  stall_check(&out);
  return out;
}

std::vector<Response> Controller::coordinate_for_test(
    const std::vector<std::vector<Request>>& per_rank) {
  std::lock_guard<std::mutex> g(mu_);
  auto pr = per_rank;
  pr.resize(cfg_.size);
  return coordinate(pr);
}

std::vector<StallReport> Controller::last_stalls() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_stalls_;
}

}  // namespace mvcore
