// mivod control-plane wire format and blocking TCP helpers.
//
// Messages are length-prefixed little-endian binary records (no FlatBuffers,
// no MPI): [u32 length][payload].  A RequestList carries a rank's newly
// submitted named collectives for one cycle; a ResponseList carries the
// coordinator's agreed, ordered, fused execution plan.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace mvcore {

enum Kind : uint8_t { ALLREDUCE = 0, ALLGATHER = 1, BROADCAST = 2, ALLTOALL = 3 };

struct Request {
  std::string name;
  uint8_t kind = 0;
  std::string dtype;
  std::vector<int64_t> shape;
  int32_t root = 0;
  int32_t op = 0;
  int32_t device = -1;  // -1 = CPU
  int64_t nbytes = 0;
  double prescale = 1.0;   // per-rank contribution scale (fused only with equal factors)
  double postscale = 1.0;
  int32_t rank = 0;     // filled by the coordinator
};

struct Response {
  uint8_t kind = 0;
  std::string error;
  std::vector<std::string> names;
};

class Writer {
 public:
  std::string buf;
  void u8(uint8_t v) { buf.push_back((char)v); }
  void u32(uint32_t v) { buf.append(reinterpret_cast<const char*>(&v), 4); }
  void i32(int32_t v) { buf.append(reinterpret_cast<const char*>(&v), 4); }
  void i64(int64_t v) { buf.append(reinterpret_cast<const char*>(&v), 8); }
  void f64(double v) { buf.append(reinterpret_cast<const char*>(&v), 8); }
  void str(const std::string& s) { u32((uint32_t)s.size()); buf.append(s); }
};

class Reader {
 public:
  explicit Reader(const std::string& b) : b_(b) {}
  uint8_t u8() { need(1); return (uint8_t)b_[p_++]; }
  uint32_t u32() { uint32_t v; cp(&v, 4); return v; }
  int32_t i32() { int32_t v; cp(&v, 4); return v; }
  int64_t i64() { int64_t v; cp(&v, 8); return v; }
  double f64() { double v; cp(&v, 8); return v; }
  bool done() const { return p_ >= b_.size(); }
  std::string str() { uint32_t n = u32(); need(n); std::string s = b_.substr(p_, n); p_ += n; return s; }

 private:
  void need(size_t n) {
    if (p_ + n > b_.size()) throw std::runtime_error("mivod wire: truncated message");
  }
  void cp(void* d, size_t n) { need(n); std::memcpy(d, b_.data() + p_, n); p_ += n; }
  const std::string& b_;
  size_t p_ = 0;
};

void encode_requests(Writer& w, const std::vector<Request>& rs, bool shutdown);
std::vector<Request> decode_requests(Reader& r, bool* shutdown);
void encode_responses(Writer& w, const std::vector<Response>& rs, bool shutdown);
std::vector<Response> decode_responses(Reader& r, bool* shutdown);

// ---- sockets ----
int tcp_listen(const std::string& host, int* port);  // port 0 => ephemeral, returns bound port
int tcp_accept(int lfd, double timeout_s);
int tcp_connect(const std::string& host, int port, double timeout_s);
void send_msg(int fd, const std::string& payload);
std::string recv_msg(int fd);
void close_fd(int fd);

}  // namespace mvcore
