#include "ring.h"

#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "wire.h"

namespace mvcore {

int ring_dtype_size(int dtype) {
  switch (dtype) {
    case kF32: case kI32: return 4;
    case kF64: case kI64: return 8;
    case kF16: case kBF16: return 2;
    case kU8: case kI8: return 1;
  }
  throw std::invalid_argument("mivod ring: unknown dtype code " + std::to_string(dtype));
}

// ---------------------------------------------------------------- reductions
namespace {

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_bf16(float f) {  // round to nearest even; NaN stays NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

inline float f16_to_f32(uint16_t h) {  // portable IEEE half -> float
  const uint32_t s = (uint32_t)(h & 0x8000) << 16;
  uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {  // subnormal: renormalise
      e = 113;
      while (!(m & 0x400)) { m <<= 1; --e; }
      u = s | (e << 23) | ((m & 0x3ff) << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 112) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_f16(float f) {  // round to nearest even, portable
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint16_t s = (uint16_t)((u >> 16) & 0x8000);
  const int32_t e = (int32_t)((u >> 23) & 0xff) - 127 + 15;
  uint32_t m = u & 0x7fffff;
  if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(s | 0x7c00 | (m ? 0x200 : 0));
  if (e >= 31) return (uint16_t)(s | 0x7c00);
  if (e <= 0) {
    if (e < -10) return s;
    m |= 0x800000;
    const int shift = 14 - e;
    uint32_t hm = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (hm & 1))) ++hm;
    return (uint16_t)(s | hm);
  }
  uint32_t hm = m >> 13;
  const uint32_t rem = m & 0x1fff;
  uint32_t out = ((uint32_t)e << 10) | hm;
  if (rem > 0x1000 || (rem == 0x1000 && (hm & 1))) ++out;  // may carry into the exponent
  return (uint16_t)(s | out);
}

#if defined(__x86_64__)
__attribute__((target("avx2,f16c"))) void sum_f16_f16c(uint16_t* d, const uint16_t* s, int64_t n,
                                                          int64_t* done) {
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    __m256 a = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(d + i)));
    __m256 b = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(s + i)));
    _mm_storeu_si128((__m128i*)(d + i), _mm256_cvtps_ph(_mm256_add_ps(a, b), _MM_FROUND_TO_NEAREST_INT));
  }
  *done = i;
}
#endif

template <typename T>
void sum_plain(T* d, const T* s, int64_t n) {
  for (int64_t i = 0; i < n; ++i) d[i] += s[i];
}

}  // namespace

void ring_reduce_sum(void* dst, const void* src, int64_t n, int dtype) {
  switch (dtype) {
    case kF32: sum_plain((float*)dst, (const float*)src, n); return;
    case kF64: sum_plain((double*)dst, (const double*)src, n); return;
    case kI32: sum_plain((int32_t*)dst, (const int32_t*)src, n); return;
    case kI64: sum_plain((int64_t*)dst, (const int64_t*)src, n); return;
    case kU8: sum_plain((uint8_t*)dst, (const uint8_t*)src, n); return;
    case kI8: sum_plain((int8_t*)dst, (const int8_t*)src, n); return;
    case kBF16: {
      uint16_t* d = (uint16_t*)dst;
      const uint16_t* s = (const uint16_t*)src;
      for (int64_t i = 0; i < n; ++i) d[i] = f32_to_bf16(bf16_to_f32(d[i]) + bf16_to_f32(s[i]));
      return;
    }
    case kF16: {
      uint16_t* d = (uint16_t*)dst;
      const uint16_t* s = (const uint16_t*)src;
      int64_t i = 0;
#if defined(__x86_64__)
      static const bool f16c = __builtin_cpu_supports("f16c") && __builtin_cpu_supports("avx2");
      if (f16c) sum_f16_f16c(d, s, n, &i);
#endif
      for (; i < n; ++i) d[i] = f32_to_f16(f16_to_f32(d[i]) + f16_to_f32(s[i]));
      return;
    }
  }
  throw std::invalid_argument("mivod ring: unknown dtype");
}

static void scale_inplace(void* data, int64_t n, int dtype, double f) {
  switch (dtype) {
    case kF32: { float* p = (float*)data; for (int64_t i = 0; i < n; ++i) p[i] = (float)(p[i] * f); return; }
    case kF64: { double* p = (double*)data; for (int64_t i = 0; i < n; ++i) p[i] *= f; return; }
    case kBF16: { uint16_t* p = (uint16_t*)data; for (int64_t i = 0; i < n; ++i) p[i] = f32_to_bf16((float)(bf16_to_f32(p[i]) * f)); return; }
    case kF16: { uint16_t* p = (uint16_t*)data; for (int64_t i = 0; i < n; ++i) p[i] = f32_to_f16((float)(f16_to_f32(p[i]) * f)); return; }
    default: throw std::invalid_argument("mivod ring: average needs a floating dtype");
  }
}

// ---------------------------------------------------------------- sockets
Ring::Ring(int rank, int size, double timeout_s) : rank_(rank), size_(size), timeout_s_(timeout_s) {
  if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("mivod ring: bad rank/size");
}

Ring::~Ring() { close(); }

int Ring::listen() {
  int port = 0;
  lfd_ = tcp_listen("0.0.0.0", &port);
  return port;
}

static void set_nonblocking(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

void Ring::connect(const std::string& next_host, int next_port) {
  std::lock_guard<std::mutex> lk(mu_);
  if (size_ == 1) return;
  if (lfd_ < 0) throw std::logic_error("mivod ring: listen() before connect()");
  // The successor's listen socket exists before its address is published, so the
  // TCP handshake completes in its backlog: connect first, then accept — no
  // ordering deadlock even when successor == predecessor (2 ranks).
  next_fd_ = tcp_connect(next_host, next_port, timeout_s_);
  int32_t hello = rank_;
  if (::send(next_fd_, &hello, 4, MSG_NOSIGNAL) != 4)
    throw std::runtime_error("mivod ring: hello send failed");
  prev_fd_ = tcp_accept(lfd_, timeout_s_);
  int32_t got = -1;
  size_t have = 0;
  while (have < 4) {
    ssize_t r = ::recv(prev_fd_, (char*)&got + have, 4 - have, 0);
    if (r <= 0) throw std::runtime_error("mivod ring: hello recv failed");
    have += (size_t)r;
  }
  const int expect = (rank_ + size_ - 1) % size_;
  if (got != expect)
    throw std::runtime_error("mivod ring: predecessor is rank " + std::to_string(got) +
                             ", expected " + std::to_string(expect));
  close_fd(lfd_);
  lfd_ = -1;
  set_nonblocking(next_fd_);
  set_nonblocking(prev_fd_);
}

void Ring::close() {
  close_fd(next_fd_);
  close_fd(prev_fd_);
  close_fd(lfd_);
  next_fd_ = prev_fd_ = lfd_ = -1;
}

// Full-duplex exchange: push sbuf to the successor while pulling rbuf from the
// predecessor; poll() drives both so neither side can block the ring.
void Ring::sendrecv(const void* sbuf, size_t sbytes, void* rbuf, size_t rbytes) {
  const char* sp = (const char*)sbuf;
  char* rp = (char*)rbuf;
  size_t sent = 0, got = 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (sent < sbytes || got < rbytes) {
    pollfd fds[2];
    int nf = 0, si = -1, ri = -1;
    if (sent < sbytes) { fds[nf] = {next_fd_, POLLOUT, 0}; si = nf++; }
    if (got < rbytes) { fds[nf] = {prev_fd_, POLLIN, 0}; ri = nf++; }
    int pr = ::poll(fds, nf, 1000);
    if (pr < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("mivod ring: poll failed: ") + std::strerror(errno));
    }
    if (pr == 0) {
      double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s_)
        throw std::runtime_error("mivod ring: rank " + std::to_string(rank_) +
                                 " timed out in a ring step (a peer died or stalled)");
      continue;
    }
    if (si >= 0 && (fds[si].revents & (POLLOUT | POLLERR | POLLHUP))) {
      ssize_t w = ::send(next_fd_, sp + sent, sbytes - sent, MSG_NOSIGNAL);
      if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
        throw std::runtime_error(std::string("mivod ring: send failed: ") + std::strerror(errno));
      if (w > 0) { sent += (size_t)w; bytes_sent_ += w; }
    }
    if (ri >= 0 && (fds[ri].revents & (POLLIN | POLLERR | POLLHUP))) {
      ssize_t r = ::recv(prev_fd_, rp + got, rbytes - got, 0);
      if (r == 0) throw std::runtime_error("mivod ring: predecessor closed the connection");
      if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
        throw std::runtime_error(std::string("mivod ring: recv failed: ") + std::strerror(errno));
      if (r > 0) got += (size_t)r;
    }
  }
}

void Ring::send_all(const void* buf, size_t n) { sendrecv(buf, n, nullptr, 0); }
void Ring::recv_all(void* buf, size_t n) { sendrecv(nullptr, 0, buf, n); }

// ---------------------------------------------------------------- collectives
void Ring::allreduce(void* data, int64_t count, int dtype, bool average) {
  std::lock_guard<std::mutex> lk(mu_);
  const int es = ring_dtype_size(dtype);
  if (size_ > 1 && count > 0) {
    const int N = size_;
    std::vector<int64_t> off(N + 1);
    for (int i = 0; i <= N; ++i) off[i] = count * i / N;
    auto csz = [&](int c) { return off[c + 1] - off[c]; };
    int64_t maxc = 0;
    for (int c = 0; c < N; ++c) maxc = std::max(maxc, csz(c));
    if ((int64_t)tmp_.size() < maxc * es) tmp_.resize((size_t)(maxc * es));
    char* base = (char*)data;
    // reduce-scatter: after N-1 steps rank r owns the full sum of chunk (r+1) % N
    for (int s = 0; s < N - 1; ++s) {
      const int sc = ((rank_ - s) % N + N) % N;
      const int rc = ((rank_ - s - 1) % N + N) % N;
      sendrecv(base + off[sc] * es, (size_t)(csz(sc) * es), tmp_.data(), (size_t)(csz(rc) * es));
      ring_reduce_sum(base + off[rc] * es, tmp_.data(), csz(rc), dtype);
    }
    if (average) {
      const int own = (rank_ + 1) % N;
      scale_inplace(base + off[own] * es, csz(own), dtype, 1.0 / N);
    }
    // allgather of the reduced chunks
    for (int s = 0; s < N - 1; ++s) {
      const int sc = ((rank_ + 1 - s) % N + N) % N;
      const int rc = ((rank_ - s) % N + N) % N;
      sendrecv(base + off[sc] * es, (size_t)(csz(sc) * es), base + off[rc] * es,
               (size_t)(csz(rc) * es));
    }
  } else if (average && size_ == 1) {
    // x / 1: nothing to do
  }
}

void Ring::allgatherv(const void* in, void* out, const std::vector<int64_t>& bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  if ((int)bytes.size() != size_) throw std::invalid_argument("mivod ring: bytes per rank");
  const int N = size_;
  std::vector<int64_t> off(N + 1, 0);
  for (int i = 0; i < N; ++i) off[i + 1] = off[i] + bytes[i];
  char* o = (char*)out;
  if (bytes[rank_] > 0 && o + off[rank_] != in) std::memcpy(o + off[rank_], in, (size_t)bytes[rank_]);
  for (int s = 0; s < N - 1; ++s) {
    const int sb = ((rank_ - s) % N + N) % N;
    const int rb = ((rank_ - s - 1) % N + N) % N;
    sendrecv(o + off[sb], (size_t)bytes[sb], o + off[rb], (size_t)bytes[rb]);
  }
}

void Ring::broadcast(void* data, int64_t bytes, int root) {
  std::lock_guard<std::mutex> lk(mu_);
  if (size_ == 1 || bytes <= 0) return;
  if (root < 0 || root >= size_) throw std::invalid_argument("mivod ring: bad root");
  // pipelined chain root -> root+1 -> ... -> root-1, 1 MiB segments
  const int dist = ((rank_ - root) % size_ + size_) % size_;
  const bool last = dist == size_ - 1;
  const int64_t seg = 1 << 20;
  char* p = (char*)data;
  for (int64_t o = 0; o < bytes; o += seg) {
    const size_t n = (size_t)std::min<int64_t>(seg, bytes - o);
    if (dist != 0) recv_all(p + o, n);
    if (!last) send_all(p + o, n);
  }
}

void Ring::barrier() {
  int32_t one = 1;
  allreduce(&one, 1, kI32, false);
}

}  // namespace mvcore
