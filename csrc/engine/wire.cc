// mivod control-plane wire encoding + blocking TCP socket helpers.
#include "wire.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <thread>

namespace mvcore {

void encode_requests(Writer& w, const std::vector<Request>& rs, bool shutdown) {
  w.u8(shutdown ? 1 : 0);
  w.u32((uint32_t)rs.size());
  for (const auto& r : rs) {
    w.str(r.name);
    w.u8(r.kind);
    w.str(r.dtype);
    w.u32((uint32_t)r.shape.size());
    for (auto d : r.shape) w.i64(d);
    w.i32(r.root);
    w.i32(r.op);
    w.i32(r.device);
    w.i64(r.nbytes);
    w.f64(r.prescale);
    w.f64(r.postscale);
  }
}

std::vector<Request> decode_requests(Reader& rd, bool* shutdown) {
  *shutdown = rd.u8() != 0;
  uint32_t n = rd.u32();
  std::vector<Request> rs(n);
  for (auto& r : rs) {
    r.name = rd.str();
    r.kind = rd.u8();
    r.dtype = rd.str();
    uint32_t nd = rd.u32();
    r.shape.resize(nd);
    for (auto& d : r.shape) d = rd.i64();
    r.root = rd.i32();
    r.op = rd.i32();
    r.device = rd.i32();
    r.nbytes = rd.i64();
    r.prescale = rd.f64();
    r.postscale = rd.f64();
  }
  return rs;
}

void encode_responses(Writer& w, const std::vector<Response>& rs, bool shutdown) {
  w.u8(shutdown ? 1 : 0);
  w.u32((uint32_t)rs.size());
  for (const auto& r : rs) {
    w.u8(r.kind);
    w.str(r.error);
    w.u32((uint32_t)r.names.size());
    for (const auto& n : r.names) w.str(n);
  }
}

std::vector<Response> decode_responses(Reader& rd, bool* shutdown) {
  *shutdown = rd.u8() != 0;
  uint32_t n = rd.u32();
  std::vector<Response> rs(n);
  for (auto& r : rs) {
    r.kind = rd.u8();
    r.error = rd.str();
    uint32_t k = rd.u32();
    r.names.resize(k);
    for (auto& s : r.names) s = rd.str();
  }
  return rs;
}

static void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int tcp_listen(const std::string& host, int* port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw std::runtime_error("mivod: socket() failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)*port);
  if (host.empty() || host == "0.0.0.0") {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  }
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    throw std::runtime_error("mivod: bind() failed: " + std::string(strerror(errno)));
  }
  if (listen(fd, 1024) != 0) {
    close(fd);
    throw std::runtime_error("mivod: listen() failed");
  }
  socklen_t len = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &len);
  *port = ntohs(a.sin_port);
  return fd;
}

int tcp_accept(int lfd, double timeout_s) {
  pollfd p{lfd, POLLIN, 0};
  int ms = timeout_s < 0 ? -1 : (int)(timeout_s * 1000);
  int r = poll(&p, 1, ms);
  if (r <= 0) throw std::runtime_error("mivod: timed out waiting for a rank to connect");
  int fd = accept(lfd, nullptr, nullptr);
  if (fd < 0) throw std::runtime_error("mivod: accept() failed");
  set_nodelay(fd);
  return fd;
}

int tcp_connect(const std::string& host, int port, double timeout_s) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    std::string ps = std::to_string(port);
    if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) == 0 && res) {
      int fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        set_nodelay(fd);
        return fd;
      }
      if (fd >= 0) close(fd);
      freeaddrinfo(res);
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("mivod: could not connect to coordinator " + host + ":" + ps);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

static void write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("mivod: peer connection lost (send)");
    }
    p += k;
    n -= (size_t)k;
  }
}

static void read_all(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) throw std::runtime_error("mivod: peer connection closed");
    if (k < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("mivod: peer connection lost (recv)");
    }
    p += k;
    n -= (size_t)k;
  }
}

void send_msg(int fd, const std::string& payload) {
  uint32_t n = (uint32_t)payload.size();
  std::string b(reinterpret_cast<const char*>(&n), 4);
  b += payload;
  write_all(fd, b.data(), b.size());
}

std::string recv_msg(int fd) {
  uint32_t n = 0;
  read_all(fd, reinterpret_cast<char*>(&n), 4);
  std::string s(n, '\0');
  if (n) read_all(fd, &s[0], n);
  return s;
}

void close_fd(int fd) {
  if (fd >= 0) ::close(fd);
}

}  // namespace mvcore
