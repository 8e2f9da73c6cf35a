#include "net.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "util.hpp"

namespace ptype {

static bool write_all_fd(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

static bool read_full_fd(int fd, char* p, size_t n) {
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

Conn::Conn(int fd) : fd_(fd) {
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

Conn::~Conn() {
  shutdown();
  ::close(fd_);
}

bool Conn::send(const std::string& payload) {
  if (!alive_.load()) return false;
  std::lock_guard<std::mutex> g(wmu_);
  uint32_t len = (uint32_t)payload.size();
  std::string buf;
  buf.reserve(4 + payload.size());
  buf.append((const char*)&len, 4);
  buf += payload;
  if (!write_all_fd(fd_, buf.data(), buf.size())) {
    alive_.store(false);
    return false;
  }
  return true;
}

bool Conn::recv(std::string* payload) {
  uint32_t len;
  if (!read_full_fd(fd_, (char*)&len, 4)) {
    alive_.store(false);
    return false;
  }
  if (len > (1u << 30)) {
    alive_.store(false);
    return false;
  }
  payload->resize(len);
  if (len && !read_full_fd(fd_, &(*payload)[0], len)) {
    alive_.store(false);
    return false;
  }
  return true;
}

bool Conn::write_raw(const std::string& bytes) {
  if (!alive_.load()) return false;
  std::lock_guard<std::mutex> g(wmu_);
  if (!write_all_fd(fd_, bytes.data(), bytes.size())) {
    alive_.store(false);
    return false;
  }
  return true;
}

bool Conn::fill() {
  if (rpos_ > 0 && rpos_ == rbuf_.size()) {
    rbuf_.clear();
    rpos_ = 0;
  }
  char tmp[16384];
  for (;;) {
    ssize_t k = ::recv(fd_, tmp, sizeof tmp, 0);
    if (k > 0) {
      rbuf_.append(tmp, (size_t)k);
      return true;
    }
    if (k < 0 && errno == EINTR) continue;
    alive_.store(false);
    return false;
  }
}

bool Conn::input_pending() {
  if (rbuf_.size() > rpos_) return true;
  pollfd pfd{fd_, POLLIN, 0};
  return ::poll(&pfd, 1, 0) > 0 && (pfd.revents & POLLIN);
}

bool Conn::read_exact(char* p, size_t n) {
  while (rbuf_.size() - rpos_ < n)
    if (!fill()) return false;
  memcpy(p, rbuf_.data() + rpos_, n);
  rpos_ += n;
  return true;
}

bool Conn::read_line(std::string* line) {
  for (;;) {
    const size_t nl = rbuf_.find('\n', rpos_);
    if (nl != std::string::npos) {
      *line = rbuf_.substr(rpos_, nl - rpos_);
      rpos_ = nl + 1;
      if (!line->empty() && line->back() == '\r') line->pop_back();
      return true;
    }
    if (rbuf_.size() - rpos_ > 65536 || !fill()) return false;
  }
}

void Conn::shutdown() {
  if (alive_.exchange(false)) ::shutdown(fd_, SHUT_RDWR);
}

std::string Conn::peer() const {
  sockaddr_in a{};
  socklen_t l = sizeof a;
  if (getpeername(fd_, (sockaddr*)&a, &l) != 0) return "";
  char b[64];
  inet_ntop(AF_INET, &a.sin_addr, b, sizeof b);
  return std::string(b) + ":" + std::to_string(ntohs(a.sin_port));
}

std::string resolve_host(const std::string& host) {
  if (host == "localhost" || host.empty()) return "127.0.0.1";
  return host;
}

std::shared_ptr<Conn> tcp_connect(const std::string& host0, int port, int64_t timeout_ms, std::string* err) {
  const std::string host = resolve_host(host0);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    if (err) *err = "dial tcp " + host0 + ":" + std::to_string(port) + ": lookup failed";
    return nullptr;
  }
  int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    freeaddrinfo(res);
    if (err) *err = strerror(errno);
    return nullptr;
  }
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    if (err) *err = "dial tcp " + host0 + ":" + std::to_string(port) + ": connect: " + strerror(errno);
    ::close(fd);
    return nullptr;
  }
  if (rc != 0) {
    pollfd p{fd, POLLOUT, 0};
    int pr = poll(&p, 1, (int)timeout_ms);
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
    if (pr <= 0 || soerr != 0) {
      if (err)
        *err = "dial tcp " + host0 + ":" + std::to_string(port) + ": connect: " +
               (pr <= 0 ? std::string("i/o timeout") : std::string(strerror(soerr)));
      ::close(fd);
      return nullptr;
    }
  }
  fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
  return std::make_shared<Conn>(fd);
}

Listener::Listener(const std::string& host0, int port, std::function<void(std::shared_ptr<Conn>)> handler)
    : handler_(std::move(handler)) {
  const std::string host = resolve_host(host0);
  fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd_ < 0) fail(Errc::kUnavailable, std::string("socket: ") + strerror(errno));
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host == "0.0.0.0" || host == "::") {
    a.sin_addr.s_addr = INADDR_ANY;
  } else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(fd_);
    fail(Errc::kUnavailable, "listen tcp " + host0 + ":" + std::to_string(port) + ": bad address");
  }
  if (::bind(fd_, (sockaddr*)&a, sizeof a) != 0 || ::listen(fd_, 128) != 0) {
    std::string e = strerror(errno);
    ::close(fd_);
    fail(Errc::kUnavailable, "listen tcp " + host0 + ":" + std::to_string(port) + ": bind: " + e);
  }
  socklen_t l = sizeof a;
  getsockname(fd_, (sockaddr*)&a, &l);
  port_ = ntohs(a.sin_port);
  th_ = std::thread([this] { loop(); });
}

Listener::~Listener() { close(); }

void Listener::loop() {
  while (!stop_.load()) {
    pollfd p{fd_, POLLIN, 0};
    int pr = poll(&p, 1, 100);
    if (pr <= 0) continue;
    int c = ::accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (c < 0) continue;
    auto conn = std::make_shared<Conn>(c);
    std::lock_guard<std::mutex> g(mu_);
    if (stop_.load()) break;
    conns_.push_back(conn);
    workers_.emplace_back([this, conn] { handler_(conn); });
  }
}

void Listener::close() {
  if (stop_.exchange(true)) return;
  if (th_.joinable()) th_.join();
  std::vector<std::thread> ws;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& w : conns_)
      if (auto c = w.lock()) c->shutdown();
    ws.swap(workers_);
  }
  for (auto& t : ws)
    if (t.joinable()) t.join();
  ::close(fd_);
}

std::string first_nonloopback_ipv4() {
  ifaddrs* ifs = nullptr;
  if (getifaddrs(&ifs) != 0) return "";
  std::string out;
  for (ifaddrs* i = ifs; i; i = i->ifa_next) {
    if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET) continue;
    auto* sa = (sockaddr_in*)i->ifa_addr;
    const uint32_t ip = ntohl(sa->sin_addr.s_addr);
    if ((ip >> 24) == 127) continue;
    char b[64];
    inet_ntop(AF_INET, &sa->sin_addr, b, sizeof b);
    out = b;
    break;
  }
  freeifaddrs(ifs);
  return out;
}

}  // namespace ptype
