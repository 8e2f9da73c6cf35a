// TCP transport for the control plane (SURVEY C7 peer transport + client API):
// length-prefixed frames over plain sockets.  Raft deliberately does NOT go over
// RCCL -- collectives hang on a dead peer, consensus must tolerate one.
#pragma once
#include <stdint.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ptype {

// Frame kinds of the control-plane protocol.
enum FrameKind : uint8_t { kFrameReq = 1, kFrameResp = 2, kFrameEvent = 3, kFrameRaft = 4 };

class Conn {
 public:
  explicit Conn(int fd);
  ~Conn();
  bool send(const std::string& payload);      // thread-safe; false when broken
  bool recv(std::string* payload);            // one frame; false on EOF / error
  // raw byte-stream access (Go net/rpc over HTTP CONNECT is not framed)
  bool write_raw(const std::string& bytes);   // thread-safe
  bool read_exact(char* p, size_t n);         // buffered
  bool read_line(std::string* line);          // up to and excluding '\n'
  // Whether more input is available right now (buffered, or readable without blocking).
  bool input_pending();
  void shutdown();
  bool alive() const { return alive_.load(); }
  int fd() const { return fd_; }
  std::string peer() const;

 private:
  bool fill();
  int fd_;
  std::atomic<bool> alive_{true};
  std::mutex wmu_;
  std::string rbuf_;
  size_t rpos_ = 0;
};

// Connect to host:port (ms timeout); nullptr on failure (errno-style message in *err).
std::shared_ptr<Conn> tcp_connect(const std::string& host, int port, int64_t timeout_ms, std::string* err);

class Listener {
 public:
  // Binds host:port (port 0 = ephemeral) and serves each accepted connection on
  // its own thread with `handler`.
  Listener(const std::string& host, int port, std::function<void(std::shared_ptr<Conn>)> handler);
  ~Listener();
  int port() const { return port_; }
  void close();

 private:
  void loop();
  int fd_ = -1;
  int port_ = 0;
  std::function<void(std::shared_ptr<Conn>)> handler_;
  std::atomic<bool> stop_{false};
  std::thread th_;
  std::mutex mu_;
  std::vector<std::weak_ptr<Conn>> conns_;
  std::vector<std::thread> workers_;
};

std::string resolve_host(const std::string& host);  // "localhost" -> 127.0.0.1
std::string first_nonloopback_ipv4();               // "" if none (cluster/cluster.go:198-213)

}  // namespace ptype
