// RPC client + connection balancer (reference cluster/rpc.go).
//
// Reproduced semantics:
//   * node selection: all nodes if len <= MaxConnections or MaxConnections == 0,
//     else nodes[FNV-1a32(localAddr + itoa(i)) % n] for i = 0,1,.. until
//     MaxConnections picks, duplicates allowed (rpc.go:246-270);
//   * round robin: atomic ++seq then clients[seq % len] -- the first call goes
//     to index 1 (rpc.go:176-183);
//   * trailing-edge debounce of registry updates, empty lists ignored, any
//     message re-arms the timer (rpc.go:197-224);
//   * initial list awaited for InitialNodeTimeout, error "no initial nodes
//     provided for <svc>"; any dial failure fails construction (rpc.go:141-170).
// Documented fixes: at most 1 + Retries attempts, each
// re-selected round robin (the reference's `retries := 0` inside the loop
// retries forever); `Go` delivers the final error (the reference tests the
// outer call's nil error and never retries); a re-balance keeps the connections
// of nodes that stay selected and closes a deselected one only once no call
// holds it (the reference leaks them); Close takes the lock; a closed registry
// channel stops the watcher instead of spinning.
#pragma once
#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "netrpc.hpp"
#include "util.hpp"

namespace ptype {

struct Node {
  std::string address;
  int64_t port = 0;
  bool operator==(const Node& o) const { return address == o.address && port == o.port; }
};
using NodesChan = Channel<std::vector<Node>>;

struct ConnConfig {
  int max_connections = 3;
  int64_t initial_node_timeout_ms = 5000;
  int64_t debounce_ms = 3000;
  int retries = 2;
  bool allow_local = true;  // in-process fast path to servers of this process
  int64_t dial_timeout_ms = 5000;
};
ConnConfig default_conn_config();  // {3, 5s, 3s, 2} (rpc.go:33-38)

// Dial hook (tests inject failures); default = dial_node().
using Dialer = std::function<std::shared_ptr<RpcConn>(const Node&, const ConnConfig&)>;

class ConnectionBalancer {
 public:
  ConnectionBalancer(std::string local_addr, std::string service, std::shared_ptr<NodesChan> nodes, ConnConfig cfg,
                     Dialer dialer = nullptr);
  ~ConnectionBalancer();
  std::shared_ptr<RpcConn> get();  // round robin; nullptr when no clients
  std::vector<Node> selected_nodes();
  size_t client_count();
  std::shared_ptr<Channel<std::string>> errs() { return errs_; }          // cap 1, non-blocking sends
  std::shared_ptr<Channel<int>> conns_updated() { return updated_; }      // cap 5 (test hook)
  void close();
  const ConnConfig& config() const { return cfg_; }

  static std::vector<Node> select_nodes(const std::string& local_addr, const std::vector<Node>& nodes, int max);
  static int hash_index(const std::string& local_addr, int conn_number, int node_count);
  // test hook mirroring rpc_test.go:390-425 (clients set directly)
  void set_clients_for_test(std::vector<std::shared_ptr<RpcConn>> clients);
  size_t retired_count();  // deselected connections still serving in-flight calls

 private:
  void handle_new_nodes(const std::vector<Node>& nodes);  // throws on dial failure
  void watch_loop();
  void reap_retired();

  std::string local_addr_, service_;
  std::shared_ptr<NodesChan> nodes_;
  ConnConfig cfg_;
  Dialer dialer_;
  std::atomic<uint64_t> seq_{0};
  std::mutex mu_;
  std::vector<Node> selected_;
  std::vector<std::shared_ptr<RpcConn>> clients_;
  std::vector<std::shared_ptr<RpcConn>> retired_;  // deselected, closed when no call holds them
  std::shared_ptr<Channel<std::string>> errs_;
  std::shared_ptr<Channel<int>> updated_;
  std::atomic<bool> stop_{false};
  std::thread th_;
};

// A call handle for Client.Go (net/rpc's *rpc.Call): completion is delivered on
// `done` (cap 10, rpc.go:70-73) carrying this same handle.
struct RpcCall {
  std::string method;
  gob::Value args, reply;
  std::string error;
  Errc code = Errc::kGeneric;
  std::shared_ptr<Channel<std::shared_ptr<RpcCall>>> done;
};

class RpcClient {
 public:
  RpcClient(std::string local_addr, std::string service, std::shared_ptr<NodesChan> nodes, ConnConfig cfg,
            Dialer dialer = nullptr);
  ~RpcClient();
  // Call (rpc.go:59-67): returns the reply, throws Error(kRpc|kNoClientAvailable|...) on failure.
  gob::Value call(const std::string& method, const gob::Value& args);
  // Go (rpc.go:69-105): asynchronous; the returned handle is later sent on `done`.
  std::shared_ptr<RpcCall> go(const std::string& method, const gob::Value& args,
                              std::shared_ptr<Channel<std::shared_ptr<RpcCall>>> done = nullptr);
  void close();
  std::shared_ptr<Channel<std::string>> connection_errs() { return bal_->errs(); }
  ConnectionBalancer& balancer() { return *bal_; }
  const ConnConfig& config() const { return cfg_; }
  uint64_t calls() const { return calls_.load(); }
  uint64_t attempts() const { return attempts_.load(); }
  std::function<void()> on_close;  // e.g. cancels the registry watch feeding the balancer

 private:
  RpcOutcome attempt(const std::string& method, const gob::Value& args);
  ConnConfig cfg_;
  std::unique_ptr<ConnectionBalancer> bal_;
  std::atomic<uint64_t> calls_{0}, attempts_{0};
  std::mutex gmu_;
  std::atomic<int> active_{0};
  std::atomic<bool> closed_{false};
};

}  // namespace ptype
