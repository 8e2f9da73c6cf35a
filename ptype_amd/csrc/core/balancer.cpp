#include "balancer.hpp"

namespace ptype {

ConnConfig default_conn_config() { return ConnConfig{}; }

int ConnectionBalancer::hash_index(const std::string& local_addr, int conn_number, int node_count) {
  // int(h.Sum32()) % nodeSize: Go's int is 64-bit, so the sum is non-negative
  return (int)((uint64_t)fnv1a32(local_addr + std::to_string(conn_number)) % (uint64_t)node_count);
}

std::vector<Node> ConnectionBalancer::select_nodes(const std::string& local_addr, const std::vector<Node>& nodes,
                                                   int max) {
  if ((int)nodes.size() <= max || max == 0) return nodes;
  std::vector<Node> out;
  out.reserve(max);
  for (int i = 0; (int)out.size() < max; ++i) out.push_back(nodes[hash_index(local_addr, i, (int)nodes.size())]);
  return out;
}

ConnectionBalancer::ConnectionBalancer(std::string local_addr, std::string service, std::shared_ptr<NodesChan> nodes,
                                       ConnConfig cfg, Dialer dialer)
    : local_addr_(std::move(local_addr)),
      service_(std::move(service)),
      nodes_(std::move(nodes)),
      cfg_(cfg),
      dialer_(std::move(dialer)),
      errs_(std::make_shared<Channel<std::string>>(1)),
      updated_(std::make_shared<Channel<int>>(5)) {
  if (!dialer_)
    dialer_ = [](const Node& n, const ConnConfig& c) {
      return dial_node(n.address, n.port, c.dial_timeout_ms, c.allow_local);
    };
  if (!nodes_) return;  // bare balancer (test hook)
  bool closed = false;
  auto initial = nodes_->recv(cfg_.initial_node_timeout_ms, &closed);
  if (!initial) fail(Errc::kGeneric, "no initial nodes provided for " + service_);
  handle_new_nodes(*initial);
  updated_->recv(0);  // consume the first update message (rpc.go:165)
  th_ = std::thread([this] { watch_loop(); });
}

ConnectionBalancer::~ConnectionBalancer() { close(); }

void ConnectionBalancer::close() {
  if (stop_.exchange(true)) return;
  if (th_.joinable()) th_.join();
  std::vector<std::shared_ptr<RpcConn>> cs;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs.swap(clients_);
    for (auto& r : retired_) cs.push_back(std::move(r));
    retired_.clear();
  }
  for (auto& c : cs) c->close();
  errs_->close();
}

std::shared_ptr<RpcConn> ConnectionBalancer::get() {
  std::vector<std::shared_ptr<RpcConn>> cs;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs = clients_;
  }
  if (cs.empty()) return nullptr;
  const uint64_t idx = ++seq_;
  return cs[idx % cs.size()];
}

std::vector<Node> ConnectionBalancer::selected_nodes() {
  std::lock_guard<std::mutex> g(mu_);
  return selected_;
}

size_t ConnectionBalancer::client_count() {
  std::lock_guard<std::mutex> g(mu_);
  return clients_.size();
}

void ConnectionBalancer::set_clients_for_test(std::vector<std::shared_ptr<RpcConn>> clients) {
  std::lock_guard<std::mutex> g(mu_);
  clients_ = std::move(clients);
}

void ConnectionBalancer::handle_new_nodes(const std::vector<Node>& nodes) {
  std::vector<Node> sel = select_nodes(local_addr_, nodes, cfg_.max_connections);
  // connections to nodes that stay selected are kept (their in-flight calls go on);
  // only newly selected nodes are dialled -- the reference re-dials every node and
  // keeps the old clients open (rpc.go:226-236)
  std::vector<std::pair<Node, std::shared_ptr<RpcConn>>> have;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < selected_.size() && i < clients_.size(); ++i) have.emplace_back(selected_[i], clients_[i]);
  }
  auto find = [](const std::vector<std::pair<Node, std::shared_ptr<RpcConn>>>& v, const Node& n) {
    for (const auto& e : v)
      if (e.first == n) return e.second;
    return std::shared_ptr<RpcConn>();
  };
  std::vector<std::pair<Node, std::shared_ptr<RpcConn>>> dialled;
  std::vector<std::shared_ptr<RpcConn>> fresh;
  fresh.reserve(sel.size());
  for (const auto& n : sel) {
    std::shared_ptr<RpcConn> c = find(have, n);
    if (!c) c = find(dialled, n);  // a duplicate pick shares its connection
    if (!c) {
      try {
        c = dialer_(n, cfg_);
      } catch (const Error& e) {
        for (auto& d : dialled) d.second->close();
        fail(Errc::kUnavailable, e.what());
      }
      dialled.emplace_back(n, c);
    }
    fresh.push_back(c);
  }
  std::vector<std::shared_ptr<RpcConn>> old;
  {
    std::lock_guard<std::mutex> g(mu_);
    old.swap(clients_);
    clients_ = std::move(fresh);
    selected_ = sel;
    // connections no longer selected close once no call holds them (see reap_retired)
    for (auto& c : old) {
      bool kept = false;
      for (auto& k : clients_) kept = kept || k == c;
      bool queued = false;
      for (auto& r : retired_) queued = queued || r == c;
      if (!kept && !queued) retired_.push_back(c);
    }
  }
  old.clear();
  reap_retired();
  updated_->try_send(1);
}

// A retired connection is closed when the balancer's reference is the only one
// left: every call holds the connection it was handed by get() until it returns.
void ConnectionBalancer::reap_retired() {
  std::vector<std::shared_ptr<RpcConn>> idle;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = retired_.begin(); it != retired_.end();) {
      if (it->use_count() == 1) {
        idle.push_back(std::move(*it));
        it = retired_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& c : idle) c->close();
}

size_t ConnectionBalancer::retired_count() {
  std::lock_guard<std::mutex> g(mu_);
  return retired_.size();
}

void ConnectionBalancer::watch_loop() {
  std::vector<Node> pending;
  bool have = false;
  int64_t deadline = mono_ms() + cfg_.debounce_ms;
  while (!stop_.load()) {
    reap_retired();
    const int64_t left = deadline - mono_ms();
    if (left <= 0) {
      if (have) {
        try {
          handle_new_nodes(pending);
        } catch (const Error& e) {
          errs_->try_send(e.what());
        }
        have = false;
      }
      deadline = mono_ms() + cfg_.debounce_ms;
      continue;
    }
    bool closed = false;
    auto v = nodes_->recv(std::min<int64_t>(left, 50), &closed);
    if (v) {
      deadline = mono_ms() + cfg_.debounce_ms;  // every message re-arms time.After
      if (v->empty()) continue;                 // empty lists are ignored
      pending = std::move(*v);
      have = true;
    } else if (closed) {
      // registry watch ended; flush what we have, then stop
      if (have && !stop_.load()) {
        const int64_t rest = deadline - mono_ms();
        if (rest > 0) sleep_ms(rest);
        try {
          handle_new_nodes(pending);
        } catch (const Error& e) {
          errs_->try_send(e.what());
        }
      }
      return;
    }
  }
}

// ---------------------------------------------------------------- client
RpcClient::RpcClient(std::string local_addr, std::string service, std::shared_ptr<NodesChan> nodes, ConnConfig cfg,
                     Dialer dialer)
    : cfg_(cfg),
      bal_(new ConnectionBalancer(std::move(local_addr), std::move(service), std::move(nodes), cfg,
                                  std::move(dialer))) {}

RpcClient::~RpcClient() { close(); }

void RpcClient::close() {
  {
    std::lock_guard<std::mutex> g(gmu_);
    if (closed_.exchange(true)) return;
  }
  while (active_.load() > 0) sleep_ms(1);
  if (on_close) on_close();
  bal_->close();
}

RpcOutcome RpcClient::attempt(const std::string& method, const gob::Value& args) {
  ++attempts_;
  auto c = bal_->get();
  if (!c) {
    RpcOutcome o;
    o.error = "no client nodes available";
    o.code = Errc::kNoClientAvailable;
    return o;
  }
  return c->call(method, args);
}

gob::Value RpcClient::call(const std::string& method, const gob::Value& args) {
  ++calls_;
  RpcOutcome o;
  for (int a = 0; a <= std::max(0, cfg_.retries); ++a) {
    o = attempt(method, args);
    if (o.ok()) return o.reply;
  }
  fail(o.code, o.error);
}

std::shared_ptr<RpcCall> RpcClient::go(const std::string& method, const gob::Value& args,
                                       std::shared_ptr<Channel<std::shared_ptr<RpcCall>>> done) {
  ++calls_;
  auto call = std::make_shared<RpcCall>();
  call->method = method;
  call->args = args;
  call->done = done ? done : std::make_shared<Channel<std::shared_ptr<RpcCall>>>(10);
  std::lock_guard<std::mutex> g(gmu_);
  if (closed_.load()) {
    call->error = "connection is shut down";
    call->code = Errc::kShutdown;
    call->done->try_send(call);
    return call;
  }
  ++active_;
  std::thread([this, call] {  // a goroutine; close() waits for every one
    RpcOutcome o;
    for (int a = 0; a <= std::max(0, cfg_.retries); ++a) {
      o = attempt(call->method, call->args);
      if (o.ok()) break;
    }
    if (o.ok())
      call->reply = std::move(o.reply);
    else {
      call->error = o.error;
      call->code = o.code;
    }
    call->done->send(call);
    --active_;
  }).detach();
  return call;
}

}  // namespace ptype
