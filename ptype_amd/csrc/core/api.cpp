#include "api.hpp"

#include <algorithm>
#include <cstdlib>

#include "json.hpp"

namespace ptype {

const char* kServicesPrefix = "services";
const char* kStorePrefix = "store";

std::string etcd_key(const std::vector<std::string>& elems) { return path_join(elems) + "/"; }

std::string node_json(const Node& n) {
  JValue v;
  v.kind = JValue::kObject;
  v.obj.emplace_back("address", JValue::string(n.address));
  v.obj.emplace_back("port", JValue::integer(n.port));
  return json_dump(v);
}

Node node_from_json(const std::string& s) {
  JValue v = json_parse(s);
  if (v.kind != JValue::kObject) fail("json: cannot unmarshal " + s + " into Go value of type cluster.Node");
  Node n;
  if (const JValue* a = v.get("address")) {
    if (a->kind != JValue::kString) fail("json: cannot unmarshal into Go struct field Node.address of type string");
    n.address = a->str;
  }
  if (const JValue* p = v.get("port")) {
    if (p->kind != JValue::kNumber || !p->is_int) fail("json: cannot unmarshal into Go struct field Node.port of type int");
    n.port = p->i;
  }
  return n;
}

static void check_ctx(const Ctx& ctx) {
  if (ctx && ctx->done()) fail(Errc::kCanceled, ctx->err());
}

// ---------------------------------------------------------------- registry
EtcdRegistry::~EtcdRegistry() { close(); }

void EtcdRegistry::close() {
  if (closed_.exchange(true)) return;
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> g(mu_);
    ts.swap(threads_);
  }
  cli_->close();  // unblocks keepalive/watch helpers
  for (auto& t : ts)
    if (t.joinable()) t.join();
}

void EtcdRegistry::register_node(const Ctx& ctx, const std::string& service, const std::string& node,
                                 const std::string& host, int64_t port) {
  check_ctx(ctx);
  const std::string val = node_json(Node{host, port});
  int64_t ttl = 0, lease;
  try {
    lease = cli_->grant(2, &ttl);  // 2 s TTL (cluster/registry.go:59)
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to create lease for service: ") + e.what());
  }
  const std::string key = etcd_key({kServicesPrefix, service, node});
  try {
    cli_->put(key, val, lease);
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to register node: ") + e.what());
  }
  std::shared_ptr<Channel<int64_t>> ka;
  try {
    ka = cli_->keepalive(ctx, lease);
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to keep service registered: ") + e.what());
  }
  std::lock_guard<std::mutex> g(mu_);
  threads_.emplace_back([ka, service] {
    for (;;) {
      auto v = ka->recv(-1);
      if (!v) {
        log_warn("service failed to refresh", {{"service", service}});
        break;
      }
      log_info("service ttl refreshed", {{"service", service}, {"ttl", std::to_string(*v)}});
    }
  });
}

static RangeOpts prefix_sorted(const std::string& key) {
  RangeOpts o;  // defaultGetOptions: WithPrefix + WithSort(Key, Ascend) (cluster/registry.go:88-91)
  o.end = key.empty() ? std::string(1, '\0') : prefix_range_end(key);
  o.sort_target = kSortKey;
  o.sort_order = kSortNone;  // clientv3 turns (Key, Ascend) into the natural order
  return o;
}

std::map<std::string, std::vector<Node>> EtcdRegistry::services(const Ctx& ctx) {
  check_ctx(ctx);
  RangeResult res;
  try {
    res = cli_->get(kServicesPrefix, prefix_sorted(kServicesPrefix));
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to get services from etcd: ") + e.what());
  }
  std::map<std::string, std::vector<Node>> out;
  for (const auto& kv : res.kvs) {
    Node n;
    try {
      n = node_from_json(kv.value);
    } catch (const Error& e) {
      fail(std::string("failed to unmarshal services nodes: ") + e.what());
    }
    const auto parts = split(kv.key, '/');
    if (parts.size() > 1) out[parts[1]].push_back(n);
  }
  return out;
}

std::vector<Node> EtcdRegistry::nodes(const Ctx& ctx, const std::string& service) {
  check_ctx(ctx);
  const std::string key = etcd_key({kServicesPrefix, service});
  RangeResult res;
  try {
    res = cli_->get(key, prefix_sorted(key));
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to get services from etcd: ") + e.what());
  }
  std::vector<Node> out;
  for (const auto& kv : res.kvs) {
    try {
      out.push_back(node_from_json(kv.value));
    } catch (const Error& e) {
      fail(std::string("failed to unmarshal services nodes: ") + e.what());
    }
  }
  return out;
}

std::shared_ptr<NodesChan> EtcdRegistry::watch_service(const Ctx& ctx, const std::string& service) {
  const std::string key = etcd_key({kServicesPrefix, service});
  auto out = std::make_shared<NodesChan>(0);  // unbuffered, like the reference
  std::shared_ptr<Channel<WatchResponse>> wch;
  try {
    wch = cli_->watch(ctx, key, prefix_range_end(key));
  } catch (const Error&) {
    out->close();  // the reference closes the channel when the watch fails
    return out;
  }
  std::lock_guard<std::mutex> g(mu_);
  threads_.emplace_back([this, ctx, service, out, wch] {
    for (;;) {
      if (closed_.load() || (ctx && ctx->done())) break;
      std::vector<Node> ns;
      try {
        ns = nodes(ctx, service);
      } catch (const Error&) {
        log_error("failed to get nodes for service", {{"service", service}});
        // the reference re-lists immediately (a hot spin); back off briefly instead
        if (ctx && ctx->wait(100)) break;
        continue;
      }
      if (!out->send(ns, ctx)) break;  // ctx-aware (the reference's send is unguarded)
      bool next = false;
      while (!next) {
        if (closed_.load() || (ctx && ctx->done())) goto done;
        bool closed = false;
        auto r = wch->recv(50, &closed);
        if (r) {
          if (!r->err.empty()) goto done;  // res.Err() != nil
          next = true;
        } else if (closed) {
          goto done;
        }
      }
    }
  done:
    out->close();
  });
  return out;
}

// ---------------------------------------------------------------- store
RangeOpts resolve_opts(std::string* key, const std::vector<OpOption>& opts) {
  RangeOpts o;
  for (const auto& op : opts) {
    switch (op.kind) {
      case OpOption::kPrefix:
        if (key->empty()) {
          *key = std::string(1, '\0');
          o.end = std::string(1, '\0');
        } else {
          o.end = prefix_range_end(*key);
        }
        break;
      case OpOption::kLimit: o.limit = op.n; break;
      case OpOption::kRev: o.rev = op.n; break;
      case OpOption::kRange: o.end = op.s; break;
      case OpOption::kFromKey:
        if (key->empty()) *key = std::string(1, '\0');
        o.end = std::string(1, '\0');
        break;
      case OpOption::kSerializable: o.serializable = true; break;
      case OpOption::kKeysOnly: o.keys_only = true; break;
      case OpOption::kCountOnly: o.count_only = true; break;
      case OpOption::kSort:
        o.sort_target = op.target;
        o.sort_order = (op.target == kSortKey && op.order == kSortAscend) ? kSortNone : op.order;
        break;
      case OpOption::kLease:
        break;
    }
  }
  return o;
}

std::vector<std::string> KVStore::get(const Ctx& ctx, const std::string& key, const std::vector<OpOption>& opts) {
  check_ctx(ctx);
  std::string k = path_join({kStorePrefix, key});
  RangeOpts o = resolve_opts(&k, opts);
  RangeResult res;
  try {
    res = cli_->get(k, o);
  } catch (const Error& e) {
    fail(e.code(), "failed to get key " + key + ": " + e.what());
  }
  if (res.kvs.empty()) fail(Errc::kNoKey, "Key could not be found");
  std::vector<std::string> out;
  for (const auto& kv : res.kvs) out.push_back(kv.value);
  return out;
}

void KVStore::put(const Ctx& ctx, const std::string& key, const std::string& value,
                  const std::vector<OpOption>& opts) {
  check_ctx(ctx);
  int64_t lease = 0;
  for (const auto& op : opts)
    if (op.kind == OpOption::kLease) lease = op.n;
  try {
    cli_->put(path_join({kStorePrefix, key}), value, lease);
  } catch (const Error& e) {
    fail(e.code(), "failed to put (key, value) (" + key + ", " + value + "): " + e.what());
  }
}

void KVStore::del(const Ctx& ctx, const std::string& key, const std::vector<OpOption>& opts) {
  check_ctx(ctx);
  std::string k = path_join({kStorePrefix, key});
  RangeOpts o = resolve_opts(&k, opts);
  int64_t deleted = 0;
  try {
    cli_->del(k, o.end, &deleted);
  } catch (const Error& e) {
    fail(e.code(), "failed to delete key " + key + ": " + e.what());
  }
  if (deleted == 0) fail(Errc::kNoKey, "Key could not be found");
}

// ---------------------------------------------------------------- cluster
std::string get_ip() {
  if (const char* e = std::getenv("PTYPE_ADVERTISE_ADDR"))
    if (*e) return e;
  const std::string ip = first_nonloopback_ipv4();
  if (ip.empty()) fail("failed to read hostname: no network address that aren't loopbacks");
  return ip;
}

std::string Cluster::join_existing_cluster(const Ctx& ctx, const Config& cfg) {
  if (cfg.initial_cluster_client_urls.empty())
    fail(Errc::kConfig,
         "joining an existing cluster requires at least one client url from a member from the existing cluster");
  check_ctx(ctx);
  auto cli = std::make_shared<KvClient>(cfg.initial_cluster_client_urls, 5000);
  std::vector<MemberInfo> members;
  try {
    cli->member_add(cfg.member->lpurls, true, &members);
  } catch (const Error& e) {
    cli->close();
    fail(e.code(), "failed to add member with peerURLs [" + ptype::join(cfg.member->lpurls, " ") + "]: " + e.what());
  }
  cli->close();
  std::vector<std::string> parts;
  for (const auto& u : cfg.member->lpurls) parts.push_back(cfg.member->name + "=" + u);
  for (const auto& m : members)
    if (!m.name.empty())
      for (const auto& u : m.peer_urls) parts.push_back(m.name + "=" + u);
  std::sort(parts.begin(), parts.end());
  return ptype::join(parts, ",");
}

std::shared_ptr<Cluster> Cluster::join(const Ctx& ctx, const Config& cfg0) {
  if (!cfg0.member) fail(Errc::kConfig, "config has no member (etcd) configuration");
  Config cfg = cfg0;
  cfg.member = std::make_shared<MemberConfig>(*cfg0.member);
  if (cfg.debug) log_set_level(LogLevel::kDebug);
  if (cfg.member->cluster_state == "existing") cfg.member->initial_cluster = join_existing_cluster(ctx, cfg);

  std::shared_ptr<Cluster> c(new Cluster());
  c->cfg_ = cfg;
  // startEmbeddedEtcd (cluster.go:161-196): its promote calls share a 10 s context
  Ctx start_ctx = Context::with_timeout(ctx, 10000);
  c->member_.reset(new Member(*cfg.member));
  try {
    c->member_->start();
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to start etcd: ") + e.what());
  }
  while (!c->member_->wait_ready(100)) {  // <-ReadyNotify(): no timeout in the reference
    if (ctx && ctx->done()) {
      c->member_->close();
      fail(Errc::kCanceled, ctx->err());
    }
  }
  log_debug("etcd started", {{"id", std::to_string(c->member_->id())},
                             {"learner", c->member_->is_learner() ? "true" : "false"}});
  if (c->member_->is_learner()) {
    auto seed = std::make_shared<KvClient>(cfg.initial_cluster_client_urls, 5000);
    for (;;) {
      try {
        if (start_ctx->done()) fail(Errc::kTimeout, "context deadline exceeded");
        seed->member_promote(c->member_->id(), 5000);
        log_debug("etcd learner successfully promoted", {{"id", std::to_string(c->member_->id())}});
        break;
      } catch (const Error& e) {
        if (e.code() == Errc::kLearnerNotReady) {
          log_debug("learner not ready to be promoted", {{"id", std::to_string(c->member_->id())}});
          if (start_ctx->wait(2000)) {
            seed->close();
            c->member_->close();
            fail(Errc::kTimeout, "can't promote member: context deadline exceeded");
          }
          continue;
        }
        seed->close();
        c->member_->close();
        fail(e.code(), std::string("can't promote member: ") + e.what());
      }
    }
    seed->close();
  }
  std::vector<std::string> curls = cfg.member->lcurls;
  c->client_ = std::make_shared<KvClient>(curls, 5000);
  c->registry = std::make_shared<EtcdRegistry>(std::make_shared<KvClient>(curls, 5000));
  c->store = std::make_shared<KVStore>(std::make_shared<KvClient>(curls, 5000));
  c->local_addr_ = get_ip();
  c->registry->register_node(ctx, cfg.service_name, cfg.node_name, c->local_addr_, cfg.port);
  return c;
}

Cluster::~Cluster() { close(); }

std::vector<MemberInfo> Cluster::member_list(const Ctx& ctx) {
  check_ctx(ctx);
  try {
    return client_->member_list();
  } catch (const Error& e) {
    fail(e.code(), std::string("failed to retrieve member list: ") + e.what());
  }
}

std::shared_ptr<RpcClient> Cluster::new_client(const std::string& service, const ConnConfig* cfg) {
  Ctx wctx = Context::with_cancel(Context::background());
  auto ch = registry->watch_service(wctx, service);
  auto cli = std::make_shared<RpcClient>(local_addr_, service, ch, cfg ? *cfg : default_conn_config());
  cli->on_close = [wctx] { wctx->cancel(); };
  std::lock_guard<std::mutex> g(mu_);
  client_ctxs_.push_back(wctx);
  return cli;
}

void Cluster::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return;
    closed_ = true;
    for (auto& c : client_ctxs_) c->cancel();
  }
  if (member_) member_->close();
  // the reference closes only etcd; we also release the three clients
  if (registry) registry->close();
  if (store) store->kv().close();
  if (client_) client_->close();
}

}  // namespace ptype
