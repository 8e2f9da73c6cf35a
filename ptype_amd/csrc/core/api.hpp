// Public control-plane API: Registry (cluster/registry.go), KVStore + option
// helpers (cluster/store.go, cluster/store_config.go) and the Cluster facade
// (cluster/cluster.go: Join, MemberList, Close, NewClient).
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "balancer.hpp"
#include "config.hpp"
#include "kvclient.hpp"
#include "member.hpp"

namespace ptype {

// ---------------------------------------------------------------- registry
extern const char* kServicesPrefix;  // "services"
std::string etcd_key(const std::vector<std::string>& elems);  // filepath.Join(...) + "/"
std::string node_json(const Node& n);                         // {"address":..,"port":..}
Node node_from_json(const std::string& s);

class Registry {
 public:
  virtual ~Registry() = default;
  virtual void register_node(const Ctx& ctx, const std::string& service, const std::string& node,
                             const std::string& host, int64_t port) = 0;
  virtual std::map<std::string, std::vector<Node>> services(const Ctx& ctx) = 0;
  virtual std::shared_ptr<NodesChan> watch_service(const Ctx& ctx, const std::string& service) = 0;
};

class EtcdRegistry : public Registry {
 public:
  explicit EtcdRegistry(std::shared_ptr<KvClient> cli) : cli_(std::move(cli)) {}
  ~EtcdRegistry() override;
  void register_node(const Ctx& ctx, const std::string& service, const std::string& node, const std::string& host,
                     int64_t port) override;
  std::map<std::string, std::vector<Node>> services(const Ctx& ctx) override;
  std::shared_ptr<NodesChan> watch_service(const Ctx& ctx, const std::string& service) override;
  std::vector<Node> nodes(const Ctx& ctx, const std::string& service);
  KvClient& kv() { return *cli_; }
  std::shared_ptr<KvClient> kv_ptr() { return cli_; }
  void close();

 private:
  std::shared_ptr<KvClient> cli_;
  std::mutex mu_;
  std::vector<std::thread> threads_;
  std::atomic<bool> closed_{false};
};

// ---------------------------------------------------------------- store
extern const char* kStorePrefix;  // "store"

// clientv3.OpOption equivalents (cluster/store_config.go:33-103)
struct OpOption {
  enum Kind { kPrefix, kLimit, kRev, kRange, kFromKey, kSerializable, kKeysOnly, kCountOnly, kSort, kLease };
  OpOption(Kind k = kPrefix) : kind(k) {}  // NOLINT: implicit from a kind, as the option helpers build them
  Kind kind;
  int64_t n = 0;
  std::string s;
  int target = 0, order = 0;
};
// Resolves options against the (already prefixed) key, exactly as clientv3 does:
// WithPrefix on "" = every key; WithRange's end is taken verbatim (NOT prefixed
// with "store/" -- a reference quirk kept for parity); SortByKey+Ascend = none.
RangeOpts resolve_opts(std::string* key, const std::vector<OpOption>& opts);

class KVStore {
 public:
  explicit KVStore(std::shared_ptr<KvClient> cli) : cli_(std::move(cli)) {}
  // Get: values of store/<key> (+options); throws kNoKey when nothing matches.
  std::vector<std::string> get(const Ctx& ctx, const std::string& key, const std::vector<OpOption>& opts = {});
  void put(const Ctx& ctx, const std::string& key, const std::string& value, const std::vector<OpOption>& opts = {});
  // Delete: throws kNoKey when nothing was deleted.
  void del(const Ctx& ctx, const std::string& key, const std::vector<OpOption>& opts = {});
  KvClient& kv() { return *cli_; }

 private:
  std::shared_ptr<KvClient> cli_;
};

// ---------------------------------------------------------------- cluster
class Cluster {
 public:
  // Join (cluster/cluster.go:28-84): optional learner add via a seed member,
  // start the local control-plane member, wait until ready, promote if a
  // learner, create clients, register this node under services/<svc>/<node>/.
  static std::shared_ptr<Cluster> join(const Ctx& ctx, const Config& cfg);
  ~Cluster();

  std::shared_ptr<EtcdRegistry> registry;
  std::shared_ptr<KVStore> store;
  std::vector<MemberInfo> member_list(const Ctx& ctx);
  std::shared_ptr<RpcClient> new_client(const std::string& service, const ConnConfig* cfg);
  void close();
  const std::string& local_addr() const { return local_addr_; }
  Member& member() { return *member_; }
  const Config& config() const { return cfg_; }

  // joinExistingCluster + memberAdd (cluster.go:105-147): returns initial-cluster
  static std::string join_existing_cluster(const Ctx& ctx, const Config& cfg);

 private:
  Config cfg_;
  std::unique_ptr<Member> member_;
  std::shared_ptr<KvClient> client_;
  std::string local_addr_;
  std::vector<std::shared_ptr<RpcClient>> clients_;
  std::vector<Ctx> client_ctxs_;
  std::mutex mu_;
  bool closed_ = false;
};

std::string get_ip();  // first non-loopback IPv4 (cluster.go:198-213); PTYPE_ADVERTISE_ADDR overrides

}  // namespace ptype
