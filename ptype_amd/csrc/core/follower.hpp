// The control side of the GPU registry mirror, compiled: it follows a
// service's shard records in the replicated store and turns them into table
// operations for the device registry (K5 upserts / deletes, K6 sweeps).
//
// Reference: clients follow a service with WatchService -- a watch on the
// service prefix, a full re-list on every event (cluster/registry.go:119-150),
// and a debounced re-selection (cluster/rpc.go:197-244).  Here:
//
//   * a watch thread collects PUT / DELETE events of
//     `store/_ptype/actors/<service>/` and, every relist period, re-lists the
//     prefix: a missed PUT or DELETE is queued, and every listed shard's
//     "last seen alive" time is refreshed (its lease is alive);
//   * take(now) -- called by the runtime at the start of every Send, on the
//     thread that owns the device table -- applies what is queued to the
//     applied-shards view and returns the table operations: the actors of new or
//     changed shards (upsert, deadline = last seen + TTL + grace), of removed
//     ones (delete), deadline refreshes, and whether K6 must sweep (a shard was
//     not seen within its deadline: the backstop when no DELETE arrives).
//   * quiet(now) is the Send's fast path: nothing queued since the last take and
//     no deadline passed -- two loads, no lock.
//
// Shard record (the node's lease-attached JSON):
//   {"rank", "world", "count", "node"[, "gen", "blocks"]}: actor b + world * k of
//   every hosted original rank b (blocks, default [rank]) in mailbox
//   j * count + k (j = b's index in blocks).  Records of data-plane generations
//   older than set_generation()'s are dropped without touching the table (the
//   recovering runtime rebuilt it).
#pragma once
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kvclient.hpp"
#include "util.hpp"

namespace ptype {

struct ShardRecord {
  int64_t rank = 0, world = 1, count = 0, gen = 0;
  std::vector<int64_t> blocks;  // original ranks hosted (empty: [rank])
  std::string json;             // as stored (compared to detect a change)
  static ShardRecord parse(const std::string& json);
  // actor ids and their mailboxes on the hosting rank
  void actors(std::vector<int64_t>* ids, std::vector<int32_t>* mbox) const;
  int64_t n_actors() const { return count * (int64_t)(blocks.empty() ? 1 : blocks.size()); }
};

struct MirrorOp {  // one device-table operation (the table lives in the GPU module)
  enum Kind : int { kUpsert = 0, kDelete = 1 };
  Kind kind = kUpsert;
  std::string key;
  int32_t rank = 0;
  int64_t deadline_ms = 0;
  std::vector<int64_t> ids;
  std::vector<int32_t> mbox;  // upserts
};

class RegistryFollower {
 public:
  // prefix: the store key prefix of the service's shard records (with the
  // store's own "store/" prefix); relist_s: the re-list period; watch=false:
  // re-list only.
  RegistryFollower(std::shared_ptr<KvClient> kv, const std::string& prefix, int64_t ttl_ms, int64_t grace_ms,
                   double relist_s, bool watch);
  ~RegistryFollower();
  RegistryFollower(const RegistryFollower&) = delete;
  RegistryFollower& operator=(const RegistryFollower&) = delete;
  void close();

  bool quiet(int64_t now_ms) const {
    return version_.load(std::memory_order_acquire) == applied_ && now_ms < next_expiry_;
  }
  // Apply what is queued; returns the table operations, sets *sweep when K6 must
  // sweep at now_ms, *changed to the shards added, changed or removed.
  std::vector<MirrorOp> take(int64_t now_ms, bool* sweep, int64_t* changed);
  void set_generation(int64_t gen);

  uint64_t version() const { return version_.load(std::memory_order_acquire); }
  uint64_t applies() const { return applies_; }
  uint64_t relists() const { return relists_.load(); }
  uint64_t events() const { return events_.load(); }
  // applied shards: key -> (record JSON, deadline ms)
  std::vector<std::tuple<std::string, std::string, int64_t>> shards() const;
  int64_t actors() const;

 private:
  struct Pending {
    bool put;
    std::string key;
    ShardRecord rec;
  };
  struct Applied {
    ShardRecord rec;
    int64_t deadline = 0;
  };
  void run();
  void relist();
  void put(const std::string& key, const ShardRecord& rec, int64_t deadline, std::vector<MirrorOp>* ops);
  void del(const std::string& key, std::vector<MirrorOp>* ops);

  std::shared_ptr<KvClient> kv_;
  std::string prefix_, end_;
  int64_t ttl_ms_, grace_ms_;
  double relist_s_;
  Ctx ctx_;
  std::shared_ptr<Channel<WatchResponse>> watch_;
  std::thread th_;
  std::atomic<bool> stop_{false};

  mutable std::mutex mu_;                // pending_, seen_, min_gen_ (watch thread vs take)
  std::vector<Pending> pending_;
  std::map<std::string, int64_t> seen_;  // key -> monotonic ms last listed / put (lease alive)
  int64_t min_gen_ = 0;
  std::map<std::string, std::string> applied_json_;  // shards_' records as of the last take (for the re-list)
  bool watching_ = false;                             // a watch was asked for (re-opened when it closes)
  uint64_t watch_reopens_ = 0;
  std::atomic<uint64_t> version_{0};
  std::atomic<uint64_t> relists_{0}, events_{0};

  // owned by the take() caller
  std::map<std::string, Applied> shards_;
  uint64_t applied_ = ~0ull;
  int64_t next_expiry_ = 0;
  uint64_t applies_ = 0;
};

// This node's shard record, attached to a lease kept alive until close()
// (graceful close revokes it: the shard disappears at once) -- the reference's
// Register (cluster/registry.go:51-86) for a data-plane shard.
class ShardLease {
 public:
  ShardLease(std::shared_ptr<KvClient> kv, const std::string& key, const std::string& record_json, int64_t ttl_s);
  ~ShardLease();
  void update(const std::string& record_json);  // same lease, new record (a new generation's placement)
  void stop_keepalive();                        // stop refreshing without revoking (a crash, for tests)
  void close();
  const std::string& record() const { return record_; }
  int64_t lease() const { return lease_; }

 private:
  std::shared_ptr<KvClient> kv_;
  std::string key_, record_;
  int64_t lease_ = 0;
  Ctx ctx_;
  std::shared_ptr<Channel<int64_t>> ka_;
  std::thread th_;
  bool closed_ = false;
};

}  // namespace ptype
