// MVCC key-value state machine with leases (the etcd server-side
// surface the reference relies on: Range with prefix/range/from-key, sort,
// limit, revision, keys-only, count-only; Put with lease; DeleteRange; lease
// grant/revoke/keepalive/expiry; watch events).  Applied identically on every
// control-plane member by the Raft applier.
//
// Reference call sites: cluster/registry.go:59,65,69,94,123,154;
// cluster/store.go:40,57,66; option semantics cluster/store_config.go:33-103.
#pragma once
#include <stdint.h>

#include <map>
#include <set>
#include <string>
#include <vector>

namespace ptype {

struct KeyValue {
  std::string key, value;
  int64_t create_revision = 0, mod_revision = 0, version = 0, lease = 0;
};

struct Event {
  enum Type : uint8_t { kPut = 0, kDelete = 1 };
  Type type = kPut;
  KeyValue kv;  // for deletes: key + mod_revision of the tombstone
};

enum SortTarget : int { kSortKey = 0, kSortVersion = 1, kSortCreate = 2, kSortMod = 3, kSortValue = 4 };
enum SortOrder : int { kSortNone = 0, kSortAscend = 1, kSortDescend = 2 };

struct RangeOpts {
  std::string end;  // "" = single key, "\0" = from key, else [key, end)
  int64_t limit = 0;
  int64_t rev = 0;
  int sort_target = kSortKey;
  int sort_order = kSortNone;
  bool serializable = false;
  bool keys_only = false;
  bool count_only = false;
};

struct RangeResult {
  std::vector<KeyValue> kvs;
  int64_t count = 0;
  bool more = false;
  int64_t rev = 0;
};

// Does [key, end) (etcd range encoding) contain k?
bool range_contains(const std::string& key, const std::string& end, const std::string& k);
// clientv3.GetPrefixRangeEnd (cluster/store_config.go:41-58)
std::string prefix_range_end(const std::string& prefix);

class MvccStore {
 public:
  int64_t rev() const { return rev_; }
  int64_t compact_rev() const { return compact_rev_; }

  RangeResult range(const std::string& key, const RangeOpts& o) const;  // throws on future/compacted rev
  // Each mutator is one transaction: one new main revision if anything changed.
  int64_t put(const std::string& key, const std::string& value, int64_t lease, std::vector<Event>* ev);
  int64_t delete_range(const std::string& key, const std::string& end, int64_t* deleted, std::vector<Event>* ev,
                       std::vector<std::string>* deleted_keys = nullptr);
  void compact(int64_t rev);
  // History for watch replay: every event with mod_revision >= from_rev in [key, end).
  std::vector<Event> events_since(int64_t from_rev, const std::string& key, const std::string& end) const;
  size_t key_count() const;

  std::string serialize() const;
  void restore(const std::string& data);

 private:
  struct Version {
    int64_t mod = 0, create = 0, ver = 0, lease = 0;
    bool tomb = false;
    std::string value;
  };
  const Version* at(const std::vector<Version>& h, int64_t rev) const;
  std::map<std::string, std::vector<Version>> idx_;
  int64_t rev_ = 1;
  int64_t compact_rev_ = 0;
};

struct LeaseInfo {
  int64_t id = 0;
  int64_t ttl = 0;         // granted TTL (s)
  int64_t expiry_ms = 0;   // leader-local monotonic deadline (0 = not tracked)
  std::set<std::string> keys;
};

class Lessor {
 public:
  explicit Lessor(int64_t min_ttl = 1) : min_ttl_(min_ttl) {}
  int64_t grant(int64_t id, int64_t ttl, int64_t now_ms);  // returns effective TTL
  bool exists(int64_t id) const { return leases_.count(id) != 0; }
  std::set<std::string> revoke(int64_t id);               // returns attached keys
  int64_t renew(int64_t id, int64_t now_ms);               // returns TTL, -1 if unknown
  int64_t remaining_ms(int64_t id, int64_t now_ms) const;  // -1 if unknown
  void attach(int64_t id, const std::string& key);
  void detach(int64_t id, const std::string& key);
  std::vector<int64_t> expired(int64_t now_ms) const;
  void promote(int64_t now_ms);  // new leader: every lease gets a full TTL from now
  void demote();                 // follower: stop tracking deadlines
  std::vector<LeaseInfo> list() const;
  int64_t min_ttl() const { return min_ttl_; }
  std::string serialize() const;
  void restore(const std::string& data, int64_t now_ms);

 private:
  std::map<int64_t, LeaseInfo> leases_;
  int64_t min_ttl_;
  bool primary_ = false;
};

}  // namespace ptype
