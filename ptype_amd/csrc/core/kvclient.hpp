// Control-plane client (the role etcd's clientv3 plays for the reference:
// cluster/cluster.go:50-57, cluster/registry.go:34-49, cluster/store.go:22-35).
// Dials lazily (clientv3.New with an unreachable or empty endpoint still
// constructs -- cluster/store_test.go:11-15), multiplexes requests by id on one
// TCP connection, fails over across endpoints, and streams watch events and
// lease keepalive responses into channels.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mvcc.hpp"
#include "net.hpp"
#include "proto.hpp"
#include "util.hpp"

namespace ptype {

struct WatchResponse {
  std::vector<Event> events;
  int64_t revision = 0;
  bool canceled = false;
  std::string err;
};

class KvClient : public std::enable_shared_from_this<KvClient> {
 public:
  KvClient(std::vector<std::string> endpoints, int64_t dial_timeout_ms = 5000);
  ~KvClient();
  void close();

  RangeResult get(const std::string& key, const RangeOpts& o, int64_t timeout_ms = 5000);
  int64_t put(const std::string& key, const std::string& value, int64_t lease = 0, int64_t timeout_ms = 5000);
  int64_t del(const std::string& key, const std::string& end, int64_t* deleted, int64_t timeout_ms = 5000);
  int64_t grant(int64_t ttl, int64_t* granted_ttl, int64_t timeout_ms = 5000);
  void revoke(int64_t id, int64_t timeout_ms = 5000);
  int64_t keepalive_once(int64_t id, int64_t timeout_ms = 5000);
  int64_t time_to_live_ms(int64_t id, int64_t timeout_ms = 5000);
  void compact(int64_t rev, int64_t timeout_ms = 5000);
  std::vector<MemberInfo> member_list(int64_t timeout_ms = 5000);
  MemberInfo member_add(const std::vector<std::string>& peer_urls, bool learner, std::vector<MemberInfo>* members,
                        int64_t timeout_ms = 10000);
  void member_promote(uint64_t id, int64_t timeout_ms = 10000);
  void member_remove(uint64_t id, int64_t timeout_ms = 10000);
  StatusInfo status(int64_t timeout_ms = 5000);

  // Streams TTL responses every ttl/3 until ctx is canceled or the lease is
  // gone; the channel is then closed (clientv3.KeepAlive).
  std::shared_ptr<Channel<int64_t>> keepalive(const Ctx& ctx, int64_t id);
  // Events in [key, end) from start_rev (0 = now) until ctx is canceled or the
  // stream breaks; a final response with canceled/err precedes the close.
  std::shared_ptr<Channel<WatchResponse>> watch(const Ctx& ctx, const std::string& key, const std::string& end,
                                                int64_t start_rev = 0);
  const std::vector<std::string>& endpoints() const { return eps_; }

 private:
  struct Pending {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    uint8_t code = 0;
    std::string err, payload;
  };
  std::string call(uint8_t op, const std::string& payload, int64_t timeout_ms);
  std::string call_once(uint8_t op, const std::string& payload, int64_t timeout_ms);
  std::shared_ptr<Conn> ensure_conn(int64_t timeout_ms);
  void reader(std::shared_ptr<Conn> c);
  void drop_conn(const std::shared_ptr<Conn>& c, const std::string& why);

  std::vector<std::string> eps_;
  int64_t dial_timeout_ms_;
  std::mutex mu_;
  std::shared_ptr<Conn> conn_;
  std::map<uint64_t, std::shared_ptr<Pending>> pending_;
  std::map<uint64_t, std::shared_ptr<Channel<WatchResponse>>> watches_;
  std::atomic<uint64_t> seq_{0};
  std::vector<std::thread> readers_;
  std::vector<std::thread> aux_;
  std::atomic<bool> closed_{false};
};

}  // namespace ptype
