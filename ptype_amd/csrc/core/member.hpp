// Control-plane member: the C++ replacement for the embedded etcd server the
// reference starts inside every process (cluster/cluster.go:161-196).
//
// Owns a Raft node (raft.hpp), durable storage (storage.hpp), the MVCC/lease
// state machine (mvcc.hpp), a watch hub and the membership table, and serves
// the control-plane protocol (proto.hpp) on its client and peer URLs.
//
// Threads: one raft loop (ticks, peer messages, proposals, persist, send,
// apply), one notifier (watch delivery), one sender per peer, and one reader
// per accepted connection whose requests run on short-lived worker threads.
// Proposals carry a request id; every member applies every entry, and the
// member that proposed resolves its waiter -- so proposals made on a follower
// or learner are forwarded by Raft itself and still answered locally.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "config.hpp"
#include "mvcc.hpp"
#include "net.hpp"
#include "proto.hpp"
#include "raft.hpp"
#include "storage.hpp"

namespace ptype {

using WatchFn = std::function<void(const std::vector<Event>&, int64_t rev, bool canceled)>;

struct ApplyResult {
  std::string err;
  Errc code = Errc::kGeneric;
  int64_t rev = 0, deleted = 0, lease_id = 0, ttl = 0;
  uint64_t member_id = 0;
  int conf_type = -1;
  std::vector<MemberInfo> members;
};

class Member {
 public:
  explicit Member(const MemberConfig& cfg);
  ~Member();

  void start();                           // storage, raft, listeners, loops
  bool wait_ready(int64_t timeout_ms);    // ReadyNotify: leader known + attributes published
  void close();                           // stop everything (no lease revoke, like the reference)
  bool closed() const { return stop_.load(); }

  uint64_t id() const { return id_; }
  std::string name() const { return cfg_.name; }
  bool is_learner();
  uint64_t leader();
  StatusInfo status();
  const MemberConfig& config() const { return cfg_; }
  std::vector<int> client_ports() const;
  uint64_t reads_served() const { return reads_served_.load(); }  // linearizable reads through ReadIndex

  // ---- local API (also what the TCP handler calls)
  RangeResult range(const std::string& key, const RangeOpts& o, int64_t timeout_ms = 5000);
  int64_t put(const std::string& key, const std::string& value, int64_t lease, int64_t timeout_ms = 5000);
  int64_t del(const std::string& key, const std::string& end, int64_t* deleted, int64_t timeout_ms = 5000);
  int64_t lease_grant(int64_t ttl, int64_t id, int64_t* granted_ttl, int64_t timeout_ms = 5000);
  void lease_revoke(int64_t id, int64_t timeout_ms = 5000);
  int64_t lease_keepalive(int64_t id);  // TTL, throws kLeaseNotFound
  int64_t lease_ttl(int64_t id);        // remaining ms on the leader view, -1 unknown
  std::vector<LeaseInfo> lease_list();
  void compact(int64_t rev, int64_t timeout_ms = 5000);
  std::vector<MemberInfo> member_list();
  MemberInfo member_add(const std::vector<std::string>& peer_urls, bool learner, std::vector<MemberInfo>* members,
                        int64_t timeout_ms = 10000);
  void member_promote(uint64_t id, int64_t timeout_ms = 10000);
  void member_remove(uint64_t id, int64_t timeout_ms = 10000);
  int64_t watch(const std::string& key, const std::string& end, int64_t start_rev, WatchFn fn);
  void cancel_watch(int64_t wid);

 private:
  struct Waiter {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    ApplyResult res;
  };
  struct Inbox {
    std::vector<raft::Message> msgs;
    std::vector<std::pair<uint8_t, std::string>> props;  // (entry type, data)
    std::vector<std::string> reads;                       // ReadIndex request ids
  };
  struct ReadWaiter {
    bool done = false, ok = false;
    uint64_t index = 0;
  };
  struct Watcher {
    std::string key, end;
    WatchFn fn;
    int64_t next_rev = 0;
  };
  struct Peer;

  ApplyResult propose_wait(uint8_t etype, uint8_t op, const std::string& payload, int64_t timeout_ms);
  // Linearizable read barrier (ReadIndex): returns once this member has applied
  // everything committed when the read arrived -- no log entry, no fsync.
  void read_barrier(int64_t timeout_ms);
  void raft_loop();
  void notifier_loop();
  void process_ready();
  void apply_entry(const raft::Entry& e);
  void apply_conf(uint64_t reqid, const std::string& body, ApplyResult* r);
  void resolve(uint64_t reqid, ApplyResult r);
  void publish_events(std::vector<Event> ev, int64_t rev);
  void send_raft(const raft::Message& m);
  void update_peers();
  std::string check_conf(const raft::Entry& e);
  void snapshot_state(uint64_t* index, uint64_t* term, std::string* data);
  void restore_state(const std::string& data);
  void maybe_snapshot();
  void handle_conn(std::shared_ptr<Conn> c);
  std::string handle_request(uint8_t op, Reader& r, const std::shared_ptr<Conn>& c,
                             std::set<int64_t>* conn_watches);
  void bootstrap_new(const std::map<std::string, std::vector<std::string>>& cluster);
  void join_existing(const std::map<std::string, std::vector<std::string>>& cluster);
  uint64_t next_reqid();
  std::string save_meta_blob() const;

  MemberConfig cfg_;
  uint64_t id_ = 0;
  std::unique_ptr<Storage> storage_;
  std::unique_ptr<raft::Node> node_;

  // state machine (guarded by sm_mu_)
  std::mutex sm_mu_;
  MvccStore kv_;
  Lessor lessor_;
  std::map<uint64_t, MemberInfo> members_;
  uint64_t applied_ = 0;

  // raft loop input
  std::mutex in_mu_;
  std::condition_variable in_cv_;
  Inbox inbox_;

  std::mutex wait_mu_;
  std::map<uint64_t, std::shared_ptr<Waiter>> waiters_;
  std::mutex read_mu_;
  std::condition_variable read_cv_;  // a read state arrived or applied_ advanced
  std::map<std::string, ReadWaiter> read_waiters_;
  std::atomic<uint64_t> applied_pub_{0};  // applied_, readable without sm_mu_
  std::atomic<uint64_t> read_seq_{0};
  std::atomic<uint64_t> reads_served_{0};
  std::atomic<uint64_t> reqseq_{0};
  std::atomic<int64_t> lease_seq_{0};

  // watch hub
  std::mutex watch_mu_;
  std::map<int64_t, Watcher> watchers_;
  std::atomic<int64_t> watch_seq_{0};
  std::mutex note_mu_;
  std::condition_variable note_cv_;
  std::deque<std::pair<std::vector<Event>, int64_t>> notes_;

  // peers
  std::mutex peer_mu_;
  std::map<uint64_t, std::shared_ptr<Peer>> peers_;

  std::vector<std::unique_ptr<Listener>> listeners_;
  std::thread raft_th_, note_th_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> ready_{false};
  std::atomic<bool> published_{false};
  bool was_leader_ = false;
  std::set<int64_t> revoking_;
  int64_t last_tick_ms_ = 0;
  uint64_t last_snap_index_ = 0;
};

// ID of a member from its peer URLs and the cluster token (+ a salt for
// runtime adds), as etcd derives member IDs.
uint64_t compute_member_id(const std::vector<std::string>& peer_urls, const std::string& token, uint64_t salt);
// "n1=url,n2=url" -> name -> urls (a name may repeat for multi-URL members)
std::map<std::string, std::vector<std::string>> parse_initial_cluster(const std::string& s);

}  // namespace ptype
