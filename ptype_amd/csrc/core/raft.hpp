// Raft consensus core: the replicated-log engine the reference gets
// from its embedded etcd member (cluster/cluster.go:161-196 starts it; learner
// add/promote at :120-147 and :183-195; MemberList at :86-93).
//
// A deterministic, message-passing state machine in the style of a "raw node":
// the owner feeds it ticks, local proposals and peer messages, then drains
// messages to send, entries to persist and committed entries to apply.  No I/O
// and no threads live here, so multi-member behaviour is unit-testable with a
// fake network.  Features: randomized elections with check-quorum (a leader
// that loses its quorum steps down; a follower that hears a live leader ignores
// disruptive vote requests), log replication with conflict back-off, follower
// proposal forwarding, learners (non-voting members that replicate) and
// single-server membership changes (one pending conf change at a time, learner
// promotion only once it has caught up), and snapshots for lagging followers.
#pragma once
#include <stdint.h>

#include <functional>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

namespace ptype {
namespace raft {

enum EntryType : uint8_t { kEntryNormal = 0, kEntryConfChange = 1 };

struct Entry {
  uint64_t term = 0, index = 0;
  uint8_t type = kEntryNormal;
  std::string data;
};

enum MsgType : uint8_t {
  kMsgProp = 1,
  kMsgApp = 2,
  kMsgAppResp = 3,
  kMsgVote = 4,
  kMsgVoteResp = 5,
  kMsgHeartbeat = 6,
  kMsgHeartbeatResp = 7,
  kMsgSnap = 8,
  kMsgPropReject = 9,   // leader -> proposer: conf change refused (context = reason)
  kMsgLeaseRenew = 10,  // follower -> leader: keepalive forwarded (context = lease id)
  kMsgReadIndex = 11,      // follower -> leader: linearizable read request (context = request id)
  kMsgReadIndexResp = 12,  // leader -> follower: index = read index (reject: no leader term commit yet)
};

// A linearizable read confirmed by a quorum (ReadIndex): serve it locally once
// the state machine has applied `index`.  ok == false: no leader, or the leader
// has not committed an entry of its term yet -- retry.
struct ReadState {
  std::string ctx;
  uint64_t index = 0;
  bool ok = false;
};

struct Message {
  uint8_t type = 0;
  uint64_t from = 0, to = 0, term = 0, log_term = 0, index = 0, commit = 0;
  bool reject = false;
  uint64_t reject_hint = 0;
  std::vector<Entry> entries;
  uint64_t snap_index = 0, snap_term = 0;
  std::string snap_data;
  std::string context;

  std::string encode() const;
  static Message decode(const std::string& s);
};

struct HardState {
  uint64_t term = 0, vote = 0, commit = 0;
  bool operator==(const HardState& o) const { return term == o.term && vote == o.vote && commit == o.commit; }
};

enum ConfChangeType : uint8_t { kAddNode = 0, kRemoveNode = 1, kAddLearner = 2, kPromoteLearner = 3 };

enum Role : uint8_t { kFollower = 0, kCandidate = 1, kLeader = 2 };

struct Progress {
  uint64_t match = 0, next = 1;
  bool learner = false;
  bool recent_active = false;
};

struct Options {
  uint64_t id = 0;
  int election_tick = 10;
  int heartbeat_tick = 1;
  size_t max_entries_per_msg = 256;
  // Leader-side validation of a conf-change proposal ("" = accept).
  std::function<std::string(const Entry&)> check_conf;
  // Leader-side snapshot source for lagging followers: fills index/term/data.
  std::function<void(uint64_t* index, uint64_t* term, std::string* data)> snapshot_source;
};

class Node {
 public:
  explicit Node(Options o);

  // ---- bootstrap / restore
  void bootstrap(const std::set<uint64_t>& voters, const std::set<uint64_t>& learners);
  void restore(const HardState& hs, uint64_t snap_index, uint64_t snap_term, const std::vector<Entry>& entries,
               const std::set<uint64_t>& voters, const std::set<uint64_t>& learners, uint64_t applied);

  // ---- inputs
  void tick();
  void step(const Message& m);
  std::string propose(uint8_t type, const std::string& data);  // "" = accepted / forwarded
  void campaign();
  // ReadIndex (Raft thesis 6.4): the leader records its commit index, confirms
  // it is still the leader with one heartbeat round acknowledged by a quorum,
  // and answers the index -- no log entry, no fsync.  A follower forwards the
  // request to the leader.  Results come out of take_read_states().
  void read_index(const std::string& ctx);

  // ---- outputs (drained by the owner)
  std::vector<Message> take_messages();
  std::vector<Entry> take_unstable();  // append to the WAL in order (an index re-appears after a conflict)
  bool take_hardstate(HardState* hs);  // true if changed since the last take
  std::vector<Entry> take_committed(size_t max = 4096);  // (applied, commit]; advances applied
  bool take_snapshot(uint64_t* index, uint64_t* term, std::string* data);  // follower: install this first
  std::vector<ReadState> take_read_states();

  // ---- membership (called by the applier when a conf change commits)
  void apply_conf_change(uint8_t type, uint64_t node);
  const std::set<uint64_t>& voters() const { return voters_; }
  const std::set<uint64_t>& learners() const { return learners_; }
  bool is_learner(uint64_t id) const { return learners_.count(id) != 0; }

  // ---- compaction: drop entries <= index (index <= applied), remember its term
  void compact(uint64_t index);

  // ---- introspection
  uint64_t id() const { return opt_.id; }
  uint64_t term() const { return term_; }
  uint64_t leader() const { return lead_; }
  Role role() const { return role_; }
  uint64_t commit() const { return commit_; }
  uint64_t applied() const { return applied_; }
  uint64_t last_index() const { return snap_index_ + log_.size(); }
  uint64_t first_index() const { return snap_index_ + 1; }
  uint64_t snap_index() const { return snap_index_; }
  uint64_t snap_term() const { return snap_term_; }
  uint64_t term_at(uint64_t i) const;
  const std::map<uint64_t, Progress>& progress() const { return prs_; }
  const Entry* entry_at(uint64_t i) const;

 private:
  void become_follower(uint64_t term, uint64_t lead);
  void become_candidate();
  void become_leader();
  void reset(uint64_t term);
  bool promotable() const { return voters_.count(opt_.id) != 0; }
  size_t quorum() const { return voters_.size() / 2 + 1; }
  void send(Message m);
  void send_append(uint64_t to);
  void send_heartbeat(uint64_t to);
  void broadcast_append();
  void broadcast_heartbeat();
  bool maybe_commit();
  void append_local(std::vector<Entry> ents);
  void handle_append(const Message& m);
  void handle_snapshot(const Message& m);
  void step_leader(const Message& m);
  void step_candidate(const Message& m);
  void step_follower(const Message& m);
  void reset_randomized_timeout();
  void leader_read(const std::string& ctx, uint64_t from);
  void read_done(const std::string& ctx, uint64_t index, uint64_t from, bool ok);

  Options opt_;
  uint64_t term_ = 0, vote_ = 0, lead_ = 0, commit_ = 0, applied_ = 0;
  Role role_ = kFollower;
  std::set<uint64_t> voters_, learners_;
  std::map<uint64_t, Progress> prs_;
  std::set<uint64_t> votes_granted_, votes_rejected_;
  std::vector<Entry> log_;  // entries (snap_index_, last]
  uint64_t snap_index_ = 0, snap_term_ = 0;
  int elapsed_ = 0, hb_elapsed_ = 0, randomized_timeout_ = 10;
  uint64_t pending_conf_index_ = 0;
  std::mt19937_64 rng_;

  struct PendingRead {
    uint64_t index = 0, from = 0;
    int age = 0;  // leader ticks since the round started (expired past kReadExpiryElections elections)
    std::set<uint64_t> acks;
  };
  static constexpr int kReadExpiryElections = 4;
  std::map<std::string, PendingRead> reads_;  // leader: awaiting a quorum of heartbeat acks
  std::vector<ReadState> read_states_;

  std::vector<Message> msgs_;
  std::vector<Entry> unstable_;
  HardState last_hs_;
  bool pending_snap_ = false;
  uint64_t psnap_index_ = 0, psnap_term_ = 0;
  std::string psnap_data_;
};

}  // namespace raft
}  // namespace ptype
