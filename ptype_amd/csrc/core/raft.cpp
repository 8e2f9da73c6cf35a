#include "raft.hpp"

#include <algorithm>

#include "codec.hpp"
#include "util.hpp"

namespace ptype {
namespace raft {

// ---------------------------------------------------------------- encoding
std::string Message::encode() const {
  Writer w;
  w.u8(type);
  w.u64(from);
  w.u64(to);
  w.u64(term);
  w.u64(log_term);
  w.u64(index);
  w.u64(commit);
  w.b(reject);
  w.u64(reject_hint);
  w.u32((uint32_t)entries.size());
  for (const auto& e : entries) {
    w.u64(e.term);
    w.u64(e.index);
    w.u8(e.type);
    w.str(e.data);
  }
  w.u64(snap_index);
  w.u64(snap_term);
  w.str(snap_data);
  w.str(context);
  return w.buf;
}

Message Message::decode(const std::string& s) {
  Reader r(s);
  Message m;
  m.type = r.u8();
  m.from = r.u64();
  m.to = r.u64();
  m.term = r.u64();
  m.log_term = r.u64();
  m.index = r.u64();
  m.commit = r.u64();
  m.reject = r.b();
  m.reject_hint = r.u64();
  const uint32_t n = r.u32();
  m.entries.resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    m.entries[i].term = r.u64();
    m.entries[i].index = r.u64();
    m.entries[i].type = r.u8();
    m.entries[i].data = r.str();
  }
  m.snap_index = r.u64();
  m.snap_term = r.u64();
  m.snap_data = r.str();
  m.context = r.str();
  return m;
}

// ---------------------------------------------------------------- node
Node::Node(Options o) : opt_(std::move(o)), rng_(opt_.id * 0x9e3779b97f4a7c15ull + (uint64_t)mono_us()) {
  reset_randomized_timeout();
}

void Node::reset_randomized_timeout() {
  std::uniform_int_distribution<int> d(opt_.election_tick, 2 * opt_.election_tick - 1);
  randomized_timeout_ = d(rng_);
}

void Node::bootstrap(const std::set<uint64_t>& voters, const std::set<uint64_t>& learners) {
  voters_ = voters;
  learners_ = learners;
}

void Node::restore(const HardState& hs, uint64_t snap_index, uint64_t snap_term, const std::vector<Entry>& entries,
                   const std::set<uint64_t>& voters, const std::set<uint64_t>& learners, uint64_t applied) {
  term_ = hs.term;
  vote_ = hs.vote;
  snap_index_ = snap_index;
  snap_term_ = snap_term;
  log_.clear();
  for (const auto& e : entries)
    if (e.index > snap_index_) log_.push_back(e);
  commit_ = std::max(hs.commit, snap_index);
  commit_ = std::min(commit_, last_index());
  applied_ = std::max(applied, snap_index);
  voters_ = voters;
  learners_ = learners;
  last_hs_ = HardState{term_, vote_, commit_};
}

uint64_t Node::term_at(uint64_t i) const {
  if (i == snap_index_) return snap_term_;
  if (i < snap_index_ || i > last_index()) return 0;
  return log_[i - snap_index_ - 1].term;
}

const Entry* Node::entry_at(uint64_t i) const {
  if (i <= snap_index_ || i > last_index()) return nullptr;
  return &log_[i - snap_index_ - 1];
}

std::vector<ReadState> Node::take_read_states() {
  std::vector<ReadState> v;
  v.swap(read_states_);
  return v;
}

void Node::reset(uint64_t term) {
  // pending reads of a leadership that ends fail; their owners retry
  for (auto& kv : reads_) read_done(kv.first, 0, kv.second.from, false);
  reads_.clear();
  if (term_ != term) {
    term_ = term;
    vote_ = 0;
  }
  lead_ = 0;
  elapsed_ = 0;
  hb_elapsed_ = 0;
  reset_randomized_timeout();
  votes_granted_.clear();
  votes_rejected_.clear();
}

void Node::read_index(const std::string& ctx) {
  if (role_ == kLeader) {
    leader_read(ctx, opt_.id);
  } else if (lead_ != 0) {
    Message m;
    m.type = kMsgReadIndex;
    m.to = lead_;
    m.context = ctx;
    send(std::move(m));
  } else {
    read_states_.push_back(ReadState{ctx, 0, false});
  }
}

void Node::read_done(const std::string& ctx, uint64_t index, uint64_t from, bool ok) {
  if (from == opt_.id) {
    read_states_.push_back(ReadState{ctx, index, ok});
    return;
  }
  Message r;
  r.type = kMsgReadIndexResp;
  r.to = from;
  r.index = index;
  r.reject = !ok;
  r.context = ctx;
  send(std::move(r));
}

void Node::leader_read(const std::string& ctx, uint64_t from) {
  // a new leader does not know what is committed until an entry of its own term
  // is (become_leader appends an empty one for exactly this)
  if (term_at(commit_) != term_) {
    read_done(ctx, 0, from, false);
    return;
  }
  if (quorum() <= 1) {
    read_done(ctx, commit_, from, true);
    return;
  }
  PendingRead& pr = reads_[ctx];
  pr.index = commit_;
  pr.from = from;
  pr.acks = {opt_.id};
  for (auto& kv : prs_) {
    if (kv.first == opt_.id) continue;
    Message m;
    m.type = kMsgHeartbeat;
    m.to = kv.first;
    m.commit = std::min(kv.second.match, commit_);
    m.context = ctx;
    send(std::move(m));
  }
}

void Node::become_follower(uint64_t term, uint64_t lead) {
  reset(term);
  role_ = kFollower;
  lead_ = lead;
}

void Node::become_candidate() {
  reset(term_ + 1);
  role_ = kCandidate;
  vote_ = opt_.id;
  votes_granted_.insert(opt_.id);
}

void Node::become_leader() {
  reset(term_);
  role_ = kLeader;
  lead_ = opt_.id;
  prs_.clear();
  for (uint64_t v : voters_) prs_[v] = Progress{0, last_index() + 1, false, true};
  for (uint64_t l : learners_) prs_[l] = Progress{0, last_index() + 1, true, true};
  Entry e;
  e.term = term_;
  e.index = last_index() + 1;
  append_local({e});  // commit an entry of this term ASAP
  pending_conf_index_ = last_index();
  broadcast_append();
  maybe_commit();
}

void Node::campaign() {
  if (!promotable()) return;
  become_candidate();
  if (votes_granted_.size() >= quorum()) {
    become_leader();
    return;
  }
  for (uint64_t v : voters_) {
    if (v == opt_.id) continue;
    Message m;
    m.type = kMsgVote;
    m.to = v;
    m.index = last_index();
    m.log_term = term_at(last_index());
    send(m);
  }
}

void Node::send(Message m) {
  m.from = opt_.id;
  if (m.type != kMsgProp && m.type != kMsgLeaseRenew) m.term = term_;
  msgs_.push_back(std::move(m));
}

void Node::send_append(uint64_t to) {
  auto it = prs_.find(to);
  if (it == prs_.end()) return;
  Progress& pr = it->second;
  const uint64_t prev = pr.next - 1;
  if (prev < snap_index_) {  // the entries it needs were compacted: ship a snapshot
    if (!opt_.snapshot_source) return;
    Message m;
    m.type = kMsgSnap;
    m.to = to;
    opt_.snapshot_source(&m.snap_index, &m.snap_term, &m.snap_data);
    pr.next = m.snap_index + 1;
    send(std::move(m));
    return;
  }
  Message m;
  m.type = kMsgApp;
  m.to = to;
  m.index = prev;
  m.log_term = term_at(prev);
  m.commit = commit_;
  for (uint64_t i = pr.next; i <= last_index() && m.entries.size() < opt_.max_entries_per_msg; ++i)
    m.entries.push_back(log_[i - snap_index_ - 1]);
  if (!m.entries.empty()) pr.next = m.entries.back().index + 1;  // optimistic pipelining
  send(std::move(m));
}

void Node::send_heartbeat(uint64_t to) {
  auto it = prs_.find(to);
  if (it == prs_.end()) return;
  Message m;
  m.type = kMsgHeartbeat;
  m.to = to;
  m.commit = std::min(it->second.match, commit_);
  send(std::move(m));
}

void Node::broadcast_append() {
  for (auto& kv : prs_)
    if (kv.first != opt_.id) send_append(kv.first);
}

void Node::broadcast_heartbeat() {
  for (auto& kv : prs_)
    if (kv.first != opt_.id) send_heartbeat(kv.first);
}

bool Node::maybe_commit() {
  std::vector<uint64_t> m;
  for (uint64_t v : voters_) {
    if (v == opt_.id)
      m.push_back(last_index());
    else {
      auto it = prs_.find(v);
      m.push_back(it == prs_.end() ? 0 : it->second.match);
    }
  }
  if (m.empty()) return false;
  std::sort(m.begin(), m.end(), std::greater<uint64_t>());
  const uint64_t q = m[quorum() - 1];
  if (q > commit_ && term_at(q) == term_) {
    commit_ = q;
    return true;
  }
  return false;
}

void Node::append_local(std::vector<Entry> ents) {
  for (auto& e : ents) {
    log_.push_back(e);
    unstable_.push_back(e);
  }
  auto it = prs_.find(opt_.id);
  if (it != prs_.end()) {
    it->second.match = last_index();
    it->second.next = last_index() + 1;
  }
}

std::string Node::propose(uint8_t type, const std::string& data) {
  if (role_ == kLeader) {
    Entry e;
    e.term = term_;
    e.index = last_index() + 1;
    e.type = type;
    e.data = data;
    if (type == kEntryConfChange) {
      if (pending_conf_index_ > applied_) return "etcdserver: unhealthy cluster (a configuration change is pending)";
      if (opt_.check_conf) {
        std::string why = opt_.check_conf(e);
        if (!why.empty()) return why;
      }
      pending_conf_index_ = e.index;
    }
    append_local({e});
    if (maybe_commit()) {
    }
    broadcast_append();
    return "";
  }
  if (lead_ == 0) return "etcdserver: no leader";
  Message m;
  m.type = kMsgProp;
  m.to = lead_;
  Entry e;
  e.type = type;
  e.data = data;
  m.entries.push_back(std::move(e));
  send(std::move(m));
  return "";
}

void Node::tick() {
  if (role_ == kLeader) {
    ++hb_elapsed_;
    ++elapsed_;
    // ReadIndex rounds whose acks never came (dropped heartbeats, a requester
    // that re-asked with a fresh ctx) expire instead of piling up
    for (auto it = reads_.begin(); it != reads_.end();) {
      if (++it->second.age > kReadExpiryElections * opt_.election_tick) {
        read_done(it->first, 0, it->second.from, false);
        it = reads_.erase(it);
      } else {
        ++it;
      }
    }
    if (hb_elapsed_ >= opt_.heartbeat_tick) {
      hb_elapsed_ = 0;
      broadcast_heartbeat();
    }
    if (elapsed_ >= opt_.election_tick) {  // check quorum
      elapsed_ = 0;
      size_t active = 0;
      for (uint64_t v : voters_) {
        if (v == opt_.id) {
          ++active;
          continue;
        }
        auto it = prs_.find(v);
        if (it != prs_.end() && it->second.recent_active) ++active;
      }
      for (auto& kv : prs_) kv.second.recent_active = false;
      if (active < quorum()) become_follower(term_, 0);
    }
    return;
  }
  ++elapsed_;
  if (elapsed_ >= randomized_timeout_) {
    elapsed_ = 0;
    if (promotable()) campaign();
  }
}

void Node::step(const Message& m) {
  if (m.type == kMsgProp) {
    if (role_ == kLeader) {
      step_leader(m);
    } else if (lead_ != 0) {  // forward to the leader we know
      Message f = m;
      f.to = lead_;
      msgs_.push_back(f);
    }
    return;
  }
  if (m.term > term_) {
    if (m.type == kMsgVote) {
      // check-quorum lease: a follower that recently heard its leader ignores disruptive votes
      if (lead_ != 0 && elapsed_ < opt_.election_tick) return;
      become_follower(m.term, 0);
    } else if (m.type == kMsgApp || m.type == kMsgHeartbeat || m.type == kMsgSnap) {
      become_follower(m.term, m.from);
    } else {
      become_follower(m.term, 0);
    }
  } else if (m.term < term_) {
    if (m.type == kMsgApp || m.type == kMsgHeartbeat) {
      Message r;  // tell the stale leader about the new term
      r.type = kMsgAppResp;
      r.to = m.from;
      send(r);
    } else if (m.type == kMsgVote) {
      Message r;
      r.type = kMsgVoteResp;
      r.to = m.from;
      r.reject = true;
      send(r);
    }
    return;
  }
  if (m.type == kMsgVote) {
    const uint64_t lt = term_at(last_index());
    const bool up_to_date = m.log_term > lt || (m.log_term == lt && m.index >= last_index());
    const bool can_vote = vote_ == m.from || (vote_ == 0 && lead_ == 0);
    Message r;
    r.type = kMsgVoteResp;
    r.to = m.from;
    if (can_vote && up_to_date && !is_learner(opt_.id)) {
      vote_ = m.from;
      elapsed_ = 0;
    } else {
      r.reject = true;
    }
    send(r);
    return;
  }
  switch (role_) {
    case kLeader:
      step_leader(m);
      break;
    case kCandidate:
      step_candidate(m);
      break;
    default:
      step_follower(m);
  }
}

void Node::step_leader(const Message& m) {
  switch (m.type) {
    case kMsgProp: {
      for (const auto& e0 : m.entries) {
        Entry e = e0;
        e.term = term_;
        e.index = last_index() + 1;
        if (e.type == kEntryConfChange) {
          std::string why;
          if (pending_conf_index_ > applied_) why = "etcdserver: unhealthy cluster (a configuration change is pending)";
          else if (opt_.check_conf)
            why = opt_.check_conf(e);
          if (!why.empty()) {
            Message r;
            r.type = kMsgPropReject;
            r.to = m.from;
            r.context = why;
            r.entries.push_back(e0);
            send(r);
            continue;
          }
          pending_conf_index_ = e.index;
        }
        append_local({e});
      }
      maybe_commit();
      broadcast_append();
      break;
    }
    case kMsgAppResp: {
      auto it = prs_.find(m.from);
      if (it == prs_.end()) return;
      Progress& pr = it->second;
      pr.recent_active = true;
      if (m.reject) {
        pr.next = std::max<uint64_t>(1, std::min(m.index, m.reject_hint + 1));
        send_append(m.from);
      } else {
        if (m.index > pr.match) {
          pr.match = m.index;
          if (pr.next <= m.index) pr.next = m.index + 1;
          if (maybe_commit()) broadcast_append();
        }
        if (pr.match < last_index() && pr.next > last_index()) pr.next = pr.match + 1;  // lost in flight
        if (pr.next <= last_index()) send_append(m.from);
      }
      break;
    }
    case kMsgReadIndex:
      leader_read(m.context, m.from);
      break;
    case kMsgHeartbeatResp: {
      auto it = prs_.find(m.from);
      if (it == prs_.end()) return;
      it->second.recent_active = true;
      if (!m.context.empty()) {  // a ReadIndex round: count the ack
        auto rd = reads_.find(m.context);
        if (rd != reads_.end() && voters_.count(m.from)) {
          rd->second.acks.insert(m.from);
          size_t n = 0;
          for (uint64_t a : rd->second.acks) n += voters_.count(a);
          if (n >= quorum()) {
            const PendingRead pr = rd->second;
            reads_.erase(rd);
            read_done(m.context, pr.index, pr.from, true);
          }
        }
      }
      if (it->second.match < last_index()) {
        if (it->second.next > last_index()) it->second.next = it->second.match + 1;
        send_append(m.from);
      }
      break;
    }
    default:
      break;
  }
}

void Node::step_candidate(const Message& m) {
  switch (m.type) {
    case kMsgApp:
      become_follower(m.term, m.from);
      handle_append(m);
      break;
    case kMsgHeartbeat:
      become_follower(m.term, m.from);
      step_follower(m);
      break;
    case kMsgSnap:
      become_follower(m.term, m.from);
      handle_snapshot(m);
      break;
    case kMsgVoteResp:
      if (m.reject)
        votes_rejected_.insert(m.from);
      else
        votes_granted_.insert(m.from);
      if (votes_granted_.size() >= quorum())
        become_leader();
      else if (votes_rejected_.size() >= quorum())
        become_follower(term_, 0);
      break;
    case kMsgReadIndex:  // no leader to ask: the requester retries (instead of waiting out its round)
      read_done(m.context, 0, m.from, false);
      break;
    case kMsgReadIndexResp:  // an answer to a read asked while this node was a follower
      read_states_.push_back(ReadState{m.context, m.index, !m.reject});
      break;
    default:
      break;
  }
}

void Node::step_follower(const Message& m) {
  switch (m.type) {
    case kMsgApp:
      elapsed_ = 0;
      lead_ = m.from;
      handle_append(m);
      break;
    case kMsgHeartbeat: {
      elapsed_ = 0;
      lead_ = m.from;
      if (m.commit > commit_) commit_ = std::min(m.commit, last_index());
      Message r;
      r.type = kMsgHeartbeatResp;
      r.to = m.from;
      r.context = m.context;  // echo a ReadIndex round's id
      send(r);
      break;
    }
    case kMsgReadIndex:  // we are not the leader (any more): the requester retries
      read_done(m.context, 0, m.from, false);
      break;
    case kMsgReadIndexResp:
      read_states_.push_back(ReadState{m.context, m.index, !m.reject});
      break;
    case kMsgSnap:
      elapsed_ = 0;
      lead_ = m.from;
      handle_snapshot(m);
      break;
    default:
      break;
  }
}

void Node::handle_append(const Message& m) {
  Message r;
  r.type = kMsgAppResp;
  r.to = m.from;
  if (m.index < commit_) {
    r.index = commit_;
    send(r);
    return;
  }
  const bool match = m.index == 0 || (m.index <= last_index() && term_at(m.index) == m.log_term) ||
                     (m.index == snap_index_ && m.log_term == snap_term_);
  if (!match) {
    r.reject = true;
    r.index = m.index;
    r.reject_hint = last_index();
    send(r);
    return;
  }
  for (const auto& e : m.entries) {
    if (e.index <= snap_index_) continue;
    if (e.index <= last_index()) {
      if (term_at(e.index) == e.term) continue;
      log_.resize(e.index - snap_index_ - 1);  // conflict: truncate, then append
    }
    log_.push_back(e);
    unstable_.push_back(e);
  }
  const uint64_t last_new = m.index + m.entries.size();
  if (m.commit > commit_) commit_ = std::min(m.commit, last_new);
  r.index = last_new;
  send(r);
}

void Node::handle_snapshot(const Message& m) {
  Message r;
  r.type = kMsgAppResp;
  r.to = m.from;
  if (m.snap_index <= commit_) {
    r.index = commit_;
    send(r);
    return;
  }
  // adopt the snapshot: the log restarts after it
  snap_index_ = m.snap_index;
  snap_term_ = m.snap_term;
  log_.clear();
  commit_ = m.snap_index;
  applied_ = m.snap_index;
  pending_snap_ = true;
  psnap_index_ = m.snap_index;
  psnap_term_ = m.snap_term;
  psnap_data_ = m.snap_data;
  r.index = m.snap_index;
  send(r);
}

std::vector<Message> Node::take_messages() {
  std::vector<Message> out;
  out.swap(msgs_);
  return out;
}

std::vector<Entry> Node::take_unstable() {
  std::vector<Entry> out;
  out.swap(unstable_);
  return out;
}

bool Node::take_hardstate(HardState* hs) {
  HardState cur{term_, vote_, commit_};
  if (cur == last_hs_) return false;
  last_hs_ = cur;
  *hs = cur;
  return true;
}

std::vector<Entry> Node::take_committed(size_t max) {
  std::vector<Entry> out;
  while (applied_ < commit_ && out.size() < max) {
    const Entry* e = entry_at(applied_ + 1);
    if (!e) break;
    out.push_back(*e);
    ++applied_;
  }
  return out;
}

bool Node::take_snapshot(uint64_t* index, uint64_t* term, std::string* data) {
  if (!pending_snap_) return false;
  pending_snap_ = false;
  *index = psnap_index_;
  *term = psnap_term_;
  data->swap(psnap_data_);
  psnap_data_.clear();
  return true;
}

void Node::apply_conf_change(uint8_t type, uint64_t node) {
  switch (type) {
    case kAddNode:
      learners_.erase(node);
      voters_.insert(node);
      if (role_ == kLeader && !prs_.count(node)) prs_[node] = Progress{0, last_index() + 1, false, true};
      if (role_ == kLeader) prs_[node].learner = false;
      break;
    case kAddLearner:
      if (voters_.count(node)) break;
      learners_.insert(node);
      if (role_ == kLeader && !prs_.count(node)) prs_[node] = Progress{0, last_index() + 1, true, true};
      break;
    case kPromoteLearner:
      if (!learners_.count(node)) break;
      learners_.erase(node);
      voters_.insert(node);
      if (role_ == kLeader) prs_[node].learner = false;
      break;
    case kRemoveNode:
      voters_.erase(node);
      learners_.erase(node);
      prs_.erase(node);
      if (node == opt_.id && role_ == kLeader) become_follower(term_, 0);
      break;
  }
  if (role_ == kLeader && maybe_commit()) broadcast_append();
}

void Node::compact(uint64_t index) {
  if (index <= snap_index_ || index > applied_) return;
  const uint64_t t = term_at(index);
  log_.erase(log_.begin(), log_.begin() + (index - snap_index_));
  snap_index_ = index;
  snap_term_ = t;
}

}  // namespace raft
}  // namespace ptype
