#include "member.hpp"

#include <algorithm>

#include "util.hpp"

namespace ptype {

namespace {

// normal-entry apply ops (first byte after the request id)
enum ApplyOp : uint8_t {
  kApplyPut = kOpPut,
  kApplyDelete = kOpDelete,
  kApplyLeaseGrant = kOpLeaseGrant,
  kApplyLeaseRevoke = kOpLeaseRevoke,
  kApplyCompact = kOpCompact,
  kApplyNoop = 100,
  kApplyPublish = 101,
};

const char* kErrLearnerNotReady = "etcdserver: can only promote a learner member which is in sync with leader";

std::vector<std::string> sorted(std::vector<std::string> v) {
  std::sort(v.begin(), v.end());
  return v;
}

int64_t clamp_timeout(int64_t t) { return t <= 0 ? 5000 : t; }

}  // namespace

uint64_t compute_member_id(const std::vector<std::string>& peer_urls, const std::string& token, uint64_t salt) {
  std::string s = join(sorted(peer_urls), "") + token;
  if (salt) s += std::to_string(salt);
  uint64_t h = fnv1a64(s);
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 32;
  return h ? h : 1;
}

std::map<std::string, std::vector<std::string>> parse_initial_cluster(const std::string& s) {
  std::map<std::string, std::vector<std::string>> out;
  for (const auto& ent0 : split(s, ',')) {
    const std::string ent = trim(ent0);
    if (ent.empty()) continue;
    const size_t eq = ent.find('=');
    if (eq == std::string::npos) fail(Errc::kConfig, "initial-cluster: bad entry " + ent);
    out[trim(ent.substr(0, eq))].push_back(trim(ent.substr(eq + 1)));
  }
  return out;
}

// ---------------------------------------------------------------- peers
struct Member::Peer {
  uint64_t id = 0;
  std::vector<std::string> urls;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::string> q;
  bool stop = false;
  std::thread th;
  std::shared_ptr<Conn> conn;

  void run() {
    for (;;) {
      std::string frame;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || !q.empty(); });
        if (stop) return;
        frame = std::move(q.front());
        q.pop_front();
      }
      if (!conn || !conn->alive()) {
        conn.reset();
        std::vector<std::string> us;
        {
          std::lock_guard<std::mutex> g(mu);
          us = urls;
        }
        for (const auto& u : us) {
          try {
            Url p = parse_url(u);
            std::string err;
            conn = tcp_connect(p.host, p.port, 300, &err);
            if (conn) break;
          } catch (...) {
          }
        }
        if (!conn) {  // unreachable: drop what is queued (raft retransmits)
          std::unique_lock<std::mutex> g(mu);
          q.clear();
          cv.wait_for(g, std::chrono::milliseconds(100), [&] { return stop; });
          continue;
        }
      }
      if (!conn->send(frame)) conn.reset();
    }
  }
  void push(std::string f) {
    std::lock_guard<std::mutex> g(mu);
    if (q.size() > 4096) q.pop_front();
    q.push_back(std::move(f));
    cv.notify_one();
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
      cv.notify_all();
    }
    if (conn) conn->shutdown();
    if (th.joinable()) th.join();
  }
};

// ---------------------------------------------------------------- lifecycle
Member::Member(const MemberConfig& cfg) : cfg_(cfg) {
  cfg_.validate();
  // leases shorter than 1.5 election timeouts could expire during a leader change
  const int64_t min_ttl = std::max<int64_t>(1, (3 * cfg_.election_ms / 2 + 999) / 1000);
  lessor_ = Lessor(min_ttl);
}

Member::~Member() { close(); }

uint64_t Member::next_reqid() { return ((id_ & 0xffff) << 48) | (++reqseq_ & 0xffffffffffffull); }

std::string Member::save_meta_blob() const {
  Writer w;
  w.u64(id_);
  w.str(cfg_.initial_cluster_token);
  return w.buf;
}

void Member::start() {
  const std::string dir = cfg_.dir.empty() ? cfg_.name + ".etcd" : cfg_.dir;
  storage_.reset(new Storage(dir, !cfg_.unsafe_no_fsync));
  raft::Options o;
  o.election_tick = std::max<int>(2, (int)(cfg_.election_ms / std::max<int64_t>(1, cfg_.heartbeat_ms)));
  o.heartbeat_tick = 1;
  o.check_conf = [this](const raft::Entry& e) { return check_conf(e); };
  o.snapshot_source = [this](uint64_t* i, uint64_t* t, std::string* d) { snapshot_state(i, t, d); };

  Storage::Loaded L = storage_->load();
  const auto cluster = parse_initial_cluster(cfg_.effective_initial_cluster());
  if (L.any && !L.meta.empty()) {  // restart on an existing data dir
    Reader r(L.meta);
    id_ = r.u64();
    o.id = id_;
    node_.reset(new raft::Node(o));
    std::set<uint64_t> voters, learners;
    if (!L.snap_data.empty()) restore_state(L.snap_data);
    for (const auto& kv : members_) (kv.second.is_learner ? learners : voters).insert(kv.first);
    node_->restore(L.hs, L.snap_index, L.snap_term, L.entries, voters, learners, L.snap_index);
    applied_ = L.snap_index;
    last_snap_index_ = L.snap_index;
    // replay the committed tail into the state machine (members first come from conf entries)
    for (const auto& e : node_->take_committed(SIZE_MAX)) apply_entry(e);
  } else if (cfg_.cluster_state == "existing") {
    join_existing(cluster);
  } else {
    bootstrap_new(cluster);
  }
  update_peers();
  // listeners on every client and peer URL (one protocol; the split is nominal)
  std::set<std::pair<std::string, int>> bound;
  for (const auto& list : {cfg_.lcurls, cfg_.lpurls}) {
    for (const auto& u : list) {
      Url p = parse_url(u);
      if (!bound.insert({resolve_host(p.host), p.port}).second) continue;
      listeners_.emplace_back(new Listener(p.host, p.port, [this](std::shared_ptr<Conn> c) { handle_conn(c); }));
    }
  }
  last_tick_ms_ = mono_ms();
  raft_th_ = std::thread([this] { raft_loop(); });
  note_th_ = std::thread([this] { notifier_loop(); });
  if (node_->voters().size() == 1 && node_->voters().count(id_)) {
    std::lock_guard<std::mutex> g(in_mu_);
    in_cv_.notify_all();
  }
}

void Member::bootstrap_new(const std::map<std::string, std::vector<std::string>>& cluster) {
  auto it = cluster.find(cfg_.name);
  if (it == cluster.end())
    fail(Errc::kConfig, "couldn't find local name \"" + cfg_.name + "\" in the initial cluster configuration");
  if (sorted(it->second) != sorted(cfg_.apurls))
    fail(Errc::kConfig, "--initial-cluster has " + cfg_.name + "=" + join(it->second, ",") +
                            " but missing from --initial-advertise-peer-urls=" + join(cfg_.apurls, ","));
  std::vector<MemberInfo> ms;
  for (const auto& kv : cluster) {
    MemberInfo m;
    m.id = compute_member_id(kv.second, cfg_.initial_cluster_token, 0);
    m.name = kv.first;
    m.peer_urls = kv.second;
    ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end(), [](const MemberInfo& a, const MemberInfo& b) { return a.id < b.id; });
  id_ = compute_member_id(cfg_.apurls, cfg_.initial_cluster_token, 0);
  raft::Options o;
  o.id = id_;
  o.election_tick = std::max<int>(2, (int)(cfg_.election_ms / std::max<int64_t>(1, cfg_.heartbeat_ms)));
  o.check_conf = [this](const raft::Entry& e) { return check_conf(e); };
  o.snapshot_source = [this](uint64_t* i, uint64_t* t, std::string* d) { snapshot_state(i, t, d); };
  node_.reset(new raft::Node(o));
  // bootstrap entries: one committed AddNode per initial member (term 1), as etcd does
  std::vector<raft::Entry> ents;
  std::set<uint64_t> voters;
  for (size_t i = 0; i < ms.size(); ++i) {
    Writer w;
    w.u64(0);
    w.u8(raft::kAddNode);
    w.u64(ms[i].id);
    put_member(w, ms[i]);
    raft::Entry e;
    e.term = 1;
    e.index = i + 1;
    e.type = raft::kEntryConfChange;
    e.data = w.buf;
    ents.push_back(e);
    voters.insert(ms[i].id);
  }
  raft::HardState hs{1, 0, ents.size()};
  node_->restore(hs, 0, 0, ents, voters, {}, 0);
  storage_->save_meta(save_meta_blob());
  storage_->append(ents, &hs);
  for (const auto& e : node_->take_committed(SIZE_MAX)) apply_entry(e);
}

void Member::join_existing(const std::map<std::string, std::vector<std::string>>& cluster) {
  std::vector<MemberInfo> remote;
  std::string last_err = "no reachable peer";
  for (const auto& kv : cluster) {
    if (kv.first == cfg_.name) continue;
    for (const auto& u : kv.second) {
      try {
        Url p = parse_url(u);
        std::string err;
        auto c = tcp_connect(p.host, p.port, 1000, &err);
        if (!c) {
          last_err = err;
          continue;
        }
        Writer w;
        w.u8(kFrameReq);
        w.u64(1);
        w.u8(kOpMemberList);
        if (!c->send(w.buf)) continue;
        std::string resp;
        if (!c->recv(&resp)) continue;
        Reader r(resp);
        if (r.u8() != kFrameResp) continue;
        r.u64();
        const uint8_t code = r.u8();
        const std::string err2 = r.str();
        if (code) {
          last_err = err2;
          continue;
        }
        remote = get_members(r);
        break;
      } catch (const std::exception& e) {
        last_err = e.what();
      }
    }
    if (!remote.empty()) break;
  }
  if (remote.empty()) fail(Errc::kUnavailable, "cannot fetch cluster info from peer urls: " + last_err);
  for (const auto& m : remote)
    if (sorted(m.peer_urls) == sorted(cfg_.apurls)) id_ = m.id;
  if (!id_) fail(Errc::kMemberNotFound, "member " + cfg_.name + " has not been added to the cluster (peer urls " +
                                             join(cfg_.apurls, ",") + ")");
  raft::Options o;
  o.id = id_;
  o.election_tick = std::max<int>(2, (int)(cfg_.election_ms / std::max<int64_t>(1, cfg_.heartbeat_ms)));
  o.check_conf = [this](const raft::Entry& e) { return check_conf(e); };
  o.snapshot_source = [this](uint64_t* i, uint64_t* t, std::string* d) { snapshot_state(i, t, d); };
  node_.reset(new raft::Node(o));
  std::set<uint64_t> voters, learners;
  for (const auto& m : remote) (m.is_learner ? learners : voters).insert(m.id);
  node_->restore(raft::HardState{}, 0, 0, {}, voters, learners, 0);
  storage_->save_meta(save_meta_blob());
  std::lock_guard<std::mutex> g(peer_mu_);
  for (const auto& m : remote) {
    if (m.id == id_) continue;
    auto p = std::make_shared<Peer>();
    p->id = m.id;
    p->urls = m.peer_urls;
    Peer* raw = p.get();
    p->th = std::thread([raw] { raw->run(); });
    peers_[m.id] = p;
  }
}

bool Member::wait_ready(int64_t timeout_ms) {
  const int64_t until = timeout_ms < 0 ? INT64_MAX : mono_ms() + timeout_ms;
  while (!ready_.load()) {
    if (stop_.load()) return false;
    if (mono_ms() >= until) return false;
    sleep_ms(5);
  }
  return true;
}

void Member::close() {
  if (stop_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    in_cv_.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(note_mu_);
    note_cv_.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(read_mu_);
    read_cv_.notify_all();
  }
  if (raft_th_.joinable()) raft_th_.join();
  if (note_th_.joinable()) note_th_.join();
  // fail every outstanding waiter
  std::map<uint64_t, std::shared_ptr<Waiter>> ws;
  {
    std::lock_guard<std::mutex> g(wait_mu_);
    ws.swap(waiters_);
  }
  for (auto& kv : ws) {
    std::lock_guard<std::mutex> g(kv.second->mu);
    kv.second->done = true;
    kv.second->res.err = "etcdserver: server stopped";
    kv.second->res.code = Errc::kShutdown;
    kv.second->cv.notify_all();
  }
  for (auto& l : listeners_) l->close();
  listeners_.clear();
  std::map<uint64_t, std::shared_ptr<Peer>> ps;
  {
    std::lock_guard<std::mutex> g(peer_mu_);
    ps.swap(peers_);
  }
  for (auto& kv : ps) kv.second->shutdown();
  std::map<int64_t, Watcher> wt;
  {
    std::lock_guard<std::mutex> g(watch_mu_);
    wt.swap(watchers_);
  }
  for (auto& kv : wt) kv.second.fn({}, 0, true);
}

std::vector<int> Member::client_ports() const {
  std::vector<int> v;
  for (const auto& l : listeners_) v.push_back(l->port());
  return v;
}

bool Member::is_learner() {
  std::lock_guard<std::mutex> g(sm_mu_);
  auto it = members_.find(id_);
  return it != members_.end() && it->second.is_learner;
}

uint64_t Member::leader() {
  std::lock_guard<std::mutex> g(in_mu_);
  return node_ ? node_->leader() : 0;
}

StatusInfo Member::status() {
  StatusInfo s;
  s.id = id_;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    s.leader = node_->leader();
    s.term = node_->term();
    s.commit = node_->commit();
  }
  std::lock_guard<std::mutex> g(sm_mu_);
  s.applied = applied_;
  s.revision = kv_.rev();
  auto it = members_.find(id_);
  s.is_learner = it != members_.end() && it->second.is_learner;
  return s;
}

// ---------------------------------------------------------------- raft loop
void Member::raft_loop() {
  int64_t last_publish = 0;
  while (!stop_.load()) {
    Inbox in;
    {
      std::unique_lock<std::mutex> g(in_mu_);
      const int64_t wait = std::max<int64_t>(1, last_tick_ms_ + cfg_.heartbeat_ms - mono_ms());
      in_cv_.wait_for(g, std::chrono::milliseconds(wait), [&] {
        return stop_.load() || !inbox_.msgs.empty() || !inbox_.props.empty() || !inbox_.reads.empty();
      });
      std::swap(in, inbox_);
    }
    if (stop_.load()) break;
    std::unique_lock<std::mutex> lk(in_mu_);  // node_ is guarded by in_mu_ for introspection
    for (auto& m : in.msgs) {
      if (m.type == raft::kMsgPropReject) {
        for (const auto& e : m.entries) {
          if (e.data.size() < 8) continue;
          Reader r(e.data);
          ApplyResult res;
          res.err = m.context;
          res.code = m.context == kErrLearnerNotReady ? Errc::kLearnerNotReady : Errc::kGeneric;
          lk.unlock();
          resolve(r.u64(), res);
          lk.lock();
        }
        continue;
      }
      node_->step(m);
    }
    for (auto& p : in.props) {
      const std::string err = node_->propose(p.first, p.second);
      if (!err.empty() && p.second.size() >= 8) {
        Reader r(p.second);
        ApplyResult res;
        res.err = err;
        res.code = err == kErrLearnerNotReady ? Errc::kLearnerNotReady
                                              : (err.find("no leader") != std::string::npos ? Errc::kNotLeader
                                                                                            : Errc::kGeneric);
        lk.unlock();
        resolve(r.u64(), res);
        lk.lock();
      }
    }
    for (const auto& ctx : in.reads) node_->read_index(ctx);
    const int64_t now = mono_ms();
    while (now - last_tick_ms_ >= cfg_.heartbeat_ms) {
      node_->tick();
      last_tick_ms_ += cfg_.heartbeat_ms;
    }
    if (node_->voters().size() == 1 && node_->voters().count(id_) && node_->role() != raft::kLeader &&
        node_->leader() == 0)
      node_->campaign();
    // leader: revoke expired leases through the log
    if (node_->role() == raft::kLeader) {
      std::vector<int64_t> exp;
      {
        std::lock_guard<std::mutex> g(sm_mu_);
        exp = lessor_.expired(now);
      }
      for (int64_t id : exp) {
        if (revoking_.count(id)) continue;
        revoking_.insert(id);
        Writer w;
        w.u64(0);
        w.u8(kApplyLeaseRevoke);
        w.i64(id);
        node_->propose(raft::kEntryNormal, w.buf);
      }
    }
    // publish our attributes (name, client URLs) once a leader exists -> ReadyNotify
    if (!published_.load() && node_->leader() != 0 && now - last_publish > 1000) {
      last_publish = now;
      Writer w;
      w.u64(0);
      w.u8(kApplyPublish);
      w.u64(id_);
      w.str(cfg_.name);
      w.strs(cfg_.acurls);
      node_->propose(raft::kEntryNormal, w.buf);
    }
    lk.unlock();
    process_ready();
    if (!ready_.load() && published_.load() && leader() != 0) ready_.store(true);
  }
}

void Member::process_ready() {
  std::unique_lock<std::mutex> lk(in_mu_);
  uint64_t si, st;
  std::string sd;
  if (node_->take_snapshot(&si, &st, &sd)) {
    {
      std::lock_guard<std::mutex> g(sm_mu_);
      restore_state(sd);
      applied_ = si;
    }
    raft::HardState hs{node_->term(), 0, node_->commit()};
    storage_->save_snapshot(si, st, sd, hs, {});
    last_snap_index_ = si;
  }
  std::vector<raft::Entry> ents = node_->take_unstable();
  raft::HardState hs;
  const bool hs_changed = node_->take_hardstate(&hs);
  storage_->append(ents, hs_changed ? &hs : nullptr);
  std::vector<raft::Message> msgs = node_->take_messages();
  std::vector<raft::Entry> committed = node_->take_committed();
  std::vector<raft::ReadState> reads = node_->take_read_states();
  const bool is_leader = node_->role() == raft::kLeader;
  lk.unlock();
  for (const auto& m : msgs) send_raft(m);
  for (const auto& e : committed) apply_entry(e);
  {
    std::lock_guard<std::mutex> g(read_mu_);
    for (const auto& rs : reads) {
      auto it = read_waiters_.find(rs.ctx);
      if (it == read_waiters_.end()) continue;
      it->second.done = true;
      it->second.ok = rs.ok;
      it->second.index = rs.index;
    }
    {
      std::lock_guard<std::mutex> g2(sm_mu_);
      applied_pub_.store(applied_);
    }
  }
  read_cv_.notify_all();
  if (is_leader != was_leader_) {
    std::lock_guard<std::mutex> g(sm_mu_);
    if (is_leader) {
      lessor_.promote(mono_ms());
      revoking_.clear();
    } else {
      lessor_.demote();
    }
    was_leader_ = is_leader;
  }
  maybe_snapshot();
  if (!committed.empty()) {  // entries applied may have produced new messages (conf changes)
    std::lock_guard<std::mutex> g(in_mu_);
    for (const auto& m : node_->take_messages()) send_raft(m);
  }
}

void Member::send_raft(const raft::Message& m) {
  std::shared_ptr<Peer> p;
  {
    std::lock_guard<std::mutex> g(peer_mu_);
    auto it = peers_.find(m.to);
    if (it == peers_.end()) return;
    p = it->second;
  }
  Writer w;
  w.u8(kFrameRaft);
  w.u64(0);
  w.raw(nullptr, 0);
  std::string f = w.buf + m.encode();
  p->push(std::move(f));
}

void Member::update_peers() {
  std::map<uint64_t, std::vector<std::string>> want;
  {
    std::lock_guard<std::mutex> g(sm_mu_);
    for (const auto& kv : members_)
      if (kv.first != id_) want[kv.first] = kv.second.peer_urls;
  }
  std::lock_guard<std::mutex> g(peer_mu_);
  for (const auto& kv : want) {
    auto it = peers_.find(kv.first);
    if (it != peers_.end()) {
      std::lock_guard<std::mutex> pg(it->second->mu);
      it->second->urls = kv.second;
      continue;
    }
    auto p = std::make_shared<Peer>();
    p->id = kv.first;
    p->urls = kv.second;
    Peer* raw = p.get();
    p->th = std::thread([raw] { raw->run(); });
    peers_[kv.first] = p;
  }
}

std::string Member::check_conf(const raft::Entry& e) {
  Reader r(e.data);
  r.u64();
  const uint8_t t = r.u8();
  const uint64_t node = r.u64();
  if (t != raft::kPromoteLearner) return "";
  auto it = members_.find(node);
  if (it == members_.end() || !it->second.is_learner) return "";  // the applier reports the error
  const auto& prs = node_->progress();
  auto pit = prs.find(node);
  const uint64_t leader_match = node_->last_index();
  const uint64_t learner_match = pit == prs.end() ? 0 : pit->second.match;
  if ((double)learner_match < (double)leader_match * 0.9) return kErrLearnerNotReady;
  return "";
}

// ---------------------------------------------------------------- apply
void Member::apply_entry(const raft::Entry& e) {
  if (e.data.size() < 8) {  // leader's empty entry
    std::lock_guard<std::mutex> g(sm_mu_);
    applied_ = e.index;
    return;
  }
  Reader r(e.data);
  const uint64_t reqid = r.u64();
  ApplyResult res;
  std::vector<Event> ev;
  int64_t rev = 0;
  bool conf = false;
  {
    std::lock_guard<std::mutex> g(sm_mu_);
    if (e.type == raft::kEntryConfChange) {
      conf = true;
      const std::string body = e.data.substr(8);
      apply_conf(reqid, body, &res);
    } else {
      const uint8_t op = r.u8();
      try {
        switch (op) {
          case kApplyPut: {
            const std::string key = r.str(), val = r.str();
            const int64_t lease = r.i64();
            if (lease != 0 && !lessor_.exists(lease)) {
              res.err = "etcdserver: requested lease not found";
              res.code = Errc::kLeaseNotFound;
              break;
            }
            RangeOpts o;
            auto old = kv_.range(key, o);
            if (!old.kvs.empty() && old.kvs[0].lease) lessor_.detach(old.kvs[0].lease, key);
            res.rev = kv_.put(key, val, lease, &ev);
            if (lease) lessor_.attach(lease, key);
            break;
          }
          case kApplyDelete: {
            const std::string key = r.str(), end = r.str();
            RangeOpts o;
            o.end = end;
            o.keys_only = true;
            auto old = kv_.range(key, o);
            res.rev = kv_.delete_range(key, end, &res.deleted, &ev);
            for (const auto& kv : old.kvs)
              if (kv.lease) lessor_.detach(kv.lease, kv.key);
            break;
          }
          case kApplyLeaseGrant: {
            const int64_t id = r.i64(), ttl = r.i64();
            res.lease_id = id;
            res.ttl = lessor_.grant(id, ttl, mono_ms());
            res.rev = kv_.rev();
            break;
          }
          case kApplyLeaseRevoke: {
            const int64_t id = r.i64();
            if (!lessor_.exists(id)) {
              res.err = "etcdserver: requested lease not found";
              res.code = Errc::kLeaseNotFound;
              break;
            }
            for (const auto& k : lessor_.revoke(id)) {
              int64_t d = 0;
              kv_.delete_range(k, "", &d, &ev);
            }
            revoking_.erase(id);
            res.rev = kv_.rev();
            break;
          }
          case kApplyCompact:
            kv_.compact(r.i64());
            res.rev = kv_.rev();
            break;
          case kApplyNoop:
            res.rev = kv_.rev();
            break;
          case kApplyPublish: {
            const uint64_t mid = r.u64();
            const std::string name = r.str();
            const auto curls = r.strs();
            auto it = members_.find(mid);
            if (it != members_.end()) {
              it->second.name = name;
              it->second.client_urls = curls;
            }
            if (mid == id_) published_.store(true);
            break;
          }
          default:
            res.err = "unknown apply op";
        }
      } catch (const Error& x) {
        res.err = x.what();
        res.code = x.code();
      }
    }
    applied_ = e.index;
    rev = kv_.rev();
  }
  if (conf && res.err.empty() && res.conf_type >= 0) {
    {
      std::lock_guard<std::mutex> g(in_mu_);
      node_->apply_conf_change((uint8_t)res.conf_type, res.member_id);
    }
    update_peers();
  }
  if (!ev.empty()) publish_events(std::move(ev), rev);
  if (reqid) resolve(reqid, std::move(res));
}

void Member::apply_conf(uint64_t reqid, const std::string& body, ApplyResult* res) {
  (void)reqid;
  Reader r(body);
  const uint8_t t = r.u8();
  const uint64_t node = r.u64();
  MemberInfo info = get_member(r);
  auto list = [&] {
    std::vector<MemberInfo> v;
    for (const auto& kv : members_) v.push_back(kv.second);
    return v;
  };
  switch (t) {
    case raft::kAddNode:
    case raft::kAddLearner: {
      if (members_.count(node)) {
        if (t == raft::kAddNode) {  // bootstrap replay on restart
          res->conf_type = t;
          res->member_id = node;
          return;
        }
        res->err = "etcdserver: member ID already exist";
        res->code = Errc::kMemberExists;
        return;
      }
      for (const auto& kv : members_)
        for (const auto& u : kv.second.peer_urls)
          for (const auto& v : info.peer_urls)
            if (u == v) {
              res->err = "etcdserver: Peer URLs already exists";
              res->code = Errc::kMemberExists;
              return;
            }
      info.id = node;
      info.is_learner = t == raft::kAddLearner;
      members_[node] = info;
      break;
    }
    case raft::kPromoteLearner: {
      auto it = members_.find(node);
      if (it == members_.end()) {
        res->err = "etcdserver: member not found";
        res->code = Errc::kMemberNotFound;
        return;
      }
      if (!it->second.is_learner) {
        res->err = "etcdserver: can only promote a learner member";
        return;
      }
      it->second.is_learner = false;
      break;
    }
    case raft::kRemoveNode: {
      if (!members_.erase(node)) {
        res->err = "etcdserver: member not found";
        res->code = Errc::kMemberNotFound;
        return;
      }
      break;
    }
  }
  res->conf_type = t;  // raft's conf state is updated by apply_entry, outside sm_mu_
  res->member_id = node;
  res->members = list();
}

void Member::resolve(uint64_t reqid, ApplyResult r) {
  std::shared_ptr<Waiter> w;
  {
    std::lock_guard<std::mutex> g(wait_mu_);
    auto it = waiters_.find(reqid);
    if (it == waiters_.end()) return;
    w = it->second;
    waiters_.erase(it);
  }
  std::lock_guard<std::mutex> g(w->mu);
  w->res = std::move(r);
  w->done = true;
  w->cv.notify_all();
}

void Member::read_barrier(int64_t timeout_ms) {
  if (stop_.load()) fail(Errc::kShutdown, "etcdserver: server stopped");
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(clamp_timeout(timeout_ms));
  for (;;) {
    const std::string ctx = std::to_string(id_) + "/" + std::to_string(++read_seq_);
    {
      std::lock_guard<std::mutex> g(read_mu_);
      read_waiters_[ctx] = ReadWaiter{};
    }
    {
      std::lock_guard<std::mutex> g(in_mu_);
      inbox_.reads.push_back(ctx);
      in_cv_.notify_all();
    }
    std::unique_lock<std::mutex> g(read_mu_);
    // a round that gets no answer (leader lost, message dropped) is retried
    const auto round_end = std::min(deadline, std::chrono::steady_clock::now() +
                                                  std::chrono::milliseconds(std::max<int64_t>(50, 4 * cfg_.heartbeat_ms)));
    read_cv_.wait_until(g, round_end, [&] { return read_waiters_[ctx].done || stop_.load(); });
    const ReadWaiter w = read_waiters_[ctx];
    read_waiters_.erase(ctx);
    if (w.done && w.ok) {
      // serve once this member's state machine has caught up with the read index
      if (!read_cv_.wait_until(g, deadline, [&] { return applied_pub_.load() >= w.index || stop_.load(); }))
        fail(Errc::kTimeout, "etcdserver: request timed out");
      if (stop_.load()) fail(Errc::kShutdown, "etcdserver: server stopped");
      ++reads_served_;
      return;
    }
    if (stop_.load()) fail(Errc::kShutdown, "etcdserver: server stopped");
    if (std::chrono::steady_clock::now() >= deadline) fail(Errc::kTimeout, "etcdserver: request timed out");
    g.unlock();
    if (w.done) sleep_ms(std::max<int64_t>(1, cfg_.heartbeat_ms / 2));  // no leader / no term commit yet
  }
}

ApplyResult Member::propose_wait(uint8_t etype, uint8_t op, const std::string& payload, int64_t timeout_ms) {
  if (stop_.load()) fail(Errc::kShutdown, "etcdserver: server stopped");
  auto w = std::make_shared<Waiter>();
  const uint64_t reqid = next_reqid();
  {
    std::lock_guard<std::mutex> g(wait_mu_);
    waiters_[reqid] = w;
  }
  Writer d;
  d.u64(reqid);
  d.u8(op);
  d.buf += payload;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    inbox_.props.emplace_back(etype, std::move(d.buf));
    in_cv_.notify_all();
  }
  std::unique_lock<std::mutex> g(w->mu);
  if (!w->cv.wait_for(g, std::chrono::milliseconds(clamp_timeout(timeout_ms)), [&] { return w->done; })) {
    std::lock_guard<std::mutex> g2(wait_mu_);
    waiters_.erase(reqid);
    fail(Errc::kTimeout, "etcdserver: request timed out");
  }
  if (!w->res.err.empty()) fail(w->res.code, w->res.err);
  return w->res;
}

// ---------------------------------------------------------------- snapshots
void Member::snapshot_state(uint64_t* index, uint64_t* term, std::string* data) {
  // called on the raft thread (leader shipping to a lagging follower) or by maybe_snapshot
  std::lock_guard<std::mutex> g(sm_mu_);
  Writer w;
  w.u64(applied_);
  w.str(kv_.serialize());
  w.str(lessor_.serialize());
  std::vector<MemberInfo> v;
  for (const auto& kv : members_) v.push_back(kv.second);
  put_members(w, v);
  *index = applied_;
  *term = node_->term_at(applied_);
  if (*term == 0) *term = node_->snap_term();
  *data = w.buf;
}

void Member::restore_state(const std::string& data) {
  Reader r(data);
  applied_ = r.u64();
  kv_.restore(r.str());
  lessor_.restore(r.str(), mono_ms());
  members_.clear();
  std::set<uint64_t> voters, learners;
  for (const auto& m : get_members(r)) {
    members_[m.id] = m;
    (m.is_learner ? learners : voters).insert(m.id);
    if (m.id == id_ && !m.name.empty()) published_.store(true);
  }
  if (node_) node_->bootstrap(voters, learners);
}

void Member::maybe_snapshot() {
  uint64_t applied;
  {
    std::lock_guard<std::mutex> g(sm_mu_);
    applied = applied_;
  }
  if (applied < last_snap_index_ + cfg_.snapshot_count) return;
  uint64_t idx, term;
  std::string data;
  std::vector<raft::Entry> tail;
  raft::HardState hs;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    snapshot_state(&idx, &term, &data);
    for (uint64_t i = idx + 1; i <= node_->last_index(); ++i)
      if (auto* e = node_->entry_at(i)) tail.push_back(*e);
    hs = raft::HardState{node_->term(), 0, node_->commit()};
  }
  storage_->save_snapshot(idx, term, data, hs, tail);
  last_snap_index_ = idx;
  std::lock_guard<std::mutex> g(in_mu_);
  // entries kept in memory for slow followers (etcd's SnapshotCatchUpEntries);
  // anyone further behind gets the snapshot
  const uint64_t keep = std::min<uint64_t>(5000, std::max<uint64_t>(1, cfg_.snapshot_count / 2));
  if (idx > keep) node_->compact(idx - keep);
}

// ---------------------------------------------------------------- watch
void Member::publish_events(std::vector<Event> ev, int64_t rev) {
  std::lock_guard<std::mutex> g(note_mu_);
  notes_.emplace_back(std::move(ev), rev);
  note_cv_.notify_all();
}

void Member::notifier_loop() {
  while (!stop_.load()) {
    std::pair<std::vector<Event>, int64_t> n;
    {
      std::unique_lock<std::mutex> g(note_mu_);
      note_cv_.wait_for(g, std::chrono::milliseconds(100), [&] { return stop_.load() || !notes_.empty(); });
      if (notes_.empty()) continue;
      n = std::move(notes_.front());
      notes_.pop_front();
    }
    std::vector<std::pair<int64_t, WatchFn>> targets;
    std::vector<std::vector<Event>> batches;
    {
      std::lock_guard<std::mutex> g(watch_mu_);
      for (auto& kv : watchers_) {
        std::vector<Event> mine;
        for (const auto& e : n.first)
          if (e.kv.mod_revision >= kv.second.next_rev && range_contains(kv.second.key, kv.second.end, e.kv.key))
            mine.push_back(e);
        if (mine.empty()) continue;
        kv.second.next_rev = mine.back().kv.mod_revision + 1;
        targets.emplace_back(kv.first, kv.second.fn);
        batches.push_back(std::move(mine));
      }
    }
    for (size_t i = 0; i < targets.size(); ++i) targets[i].second(batches[i], n.second, false);
  }
}

int64_t Member::watch(const std::string& key, const std::string& end, int64_t start_rev, WatchFn fn) {
  const int64_t wid = ++watch_seq_;
  std::vector<Event> replay;
  int64_t rev0;
  {
    std::lock_guard<std::mutex> g(sm_mu_);
    rev0 = kv_.rev();
    if (start_rev > 0 && start_rev <= rev0) replay = kv_.events_since(start_rev, key, end);
    std::lock_guard<std::mutex> g2(watch_mu_);
    Watcher w;
    w.key = key;
    w.end = end;
    w.fn = fn;
    w.next_rev = std::max(rev0 + 1, start_rev);
    watchers_[wid] = w;
  }
  if (!replay.empty()) fn(replay, rev0, false);
  return wid;
}

void Member::cancel_watch(int64_t wid) {
  WatchFn fn;
  {
    std::lock_guard<std::mutex> g(watch_mu_);
    auto it = watchers_.find(wid);
    if (it == watchers_.end()) return;
    fn = it->second.fn;
    watchers_.erase(it);
  }
  fn({}, 0, true);
}

// ---------------------------------------------------------------- local API
RangeResult Member::range(const std::string& key, const RangeOpts& o, int64_t timeout_ms) {
  if (!o.serializable) read_barrier(timeout_ms);  // linearizable: ReadIndex, not a log write
  std::lock_guard<std::mutex> g(sm_mu_);
  return kv_.range(key, o);
}

int64_t Member::put(const std::string& key, const std::string& value, int64_t lease, int64_t timeout_ms) {
  Writer w;
  w.str(key);
  w.str(value);
  w.i64(lease);
  return propose_wait(raft::kEntryNormal, kApplyPut, w.buf, timeout_ms).rev;
}

int64_t Member::del(const std::string& key, const std::string& end, int64_t* deleted, int64_t timeout_ms) {
  Writer w;
  w.str(key);
  w.str(end);
  ApplyResult r = propose_wait(raft::kEntryNormal, kApplyDelete, w.buf, timeout_ms);
  if (deleted) *deleted = r.deleted;
  return r.rev;
}

int64_t Member::lease_grant(int64_t ttl, int64_t id, int64_t* granted_ttl, int64_t timeout_ms) {
  if (id == 0) {
    const uint64_t hi = (id_ & 0x7fff) << 48;
    id = (int64_t)(hi | (((uint64_t)mono_us() & 0xffffffffull) << 16) | ((uint64_t)(++lease_seq_) & 0xffff));
    if (id == 0) id = 1;
  }
  Writer w;
  w.i64(id);
  w.i64(ttl);
  ApplyResult r = propose_wait(raft::kEntryNormal, kApplyLeaseGrant, w.buf, timeout_ms);
  if (granted_ttl) *granted_ttl = r.ttl;
  return r.lease_id;
}

void Member::lease_revoke(int64_t id, int64_t timeout_ms) {
  Writer w;
  w.i64(id);
  propose_wait(raft::kEntryNormal, kApplyLeaseRevoke, w.buf, timeout_ms);
}

int64_t Member::lease_keepalive(int64_t id) {
  int64_t ttl;
  bool leader_here;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    leader_here = node_->role() == raft::kLeader;
  }
  {
    std::lock_guard<std::mutex> g(sm_mu_);
    ttl = lessor_.renew(id, mono_ms());
  }
  if (ttl < 0) fail(Errc::kLeaseNotFound, "etcdserver: requested lease not found");
  if (!leader_here) {  // the leader tracks deadlines: forward the renewal
    raft::Message m;
    m.type = raft::kMsgLeaseRenew;
    m.from = id_;
    m.to = leader();
    m.context = std::to_string(id);
    if (m.to) send_raft(m);
  }
  return ttl;
}

int64_t Member::lease_ttl(int64_t id) {
  std::lock_guard<std::mutex> g(sm_mu_);
  return lessor_.remaining_ms(id, mono_ms());
}

std::vector<LeaseInfo> Member::lease_list() {
  std::lock_guard<std::mutex> g(sm_mu_);
  return lessor_.list();
}

void Member::compact(int64_t rev, int64_t timeout_ms) {
  Writer w;
  w.i64(rev);
  propose_wait(raft::kEntryNormal, kApplyCompact, w.buf, timeout_ms);
}

std::vector<MemberInfo> Member::member_list() {
  std::lock_guard<std::mutex> g(sm_mu_);
  std::vector<MemberInfo> v;
  for (const auto& kv : members_) v.push_back(kv.second);
  return v;
}

MemberInfo Member::member_add(const std::vector<std::string>& peer_urls, bool learner,
                              std::vector<MemberInfo>* members, int64_t timeout_ms) {
  for (const auto& u : peer_urls) parse_url(u);
  const uint64_t nid = compute_member_id(peer_urls, cfg_.initial_cluster_token, (uint64_t)mono_us());
  MemberInfo info;
  info.id = nid;
  info.peer_urls = peer_urls;
  info.is_learner = learner;
  Writer w;
  w.u64(nid);
  put_member(w, info);
  ApplyResult r =
      propose_wait(raft::kEntryConfChange, learner ? raft::kAddLearner : raft::kAddNode, w.buf, timeout_ms);
  if (members) *members = r.members;
  return info;
}

void Member::member_promote(uint64_t nid, int64_t timeout_ms) {
  Writer w;
  w.u64(nid);
  put_member(w, MemberInfo{});
  propose_wait(raft::kEntryConfChange, raft::kPromoteLearner, w.buf, timeout_ms);
}

void Member::member_remove(uint64_t nid, int64_t timeout_ms) {
  Writer w;
  w.u64(nid);
  put_member(w, MemberInfo{});
  propose_wait(raft::kEntryConfChange, raft::kRemoveNode, w.buf, timeout_ms);
}

// ---------------------------------------------------------------- TCP server
void Member::handle_conn(std::shared_ptr<Conn> c) {
  auto conn_watches = std::make_shared<std::set<int64_t>>();
  auto wmu = std::make_shared<std::mutex>();
  std::atomic<int> inflight{0};
  std::string frame;
  while (!stop_.load() && c->recv(&frame)) {
    Reader r(frame);
    const uint8_t kind = r.u8();
    const uint64_t rid = r.u64();
    if (kind == kFrameRaft) {
      raft::Message m = raft::Message::decode(frame.substr(r.i));
      if (m.type == raft::kMsgLeaseRenew) {
        std::lock_guard<std::mutex> g(sm_mu_);
        lessor_.renew(atoll(m.context.c_str()), mono_ms());
        continue;
      }
      std::lock_guard<std::mutex> g(in_mu_);
      inbox_.msgs.push_back(std::move(m));
      in_cv_.notify_all();
      continue;
    }
    if (kind != kFrameReq) continue;
    const uint8_t op = r.u8();
    std::string body = frame.substr(r.i);
    ++inflight;
    std::thread([this, c, rid, op, body, conn_watches, wmu, &inflight] {
      Writer w;
      w.u8(kFrameResp);
      w.u64(rid);
      try {
        Reader br(body);
        std::set<int64_t> added;
        std::string payload = handle_request(op, br, c, &added);
        if (!added.empty()) {
          std::lock_guard<std::mutex> g(*wmu);
          conn_watches->insert(added.begin(), added.end());
        }
        w.u8(0);
        w.str("");
        w.buf += payload;
      } catch (const Error& e) {
        w.u8((uint8_t)e.code());
        w.str(e.what());
      } catch (const std::exception& e) {
        w.u8((uint8_t)Errc::kGeneric);
        w.str(e.what());
      }
      c->send(w.buf);
      --inflight;
    }).detach();
  }
  c->shutdown();
  while (inflight.load() > 0) sleep_ms(1);
  std::set<int64_t> ws;
  {
    std::lock_guard<std::mutex> g(*wmu);
    ws.swap(*conn_watches);
  }
  for (int64_t wid : ws) cancel_watch(wid);
}

std::string Member::handle_request(uint8_t op, Reader& r, const std::shared_ptr<Conn>& c,
                                   std::set<int64_t>* conn_watches) {
  Writer w;
  switch (op) {
    case kOpRange: {
      const std::string key = r.str();
      RangeOpts o = get_opts(r);
      RangeResult res = range(key, o);
      w.i64(res.rev);
      w.i64(res.count);
      w.b(res.more);
      w.u32((uint32_t)res.kvs.size());
      for (const auto& kv : res.kvs) put_kv(w, kv);
      break;
    }
    case kOpPut: {
      const std::string key = r.str(), val = r.str();
      w.i64(put(key, val, r.i64()));
      break;
    }
    case kOpDelete: {
      const std::string key = r.str(), end = r.str();
      int64_t d = 0;
      const int64_t rev = del(key, end, &d);
      w.i64(d);
      w.i64(rev);
      break;
    }
    case kOpLeaseGrant: {
      const int64_t ttl = r.i64(), id = r.i64();
      int64_t g = 0;
      w.i64(lease_grant(ttl, id, &g));
      w.i64(g);
      break;
    }
    case kOpLeaseRevoke:
      lease_revoke(r.i64());
      break;
    case kOpLeaseKeepAlive:
      w.i64(lease_keepalive(r.i64()));
      break;
    case kOpLeaseTTL:
      w.i64(lease_ttl(r.i64()));
      break;
    case kOpLeaseList: {
      auto v = lease_list();
      w.u32((uint32_t)v.size());
      for (const auto& l : v) {
        w.i64(l.id);
        w.i64(l.ttl);
      }
      break;
    }
    case kOpWatch: {
      const uint64_t client_wid = r.u64();
      const std::string key = r.str(), end = r.str();
      const int64_t start = r.i64();
      std::weak_ptr<Conn> wc = c;
      const int64_t wid = watch(key, end, start, [wc, client_wid](const std::vector<Event>& ev, int64_t rev, bool canceled) {
        auto conn = wc.lock();
        if (!conn) return;
        Writer f;
        f.u8(kFrameEvent);
        f.u64(client_wid);
        f.i64(rev);
        f.b(canceled);
        put_events(f, ev);
        conn->send(f.buf);
      });
      conn_watches->insert(wid);
      w.i64(wid);
      break;
    }
    case kOpWatchCancel:
      cancel_watch(r.i64());
      break;
    case kOpMemberList:
      put_members(w, member_list());
      break;
    case kOpMemberAdd: {
      const auto urls = r.strs();
      const bool learner = r.b();
      std::vector<MemberInfo> ms;
      MemberInfo m = member_add(urls, learner, &ms);
      put_member(w, m);
      put_members(w, ms);
      break;
    }
    case kOpMemberPromote:
      member_promote(r.u64());
      break;
    case kOpMemberRemove:
      member_remove(r.u64());
      break;
    case kOpStatus: {
      StatusInfo s = status();
      w.u64(s.id);
      w.u64(s.leader);
      w.u64(s.term);
      w.u64(s.commit);
      w.u64(s.applied);
      w.i64(s.revision);
      w.b(s.is_learner);
      break;
    }
    case kOpCompact:
      compact(r.i64());
      break;
    default:
      fail("unknown op " + std::to_string(op));
  }
  return w.buf;
}

}  // namespace ptype
