#include "kvclient.hpp"

#include "config.hpp"

namespace ptype {

KvClient::KvClient(std::vector<std::string> endpoints, int64_t dial_timeout_ms)
    : eps_(std::move(endpoints)), dial_timeout_ms_(dial_timeout_ms) {}

KvClient::~KvClient() { close(); }

void KvClient::close() {
  if (closed_.exchange(true)) return;
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> g(mu_);
    c = conn_;
  }
  if (c) drop_conn(c, "client closed");
  std::vector<std::thread> rs, as;
  {
    std::lock_guard<std::mutex> g(mu_);
    rs.swap(readers_);
    as.swap(aux_);
  }
  for (auto& t : rs)
    if (t.joinable()) t.join();
  for (auto& t : as)
    if (t.joinable()) t.join();
}

std::shared_ptr<Conn> KvClient::ensure_conn(int64_t timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  if (closed_.load()) fail(Errc::kShutdown, "client: closed");
  if (conn_ && conn_->alive()) return conn_;
  std::string last = "no endpoints";
  for (const auto& ep : eps_) {
    if (ep.empty()) continue;
    try {
      Url u = parse_url(ep.find("://") == std::string::npos ? "http://" + ep : ep);
      std::string err;
      auto c = tcp_connect(u.host, u.port, std::min(dial_timeout_ms_, timeout_ms), &err);
      if (!c) {
        last = err;
        continue;
      }
      conn_ = c;
      readers_.emplace_back([this, c] { reader(c); });
      return c;
    } catch (const std::exception& e) {
      last = e.what();
    }
  }
  fail(Errc::kUnavailable, "all endpoints unavailable: " + last);
}

void KvClient::reader(std::shared_ptr<Conn> c) {
  std::string f;
  while (c->recv(&f)) {
    try {
      Reader r(f);
      const uint8_t kind = r.u8();
      const uint64_t id = r.u64();
      if (kind == kFrameResp) {
        std::shared_ptr<Pending> p;
        {
          std::lock_guard<std::mutex> g(mu_);
          auto it = pending_.find(id);
          if (it == pending_.end()) continue;
          p = it->second;
          pending_.erase(it);
        }
        std::lock_guard<std::mutex> g(p->mu);
        p->code = r.u8();
        p->err = r.str();
        p->payload = f.substr(r.i);
        p->done = true;
        p->cv.notify_all();
      } else if (kind == kFrameEvent) {
        WatchResponse w;
        w.revision = r.i64();
        w.canceled = r.b();
        w.events = get_events(r);
        std::shared_ptr<Channel<WatchResponse>> ch;
        {
          std::lock_guard<std::mutex> g(mu_);
          auto it = watches_.find(id);
          if (it == watches_.end()) continue;
          ch = it->second;
          if (w.canceled) watches_.erase(it);
        }
        const bool canceled = w.canceled;
        ch->try_send(std::move(w));
        if (canceled) ch->close();
      }
    } catch (const std::exception&) {
    }
  }
  drop_conn(c, "connection lost");
}

void KvClient::drop_conn(const std::shared_ptr<Conn>& c, const std::string& why) {
  c->shutdown();
  std::map<uint64_t, std::shared_ptr<Pending>> ps;
  std::map<uint64_t, std::shared_ptr<Channel<WatchResponse>>> ws;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (conn_ == c) conn_.reset();
    ps.swap(pending_);
    ws.swap(watches_);
  }
  for (auto& kv : ps) {
    std::lock_guard<std::mutex> g(kv.second->mu);
    kv.second->done = true;
    kv.second->code = (uint8_t)Errc::kUnavailable;
    kv.second->err = why;
    kv.second->cv.notify_all();
  }
  for (auto& kv : ws) {
    WatchResponse w;
    w.canceled = true;
    w.err = "watch stream broken: " + why;
    kv.second->try_send(std::move(w));
    kv.second->close();
  }
}

// Requests rejected with "no leader" were never appended to the log, so they are
// retried (with backoff) until the call's deadline, as clientv3's retry policy
// does for Unavailable: an election in progress is not an error to the caller.
std::string KvClient::call(uint8_t op, const std::string& payload, int64_t timeout_ms) {
  const int64_t budget = timeout_ms <= 0 ? 5000 : timeout_ms;
  const int64_t deadline = mono_ms() + budget;
  int64_t backoff = 10;
  for (;;) {
    const int64_t left = deadline - mono_ms();
    try {
      return call_once(op, payload, std::max<int64_t>(1, left));
    } catch (const Error& e) {
      if (e.code() != Errc::kNotLeader || mono_ms() + backoff >= deadline) throw;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(backoff));
    backoff = std::min<int64_t>(backoff * 2, 200);
  }
}

std::string KvClient::call_once(uint8_t op, const std::string& payload, int64_t timeout_ms) {
  auto c = ensure_conn(timeout_ms);
  auto p = std::make_shared<Pending>();
  const uint64_t id = ++seq_;
  {
    std::lock_guard<std::mutex> g(mu_);
    pending_[id] = p;
  }
  Writer w;
  w.u8(kFrameReq);
  w.u64(id);
  w.u8(op);
  w.buf += payload;
  if (!c->send(w.buf)) {
    drop_conn(c, "send failed");
    fail(Errc::kUnavailable, "client: send failed");
  }
  std::unique_lock<std::mutex> g(p->mu);
  if (!p->cv.wait_for(g, std::chrono::milliseconds(timeout_ms <= 0 ? 5000 : timeout_ms), [&] { return p->done; })) {
    std::lock_guard<std::mutex> g2(mu_);
    pending_.erase(id);
    fail(Errc::kTimeout, "context deadline exceeded");
  }
  if (p->code) fail((Errc)p->code, p->err);
  return p->payload;
}

RangeResult KvClient::get(const std::string& key, const RangeOpts& o, int64_t timeout_ms) {
  Writer w;
  w.str(key);
  put_opts(w, o);
  const std::string resp = call(kOpRange, w.buf, timeout_ms);
  Reader r(resp);
  RangeResult res;
  res.rev = r.i64();
  res.count = r.i64();
  res.more = r.b();
  const uint32_t n = r.u32();
  for (uint32_t i = 0; i < n; ++i) res.kvs.push_back(get_kv(r));
  return res;
}

int64_t KvClient::put(const std::string& key, const std::string& value, int64_t lease, int64_t timeout_ms) {
  Writer w;
  w.str(key);
  w.str(value);
  w.i64(lease);
  const std::string resp = call(kOpPut, w.buf, timeout_ms);
  Reader r(resp);
  return r.i64();
}

int64_t KvClient::del(const std::string& key, const std::string& end, int64_t* deleted, int64_t timeout_ms) {
  Writer w;
  w.str(key);
  w.str(end);
  const std::string resp = call(kOpDelete, w.buf, timeout_ms);
  Reader r(resp);
  const int64_t d = r.i64();
  if (deleted) *deleted = d;
  return r.i64();
}

int64_t KvClient::grant(int64_t ttl, int64_t* granted_ttl, int64_t timeout_ms) {
  Writer w;
  w.i64(ttl);
  w.i64(0);
  const std::string resp = call(kOpLeaseGrant, w.buf, timeout_ms);
  Reader r(resp);
  const int64_t id = r.i64();
  const int64_t t = r.i64();
  if (granted_ttl) *granted_ttl = t;
  return id;
}

void KvClient::revoke(int64_t id, int64_t timeout_ms) {
  Writer w;
  w.i64(id);
  call(kOpLeaseRevoke, w.buf, timeout_ms);
}

int64_t KvClient::keepalive_once(int64_t id, int64_t timeout_ms) {
  Writer w;
  w.i64(id);
  const std::string resp = call(kOpLeaseKeepAlive, w.buf, timeout_ms);
  Reader r(resp);
  return r.i64();
}

int64_t KvClient::time_to_live_ms(int64_t id, int64_t timeout_ms) {
  Writer w;
  w.i64(id);
  const std::string resp = call(kOpLeaseTTL, w.buf, timeout_ms);
  Reader r(resp);
  return r.i64();
}

void KvClient::compact(int64_t rev, int64_t timeout_ms) {
  Writer w;
  w.i64(rev);
  call(kOpCompact, w.buf, timeout_ms);
}

std::vector<MemberInfo> KvClient::member_list(int64_t timeout_ms) {
  const std::string resp = call(kOpMemberList, "", timeout_ms);
  Reader r(resp);
  return get_members(r);
}

MemberInfo KvClient::member_add(const std::vector<std::string>& peer_urls, bool learner,
                                std::vector<MemberInfo>* members, int64_t timeout_ms) {
  Writer w;
  w.strs(peer_urls);
  w.b(learner);
  const std::string resp = call(kOpMemberAdd, w.buf, timeout_ms);
  Reader r(resp);
  MemberInfo m = get_member(r);
  auto ms = get_members(r);
  if (members) *members = ms;
  return m;
}

void KvClient::member_promote(uint64_t id, int64_t timeout_ms) {
  Writer w;
  w.u64(id);
  call(kOpMemberPromote, w.buf, timeout_ms);
}

void KvClient::member_remove(uint64_t id, int64_t timeout_ms) {
  Writer w;
  w.u64(id);
  call(kOpMemberRemove, w.buf, timeout_ms);
}

StatusInfo KvClient::status(int64_t timeout_ms) {
  const std::string resp = call(kOpStatus, "", timeout_ms);
  Reader r(resp);
  StatusInfo s;
  s.id = r.u64();
  s.leader = r.u64();
  s.term = r.u64();
  s.commit = r.u64();
  s.applied = r.u64();
  s.revision = r.i64();
  s.is_learner = r.b();
  return s;
}

std::shared_ptr<Channel<int64_t>> KvClient::keepalive(const Ctx& ctx, int64_t id) {
  auto ch = std::make_shared<Channel<int64_t>>(16);
  // the thread never owns the client: close() joins it (a last-reference drop
  // on this thread would make close() join itself)
  std::lock_guard<std::mutex> g(mu_);
  if (closed_.load()) fail(Errc::kShutdown, "client: closed");
  aux_.emplace_back([this, ctx, id, ch] {
    int64_t ttl = 2;
    int failures = 0;
    for (;;) {
      if (closed_.load() || (ctx && ctx->done())) break;
      try {
        ttl = keepalive_once(id, 2000);
        failures = 0;
        ch->try_send(ttl);
      } catch (const Error& e) {
        if (e.code() == Errc::kLeaseNotFound || e.code() == Errc::kShutdown || ++failures > 3) break;
      }
      // renew at ttl/3 like clientv3, waking early on cancel / close
      const int64_t until = mono_ms() + std::max<int64_t>(100, ttl * 1000 / 3);
      bool stop = false;
      while (!stop && mono_ms() < until) {
        if (closed_.load() || (ctx && ctx->done())) stop = true;
        else sleep_ms(20);
      }
      if (stop) break;
    }
    ch->close();
  });
  return ch;
}

std::shared_ptr<Channel<WatchResponse>> KvClient::watch(const Ctx& ctx, const std::string& key, const std::string& end,
                                                        int64_t start_rev) {
  auto ch = std::make_shared<Channel<WatchResponse>>(1u << 20);
  auto c = ensure_conn(dial_timeout_ms_);
  const uint64_t wid = ++seq_;
  {
    std::lock_guard<std::mutex> g(mu_);
    watches_[wid] = ch;
  }
  Writer w;
  w.u64(wid);
  w.str(key);
  w.str(end);
  w.i64(start_rev);
  int64_t server_wid = 0;
  try {
    const std::string resp = call(kOpWatch, w.buf, 5000);
    Reader r(resp);
    server_wid = r.i64();
  } catch (...) {
    std::lock_guard<std::mutex> g(mu_);
    watches_.erase(wid);
    throw;
  }
  if (ctx) {
    std::weak_ptr<KvClient> self = shared_from_this();
    ctx->on_done([self, wid, server_wid, ch] {
      ch->close();
      auto cli = self.lock();
      if (!cli) return;
      {
        std::lock_guard<std::mutex> g(cli->mu_);
        cli->watches_.erase(wid);
        if (cli->closed_.load()) return;
        // cancel server-side asynchronously (never block the canceling thread);
        // the thread does not own the client, close() joins it
        KvClient* raw = cli.get();
        cli->aux_.emplace_back([raw, server_wid] {
          if (raw->closed_.load()) return;
          try {
            Writer w2;
            w2.i64(server_wid);
            raw->call(kOpWatchCancel, w2.buf, 1000);
          } catch (...) {
          }
        });
      }
    });
  }
  return ch;
}

}  // namespace ptype
