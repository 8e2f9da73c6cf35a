// RegistryFollower / ShardLease (follower.hpp).
#include "follower.hpp"

#include <algorithm>
#include <chrono>

#include "json.hpp"

namespace ptype {

namespace {
std::string prefix_end(const std::string& p) {
  std::string e = p;
  e.back() = (char)(e.back() + 1);
  return e;
}

int64_t want_int(const JValue& o, const char* k, int64_t dflt, bool required) {
  const JValue* v = o.get(k);
  if (!v) {
    if (required) fail(Errc::kGeneric, std::string("shard record: no \"") + k + "\"");
    return dflt;
  }
  if (v->kind != JValue::kNumber) fail(Errc::kGeneric, std::string("shard record: \"") + k + "\" is not a number");
  return v->is_int ? (int64_t)v->i : (int64_t)v->num;
}
}  // namespace

ShardRecord ShardRecord::parse(const std::string& json) {
  const JValue v = json_parse(json);
  if (v.kind != JValue::kObject) fail(Errc::kGeneric, "shard record: not an object");
  ShardRecord r;
  r.rank = want_int(v, "rank", 0, true);
  r.world = want_int(v, "world", 1, true);
  r.count = want_int(v, "count", 0, true);
  r.gen = want_int(v, "gen", 0, false);
  if (const JValue* b = v.get("blocks"); b && b->kind == JValue::kArray)
    for (const auto& x : b->arr) r.blocks.push_back(x.is_int ? (int64_t)x.i : (int64_t)x.num);
  if (r.world < 1 || r.count < 0) fail(Errc::kGeneric, "shard record: bad geometry");
  r.json = json;
  return r;
}

void ShardRecord::actors(std::vector<int64_t>* ids, std::vector<int32_t>* mbox) const {
  const std::vector<int64_t> bl = blocks.empty() ? std::vector<int64_t>{rank} : blocks;
  ids->clear();
  mbox->clear();
  ids->reserve((size_t)(count * (int64_t)bl.size()));
  mbox->reserve(ids->capacity());
  for (size_t j = 0; j < bl.size(); ++j)
    for (int64_t k = 0; k < count; ++k) {
      ids->push_back(bl[j] + world * k);
      mbox->push_back((int32_t)((int64_t)j * count + k));
    }
}

// ---------------------------------------------------------------- RegistryFollower
RegistryFollower::RegistryFollower(std::shared_ptr<KvClient> kv, const std::string& prefix, int64_t ttl_ms,
                                   int64_t grace_ms, double relist_s, bool watch)
    : kv_(std::move(kv)), prefix_(prefix), end_(prefix_end(prefix)), ttl_ms_(ttl_ms), grace_ms_(grace_ms),
      relist_s_(relist_s) {
  if (prefix_.empty()) throw std::invalid_argument("RegistryFollower: empty prefix");
  RangeOpts o;
  o.end = end_;
  const RangeResult res = kv_->get(prefix_, o);
  const int64_t now = mono_ms();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& x : res.kvs) {
      try {
        pending_.push_back({true, x.key, ShardRecord::parse(x.value)});
        seen_[x.key] = now;
      } catch (const std::exception&) {  // a malformed record routes nothing
      }
    }
  }
  version_.fetch_add(1, std::memory_order_release);
  ctx_ = Context::with_cancel(Context::background());
  watching_ = watch;
  if (watch) watch_ = kv_->watch(ctx_, prefix_, end_, res.rev + 1);
  th_ = std::thread([this] { run(); });
}

RegistryFollower::~RegistryFollower() { close(); }

void RegistryFollower::close() {
  if (stop_.exchange(true)) return;
  if (ctx_) ctx_->cancel();
  if (th_.joinable()) th_.join();
}

void RegistryFollower::run() {
  auto next_list = std::chrono::steady_clock::now() + std::chrono::milliseconds((int64_t)(relist_s_ * 1000));
  const int64_t poll_ms = std::max<int64_t>(1, std::min<int64_t>(100, (int64_t)(relist_s_ * 1000)));
  while (!stop_.load()) {
    if (watch_ && !watch_->closed()) {
      bool closed = false;
      auto resp = watch_->recv(poll_ms, &closed);
      if (resp && !resp->events.empty()) {
        const int64_t now = mono_ms();
        std::lock_guard<std::mutex> g(mu_);
        for (const Event& ev : resp->events) {
          if (ev.type == Event::kPut) {
            try {
              pending_.push_back({true, ev.kv.key, ShardRecord::parse(ev.kv.value)});
              seen_[ev.kv.key] = now;
            } catch (const std::exception&) {
            }
          } else {
            pending_.push_back({false, ev.kv.key, {}});
            seen_.erase(ev.kv.key);
          }
          events_.fetch_add(1);
        }
        version_.fetch_add(1, std::memory_order_release);
      }
    } else if (ctx_->wait(poll_ms)) {
      break;
    }
    if (std::chrono::steady_clock::now() >= next_list) {
      next_list = std::chrono::steady_clock::now() + std::chrono::milliseconds((int64_t)(relist_s_ * 1000));
      relist();
    }
  }
}

// A full re-list (the reference re-lists on every event, cluster/registry.go:131):
// refreshes every listed shard's liveness and queues what the watch missed -- a
// key never applied, a record that changed since it was applied (or queued), a
// key gone -- and re-opens a watch that closed, from just past the listing.
void RegistryFollower::relist() {
  RangeResult res;
  try {
    RangeOpts o;
    o.end = end_;
    res = kv_->get(prefix_, o, 2000);
  } catch (const std::exception&) {
    return;  // control plane electing: keep the last view; the K6 deadlines keep running
  }
  const int64_t now = mono_ms();
  if (watching_ && watch_ && watch_->closed() && !stop_.load()) {
    try {
      watch_ = kv_->watch(ctx_, prefix_, end_, res.rev + 1);
      ++watch_reopens_;
    } catch (const std::exception&) {
    }
  }
  std::map<std::string, const KeyValue*> listed;
  for (const auto& x : res.kvs) listed[x.key] = &x;
  std::lock_guard<std::mutex> g(mu_);
  // the newest queued operation on k (nullptr: none) -- what take() will leave applied
  auto last_queued = [&](const std::string& k) -> const Pending* {
    for (auto it = pending_.rbegin(); it != pending_.rend(); ++it)
      if (it->key == k) return &*it;
    return nullptr;
  };
  for (const auto& [k, x] : listed) {
    seen_[k] = now;
    // shards_ belongs to take(); a missed PUT is detected against what was queued or applied
    const Pending* q = last_queued(k);
    const auto a = applied_json_.find(k);
    const std::string* have = q ? (q->put ? &q->rec.json : nullptr) : (a != applied_json_.end() ? &a->second : nullptr);
    if (!have || *have != x->value) {
      try {
        pending_.push_back({true, k, ShardRecord::parse(x->value)});
      } catch (const std::exception&) {
      }
    }
  }
  for (const auto& [k, json] : applied_json_) {
    (void)json;
    const Pending* q = last_queued(k);
    if (!listed.count(k) && (!q || q->put)) {
      pending_.push_back({false, k, {}});  // a missed DELETE
      seen_.erase(k);
    }
  }
  relists_.fetch_add(1);
  version_.fetch_add(1, std::memory_order_release);
}

void RegistryFollower::put(const std::string& key, const ShardRecord& rec, int64_t deadline,
                           std::vector<MirrorOp>* ops) {
  if (rec.gen < min_gen_) return;
  auto it = shards_.find(key);
  if (it != shards_.end() && it->second.rec.json != rec.json) del(key, ops);
  MirrorOp op;
  op.kind = MirrorOp::kUpsert;
  op.key = key;
  op.rank = (int32_t)rec.rank;
  op.deadline_ms = deadline;
  rec.actors(&op.ids, &op.mbox);
  ops->push_back(std::move(op));
  shards_[key] = Applied{rec, deadline};
}

void RegistryFollower::del(const std::string& key, std::vector<MirrorOp>* ops) {
  auto it = shards_.find(key);
  if (it == shards_.end()) return;
  MirrorOp op;
  op.kind = MirrorOp::kDelete;
  op.key = key;
  std::vector<int32_t> unused;
  it->second.rec.actors(&op.ids, &unused);
  ops->push_back(std::move(op));
  shards_.erase(it);
}

std::vector<MirrorOp> RegistryFollower::take(int64_t now_ms, bool* sweep, int64_t* changed) {
  std::vector<MirrorOp> ops;
  *sweep = false;
  *changed = 0;
  if (quiet(now_ms)) return ops;
  std::vector<Pending> todo;
  std::map<std::string, int64_t> seen;
  uint64_t version;
  {
    std::lock_guard<std::mutex> g(mu_);
    todo.swap(pending_);
    seen = seen_;
    version = version_.load(std::memory_order_acquire);
  }
  for (const Pending& p : todo) {
    if (p.put) {
      auto s = seen.find(p.key);
      put(p.key, p.rec, (s != seen.end() ? s->second : now_ms) + ttl_ms_ + grace_ms_, &ops);
    } else {
      del(p.key, &ops);
    }
    ++*changed;
  }
  // K6: deadlines of shards seen alive since refreshed (re-upserted when they
  // moved by more than half a TTL); the rest expire at their deadline
  std::vector<std::string> keys;
  for (const auto& kv : shards_) keys.push_back(kv.first);
  for (const std::string& k : keys) {
    auto s = seen.find(k);
    const int64_t dl = (s != seen.end() ? s->second : 0) + ttl_ms_ + grace_ms_;
    Applied& a = shards_[k];
    if (dl - a.deadline > ttl_ms_ / 2) {
      const ShardRecord rec = a.rec;
      put(k, rec, dl, &ops);
    }
  }
  const size_t before = shards_.size();
  for (auto it = shards_.begin(); it != shards_.end();) {
    if (it->second.deadline < now_ms) {
      *sweep = true;  // the device sweep tombstones its actors (their entries carry the deadline)
      it = shards_.erase(it);
    } else {
      ++it;
    }
  }
  *changed += (int64_t)(before - shards_.size());
  if (*changed) ++applies_;
  applied_ = version;
  int64_t nx = now_ms + ttl_ms_;
  bool any = false;
  for (const auto& kv : shards_) {
    nx = any ? std::min(nx, kv.second.deadline) : kv.second.deadline;
    any = true;
  }
  next_expiry_ = nx;
  {
    std::lock_guard<std::mutex> g(mu_);
    applied_json_.clear();
    for (const auto& kv : shards_) applied_json_[kv.first] = kv.second.rec.json;
  }
  return ops;
}

void RegistryFollower::set_generation(int64_t gen) {
  {
    std::lock_guard<std::mutex> g(mu_);
    min_gen_ = gen;
    pending_.erase(std::remove_if(pending_.begin(), pending_.end(),
                                  [&](const Pending& p) { return p.put && p.rec.gen < gen; }),
                   pending_.end());
  }
  for (auto it = shards_.begin(); it != shards_.end();) {
    if (it->second.rec.gen < gen) it = shards_.erase(it);
    else ++it;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    applied_json_.clear();
    for (const auto& kv : shards_) applied_json_[kv.first] = kv.second.rec.json;
  }
  version_.fetch_add(1, std::memory_order_release);
}

std::vector<std::tuple<std::string, std::string, int64_t>> RegistryFollower::shards() const {
  std::vector<std::tuple<std::string, std::string, int64_t>> out;
  for (const auto& kv : shards_) out.emplace_back(kv.first, kv.second.rec.json, kv.second.deadline);
  return out;
}

int64_t RegistryFollower::actors() const {
  int64_t n = 0;
  for (const auto& kv : shards_) n += kv.second.rec.n_actors();
  return n;
}

// ---------------------------------------------------------------- ShardLease
ShardLease::ShardLease(std::shared_ptr<KvClient> kv, const std::string& key, const std::string& record_json,
                       int64_t ttl_s)
    : kv_(std::move(kv)), key_(key), record_(record_json) {
  int64_t granted = 0;
  lease_ = kv_->grant(ttl_s, &granted);
  kv_->put(key_, record_, lease_);
  ctx_ = Context::with_cancel(Context::background());
  ka_ = kv_->keepalive(ctx_, lease_);
  auto ka = ka_;
  th_ = std::thread([ka] {  // drain the keepalive responses until the stream closes
    for (;;) {
      bool closed = false;
      auto r = ka->recv(1000, &closed);
      if (!r && (closed || ka->closed())) break;
    }
  });
}

ShardLease::~ShardLease() {
  try {
    close();
  } catch (...) {
  }
}

void ShardLease::update(const std::string& record_json) {
  record_ = record_json;
  kv_->put(key_, record_, lease_);
}

void ShardLease::stop_keepalive() {
  if (ctx_) ctx_->cancel();
}

void ShardLease::close() {
  if (closed_) return;
  closed_ = true;
  if (ctx_) ctx_->cancel();
  try {
    kv_->revoke(lease_, 2000);
  } catch (const std::exception&) {
  }
  if (th_.joinable()) th_.join();
}

}  // namespace ptype
