#include "mvcc.hpp"

#include <algorithm>

#include "codec.hpp"
#include "util.hpp"

namespace ptype {

// ---------------------------------------------------------------- crc32c
namespace {
struct Crc32cTable {
  uint32_t t[256];
  Crc32cTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0x82F63B78u ^ (c >> 1) : c >> 1;
      t[i] = c;
    }
  }
};
}  // namespace

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  // magic static: initialised once, thread-safe (several members may start
  // concurrently in one process; TSan flagged the old lazy flag)
  static const Crc32cTable tab;
  const uint32_t* table = tab.t;
  crc = ~crc;
  const unsigned char* p = (const unsigned char*)data;
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

bool range_contains(const std::string& key, const std::string& end, const std::string& k) {
  if (end.empty()) return k == key;
  if (end == std::string(1, '\0')) return k >= key;
  return k >= key && k < end;
}

std::string prefix_range_end(const std::string& prefix) {
  std::string end = prefix;
  for (int i = (int)end.size() - 1; i >= 0; --i) {
    if ((unsigned char)end[i] < 0xff) {
      end[i] = (char)((unsigned char)end[i] + 1);
      return end.substr(0, i + 1);
    }
  }
  return std::string(1, '\0');  // no prefix end (e.g. 0xffff): from-key
}

// ---------------------------------------------------------------- MvccStore
const MvccStore::Version* MvccStore::at(const std::vector<Version>& h, int64_t rev) const {
  for (auto it = h.rbegin(); it != h.rend(); ++it)
    if (it->mod <= rev) return it->tomb ? nullptr : &*it;
  return nullptr;
}

RangeResult MvccStore::range(const std::string& key, const RangeOpts& o) const {
  RangeResult r;
  r.rev = rev_;
  const int64_t rev = o.rev > 0 ? o.rev : rev_;
  if (rev > rev_) fail(Errc::kGeneric, "mvcc: required revision is a future revision");
  if (o.rev > 0 && o.rev < compact_rev_) fail(Errc::kCompacted, "mvcc: required revision has been compacted");
  auto emit = [&](const std::string& k, const std::vector<Version>& h) {
    const Version* v = at(h, rev);
    if (!v) return;
    ++r.count;
    if (o.count_only) return;
    KeyValue kv;
    kv.key = k;
    if (!o.keys_only) kv.value = v->value;
    kv.create_revision = v->create;
    kv.mod_revision = v->mod;
    kv.version = v->ver;
    kv.lease = v->lease;
    r.kvs.push_back(std::move(kv));
  };
  if (o.end.empty()) {
    auto it = idx_.find(key);
    if (it != idx_.end()) emit(it->first, it->second);
  } else {
    const bool from_key = o.end == std::string(1, '\0');
    for (auto it = idx_.lower_bound(key); it != idx_.end(); ++it) {
      if (!from_key && it->first >= o.end) break;
      emit(it->first, it->second);
    }
  }
  // etcd: a non-key sort target with no order sorts ascending by that target
  int order = o.sort_order;
  if (o.sort_target != kSortKey && order == kSortNone) order = kSortAscend;
  if (order != kSortNone && !(o.sort_target == kSortKey && order == kSortAscend)) {
    auto cmp = [&](const KeyValue& a, const KeyValue& b) {
      switch (o.sort_target) {
        case kSortVersion: return a.version < b.version;
        case kSortCreate: return a.create_revision < b.create_revision;
        case kSortMod: return a.mod_revision < b.mod_revision;
        case kSortValue: return a.value < b.value;
        default: return a.key < b.key;
      }
    };
    std::stable_sort(r.kvs.begin(), r.kvs.end(), cmp);
    if (order == kSortDescend) std::reverse(r.kvs.begin(), r.kvs.end());
  }
  if (o.limit > 0 && (int64_t)r.kvs.size() > o.limit) {
    r.kvs.resize(o.limit);
    r.more = true;
  }
  return r;
}

int64_t MvccStore::put(const std::string& key, const std::string& value, int64_t lease, std::vector<Event>* ev) {
  const int64_t rev = ++rev_;
  auto& h = idx_[key];
  Version v;
  v.mod = rev;
  v.lease = lease;
  v.value = value;
  if (!h.empty() && !h.back().tomb) {
    v.create = h.back().create;
    v.ver = h.back().ver + 1;
  } else {
    v.create = rev;
    v.ver = 1;
  }
  h.push_back(v);
  if (ev) {
    Event e;
    e.type = Event::kPut;
    e.kv = KeyValue{key, value, v.create, v.mod, v.ver, v.lease};
    ev->push_back(std::move(e));
  }
  return rev;
}

int64_t MvccStore::delete_range(const std::string& key, const std::string& end, int64_t* deleted,
                                std::vector<Event>* ev, std::vector<std::string>* deleted_keys) {
  std::vector<std::string> keys;
  if (end.empty()) {
    auto it = idx_.find(key);
    if (it != idx_.end() && !it->second.empty() && !it->second.back().tomb) keys.push_back(key);
  } else {
    const bool from_key = end == std::string(1, '\0');
    for (auto it = idx_.lower_bound(key); it != idx_.end(); ++it) {
      if (!from_key && it->first >= end) break;
      if (!it->second.empty() && !it->second.back().tomb) keys.push_back(it->first);
    }
  }
  if (deleted) *deleted = (int64_t)keys.size();
  if (keys.empty()) return rev_;
  const int64_t rev = ++rev_;
  for (const auto& k : keys) {
    auto& h = idx_[k];
    Version v;
    v.mod = rev;
    v.tomb = true;
    v.lease = h.back().lease;
    h.push_back(v);
    if (ev) {
      Event e;
      e.type = Event::kDelete;
      e.kv.key = k;
      e.kv.mod_revision = rev;
      ev->push_back(std::move(e));
    }
    if (deleted_keys) deleted_keys->push_back(k);
  }
  return rev;
}

void MvccStore::compact(int64_t rev) {
  if (rev <= compact_rev_) return;
  if (rev > rev_) fail(Errc::kGeneric, "mvcc: required revision is a future revision");
  for (auto it = idx_.begin(); it != idx_.end();) {
    auto& h = it->second;
    // keep the latest version <= rev (unless a tombstone) and everything newer
    size_t keep_from = 0;
    for (size_t i = 0; i < h.size(); ++i)
      if (h[i].mod <= rev) keep_from = i;
    if (!h.empty() && h[keep_from].mod <= rev && h[keep_from].tomb) ++keep_from;
    h.erase(h.begin(), h.begin() + std::min(keep_from, h.size()));
    if (h.empty())
      it = idx_.erase(it);
    else
      ++it;
  }
  compact_rev_ = rev;
}

std::vector<Event> MvccStore::events_since(int64_t from_rev, const std::string& key, const std::string& end) const {
  if (from_rev > 0 && from_rev <= compact_rev_) fail(Errc::kCompacted, "mvcc: required revision has been compacted");
  std::vector<std::pair<int64_t, Event>> out;
  auto visit = [&](const std::string& k, const std::vector<Version>& h) {
    for (size_t i = 0; i < h.size(); ++i) {
      const Version& v = h[i];
      if (v.mod < from_rev) continue;
      Event e;
      e.type = v.tomb ? Event::kDelete : Event::kPut;
      e.kv.key = k;
      e.kv.mod_revision = v.mod;
      if (!v.tomb) {
        e.kv.value = v.value;
        e.kv.create_revision = v.create;
        e.kv.version = v.ver;
        e.kv.lease = v.lease;
      }
      out.emplace_back(v.mod, std::move(e));
    }
  };
  if (end.empty()) {
    auto it = idx_.find(key);
    if (it != idx_.end()) visit(it->first, it->second);
  } else {
    const bool from_key = end == std::string(1, '\0');
    for (auto it = idx_.lower_bound(key); it != idx_.end(); ++it) {
      if (!from_key && it->first >= end) break;
      visit(it->first, it->second);
    }
  }
  std::stable_sort(out.begin(), out.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<Event> ev;
  for (auto& p : out) ev.push_back(std::move(p.second));
  return ev;
}

size_t MvccStore::key_count() const {
  size_t n = 0;
  for (const auto& kv : idx_)
    if (!kv.second.empty() && !kv.second.back().tomb) ++n;
  return n;
}

std::string MvccStore::serialize() const {
  Writer w;
  w.u32(0x4d564343);  // "MVCC"
  w.i64(rev_);
  w.i64(compact_rev_);
  w.u64(idx_.size());
  for (const auto& kv : idx_) {
    w.str(kv.first);
    w.u32((uint32_t)kv.second.size());
    for (const auto& v : kv.second) {
      w.i64(v.mod);
      w.i64(v.create);
      w.i64(v.ver);
      w.i64(v.lease);
      w.b(v.tomb);
      w.str(v.value);
    }
  }
  return w.buf;
}

void MvccStore::restore(const std::string& data) {
  Reader r(data);
  if (r.u32() != 0x4d564343) fail("mvcc: bad snapshot magic");
  idx_.clear();
  rev_ = r.i64();
  compact_rev_ = r.i64();
  const uint64_t n = r.u64();
  for (uint64_t i = 0; i < n; ++i) {
    std::string k = r.str();
    auto& h = idx_[k];
    const uint32_t m = r.u32();
    h.resize(m);
    for (uint32_t j = 0; j < m; ++j) {
      h[j].mod = r.i64();
      h[j].create = r.i64();
      h[j].ver = r.i64();
      h[j].lease = r.i64();
      h[j].tomb = r.b();
      h[j].value = r.str();
    }
  }
}

// ---------------------------------------------------------------- Lessor
int64_t Lessor::grant(int64_t id, int64_t ttl, int64_t now_ms) {
  if (leases_.count(id)) fail(Errc::kGeneric, "etcdserver: lease already exists");
  LeaseInfo l;
  l.id = id;
  l.ttl = std::max(ttl, min_ttl_);
  l.expiry_ms = primary_ ? now_ms + l.ttl * 1000 : 0;
  leases_[id] = l;
  return l.ttl;
}

std::set<std::string> Lessor::revoke(int64_t id) {
  auto it = leases_.find(id);
  if (it == leases_.end()) fail(Errc::kLeaseNotFound, "etcdserver: requested lease not found");
  std::set<std::string> keys = it->second.keys;
  leases_.erase(it);
  return keys;
}

int64_t Lessor::renew(int64_t id, int64_t now_ms) {
  auto it = leases_.find(id);
  if (it == leases_.end()) return -1;
  if (primary_) it->second.expiry_ms = now_ms + it->second.ttl * 1000;
  return it->second.ttl;
}

int64_t Lessor::remaining_ms(int64_t id, int64_t now_ms) const {
  auto it = leases_.find(id);
  if (it == leases_.end()) return -1;
  if (!primary_ || it->second.expiry_ms == 0) return it->second.ttl * 1000;
  return std::max<int64_t>(0, it->second.expiry_ms - now_ms);
}

void Lessor::attach(int64_t id, const std::string& key) {
  auto it = leases_.find(id);
  if (it != leases_.end()) it->second.keys.insert(key);
}

void Lessor::detach(int64_t id, const std::string& key) {
  auto it = leases_.find(id);
  if (it != leases_.end()) it->second.keys.erase(key);
}

std::vector<int64_t> Lessor::expired(int64_t now_ms) const {
  std::vector<int64_t> out;
  if (!primary_) return out;
  for (const auto& kv : leases_)
    if (kv.second.expiry_ms && kv.second.expiry_ms <= now_ms) out.push_back(kv.first);
  return out;
}

void Lessor::promote(int64_t now_ms) {
  primary_ = true;
  for (auto& kv : leases_) kv.second.expiry_ms = now_ms + kv.second.ttl * 1000;
}

void Lessor::demote() {
  primary_ = false;
  for (auto& kv : leases_) kv.second.expiry_ms = 0;
}

std::vector<LeaseInfo> Lessor::list() const {
  std::vector<LeaseInfo> v;
  for (const auto& kv : leases_) v.push_back(kv.second);
  return v;
}

std::string Lessor::serialize() const {
  Writer w;
  w.u64(leases_.size());
  for (const auto& kv : leases_) {
    w.i64(kv.first);
    w.i64(kv.second.ttl);
    w.u32((uint32_t)kv.second.keys.size());
    for (const auto& k : kv.second.keys) w.str(k);
  }
  return w.buf;
}

void Lessor::restore(const std::string& data, int64_t now_ms) {
  Reader r(data);
  leases_.clear();
  const uint64_t n = r.u64();
  for (uint64_t i = 0; i < n; ++i) {
    LeaseInfo l;
    l.id = r.i64();
    l.ttl = r.i64();
    const uint32_t m = r.u32();
    for (uint32_t j = 0; j < m; ++j) l.keys.insert(r.str());
    l.expiry_ms = primary_ ? now_ms + l.ttl * 1000 : 0;
    leases_[l.id] = l;
  }
}

}  // namespace ptype
