// Control-plane request/response protocol shared by the member server and the
// client library (the role etcd's gRPC API plays for the reference:
// clientv3 KV / Lease / Watch / Cluster calls at cluster/registry.go:59-154,
// cluster/store.go:40-66, cluster/cluster.go:87,126,184).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "codec.hpp"
#include "mvcc.hpp"

namespace ptype {

enum Op : uint8_t {
  kOpRange = 1,
  kOpPut = 2,
  kOpDelete = 3,
  kOpLeaseGrant = 4,
  kOpLeaseRevoke = 5,
  kOpLeaseKeepAlive = 6,
  kOpLeaseTTL = 7,
  kOpWatch = 8,
  kOpWatchCancel = 9,
  kOpMemberList = 10,
  kOpMemberAdd = 11,
  kOpMemberPromote = 12,
  kOpMemberRemove = 13,
  kOpStatus = 14,
  kOpCompact = 15,
  kOpLeaseList = 16,
};

struct MemberInfo {
  uint64_t id = 0;
  std::string name;  // empty until the member has started and published itself
  std::vector<std::string> peer_urls, client_urls;
  bool is_learner = false;
};

inline void put_member(Writer& w, const MemberInfo& m) {
  w.u64(m.id);
  w.str(m.name);
  w.strs(m.peer_urls);
  w.strs(m.client_urls);
  w.b(m.is_learner);
}
inline MemberInfo get_member(Reader& r) {
  MemberInfo m;
  m.id = r.u64();
  m.name = r.str();
  m.peer_urls = r.strs();
  m.client_urls = r.strs();
  m.is_learner = r.b();
  return m;
}
inline void put_members(Writer& w, const std::vector<MemberInfo>& v) {
  w.u32((uint32_t)v.size());
  for (const auto& m : v) put_member(w, m);
}
inline std::vector<MemberInfo> get_members(Reader& r) {
  std::vector<MemberInfo> v(r.u32());
  for (auto& m : v) m = get_member(r);
  return v;
}

inline void put_kv(Writer& w, const KeyValue& kv) {
  w.str(kv.key);
  w.str(kv.value);
  w.i64(kv.create_revision);
  w.i64(kv.mod_revision);
  w.i64(kv.version);
  w.i64(kv.lease);
}
inline KeyValue get_kv(Reader& r) {
  KeyValue kv;
  kv.key = r.str();
  kv.value = r.str();
  kv.create_revision = r.i64();
  kv.mod_revision = r.i64();
  kv.version = r.i64();
  kv.lease = r.i64();
  return kv;
}
inline void put_opts(Writer& w, const RangeOpts& o) {
  w.str(o.end);
  w.i64(o.limit);
  w.i64(o.rev);
  w.u8((uint8_t)o.sort_target);
  w.u8((uint8_t)o.sort_order);
  w.b(o.serializable);
  w.b(o.keys_only);
  w.b(o.count_only);
}
inline RangeOpts get_opts(Reader& r) {
  RangeOpts o;
  o.end = r.str();
  o.limit = r.i64();
  o.rev = r.i64();
  o.sort_target = r.u8();
  o.sort_order = r.u8();
  o.serializable = r.b();
  o.keys_only = r.b();
  o.count_only = r.b();
  return o;
}
inline void put_events(Writer& w, const std::vector<Event>& ev) {
  w.u32((uint32_t)ev.size());
  for (const auto& e : ev) {
    w.u8(e.type);
    put_kv(w, e.kv);
  }
}
inline std::vector<Event> get_events(Reader& r) {
  std::vector<Event> ev(r.u32());
  for (auto& e : ev) {
    e.type = (Event::Type)r.u8();
    e.kv = get_kv(r);
  }
  return ev;
}

struct StatusInfo {
  uint64_t id = 0, leader = 0, term = 0, commit = 0, applied = 0;
  int64_t revision = 0;
  bool is_learner = false;
};

}  // namespace ptype
