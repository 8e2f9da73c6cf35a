// Data-plane communicator lifecycle and rank-failure handling (dataplane.hpp).
#include "dataplane.hpp"

#include <dlfcn.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <set>
#include <stdexcept>

#include "json.hpp"

namespace ptype {

namespace {

// ---- RCCL / HIP entry points, resolved from the libraries already in the process
struct NcclUid {  // ncclUniqueId: NCCL_UNIQUE_ID_BYTES opaque bytes, passed by value
  char internal[128];
};
struct Api {
  int (*get_uid)(NcclUid*) = nullptr;
  int (*init_rank)(void**, int, NcclUid, int) = nullptr;
  int (*abort)(void*) = nullptr;
  int (*async_error)(void*, int*) = nullptr;
  int (*allreduce)(const void*, void*, size_t, int, int, void*, void*) = nullptr;
  int (*send)(const void*, size_t, int, int, void*, void*) = nullptr;
  int (*recv)(void*, size_t, int, int, void*, void*) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  const char* (*errstr)(int) = nullptr;
  int (*set_device)(int) = nullptr;
  int (*hmalloc)(void**, size_t) = nullptr;
  int (*hfree)(void*) = nullptr;
  int (*memcpy_)(void*, const void*, size_t, int) = nullptr;
  int (*stream_create)(void**, unsigned) = nullptr;
  int (*stream_sync)(void*) = nullptr;
  int (*stream_query)(void*) = nullptr;
  int (*stream_destroy)(void*) = nullptr;
  int (*event_create)(void**, unsigned) = nullptr;
  int (*event_record)(void*, void*) = nullptr;
  int (*event_query)(void*) = nullptr;
  int (*event_destroy)(void*) = nullptr;

  template <class F>
  static void bind(F& f, void* h, const char* name) {
    if (!f) f = reinterpret_cast<F>(dlsym(h, name));
  }
  void bind_all(void* h) {
    bind(get_uid, h, "ncclGetUniqueId");
    bind(init_rank, h, "ncclCommInitRank");
    bind(abort, h, "ncclCommAbort");
    bind(async_error, h, "ncclCommGetAsyncError");
    bind(allreduce, h, "ncclAllReduce");
    bind(send, h, "ncclSend");
    bind(recv, h, "ncclRecv");
    bind(group_start, h, "ncclGroupStart");
    bind(group_end, h, "ncclGroupEnd");
    bind(errstr, h, "ncclGetErrorString");
    bind(set_device, h, "hipSetDevice");
    bind(hmalloc, h, "hipMalloc");
    bind(hfree, h, "hipFree");
    bind(memcpy_, h, "hipMemcpy");
    bind(stream_create, h, "hipStreamCreateWithFlags");
    bind(stream_sync, h, "hipStreamSynchronize");
    bind(stream_query, h, "hipStreamQuery");
    bind(stream_destroy, h, "hipStreamDestroy");
    bind(event_create, h, "hipEventCreateWithFlags");
    bind(event_record, h, "hipEventRecord");
    bind(event_query, h, "hipEventQuery");
    bind(event_destroy, h, "hipEventDestroy");
  }
  Api() {
    bind_all(RTLD_DEFAULT);
    for (const char* lib : {"librccl.so", "librccl.so.1", "libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"}) {
      if (ok()) break;
      void* h = dlopen(lib, RTLD_NOW | RTLD_NOLOAD);  // only what the process already loaded
      if (h) bind_all(h);
    }
  }
  bool hip_ok() const {
    return set_device && hmalloc && hfree && memcpy_ && stream_create && stream_sync && stream_query &&
           stream_destroy && event_create && event_record && event_query && event_destroy;
  }
  bool ok() const {
    return get_uid && init_rank && abort && async_error && allreduce && send && recv && group_start && group_end &&
           hip_ok();
  }
};
Api& api() {
  static Api a;
  return a;
}
Api& need() {
  Api& a = api();
  if (!a.ok()) throw std::runtime_error("DataPlane: RCCL / HIP not loaded in this process (import the device runtime)");
  return a;
}
void nccl_check(int rc, const char* what) {
  if (rc != 0)
    throw std::runtime_error(std::string("DataPlane: ") + what + " failed: " +
                             (api().errstr ? api().errstr(rc) : std::to_string(rc)));
}
void hip_check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("DataPlane: ") + what + " failed: hip error " + std::to_string(rc));
}
constexpr int kNcclUint64 = 5, kNcclInt8 = 0, kNcclMax = 2, kNcclInProgress = 7;
constexpr int kHipH2D = 1, kHipD2H = 2, kHipD2D = 3, kHipNotReady = 600;

std::string hex(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t b = static_cast<const uint8_t*>(p)[i];
    s += d[b >> 4];
    s += d[b & 15];
  }
  return s;
}
bool unhex(const std::string& s, void* out, size_t n) {
  if (s.size() != 2 * n) return false;
  auto v = [](char c) { return c >= 'a' ? c - 'a' + 10 : c - '0'; };
  for (size_t i = 0; i < n; ++i) static_cast<uint8_t*>(out)[i] = (uint8_t)(v(s[2 * i]) << 4 | v(s[2 * i + 1]));
  return true;
}
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

bool DataPlane::available() { return api().ok(); }

DataPlane::DataPlane(std::shared_ptr<EtcdRegistry> registry, std::shared_ptr<KvClient> kv, std::string service,
                     std::string me, int device, double timeout_s)
    : reg_(std::move(registry)), kv_(std::move(kv)), service_(std::move(service)), me_(std::move(me)),
      device_(device), timeout_s_(timeout_s) {
  (void)need();  // (the device is taken at form(): a member's rank -- and so its GPU -- may only be known then)
}

void DataPlane::use_transport(uintptr_t ops, uint64_t cap_bytes) {
  if (cell_.comm.load() || ep_) throw std::runtime_error("DataPlane: the transport is fixed once a generation formed");
  const auto* t = reinterpret_cast<const DpTransportOps*>(ops);
  if (t && t->abi != kDpTransportAbi) throw std::invalid_argument("DataPlane: transport ABI mismatch");
  ops_ = t;
  cap_bytes_ = cap_bytes;
}

void DataPlane::set_device(int device) {
  if (cell_.comm.load() || ep_) throw std::runtime_error("DataPlane: the device is fixed while a communicator exists");
  if (stream_ && device != device_) {
    (void)api().set_device(device_);
    (void)api().stream_destroy(stream_);
    stream_ = nullptr;
  }
  device_ = device;
}

DataPlane::~DataPlane() {
  {
    std::lock_guard<std::mutex> lk(wd_mu_);
    wd_stop_ = true;
  }
  wd_cv_.notify_all();
  if (wd_thread_.joinable()) wd_thread_.join();
  Api& a = api();
  if (!a.ok() || device_ < 0) return;
  (void)a.set_device(device_);
  destroy_comm();
  for (auto& e : armed_) (void)a.event_destroy(e.first);
  if (scratch_) (void)a.hfree(scratch_);
  if (stream_) (void)a.stream_destroy(stream_);
}

// ---------------------------------------------------------------- abort / teardown
void DataPlane::abort() {
  if (!api().ok()) return;
  if (ops_) {
    if (ep_) ops_->abort(ep_);  // every wait of this endpoint ends at once
    ep_failed_ = true;
    return;
  }
  // no engine is inside an RCCL enqueue on this communicator once it is retired
  if (void* c = cell_.retire(5.0)) {
    (void)api().set_device(device_);
    (void)api().abort(c);
  }
}

bool DataPlane::aborted() const { return ops_ ? (!ep_ || ep_failed_.load()) : cell_.comm.load() == nullptr; }

void DataPlane::destroy_comm() {
  abort();
  if (ops_ && ep_) {
    ops_->release(ep_);  // (engines may hold their own references: the segments stay mapped for them)
    ep_ = nullptr;
  }
}

void* DataPlane::live_comm() {
  void* c = cell_.enter();
  if (!c) throw std::runtime_error("DataPlane: ncclRemoteError: no communicator (aborted or never formed)");
  return c;
}

// A host wait for this object's stream that a dead peer cannot hang: poll the
// stream and the transport's failure state; past timeout_s the generation is
// aborted (its kernels return) and the wait raises a peer failure
// (parallel/elastic.py is_rank_failure).
void DataPlane::wait_stream() {
  Api& a = need();
  const double t_end = now_s() + timeout_s_;
  for (int spin = 0;; ++spin) {
    const int q = a.stream_query(stream_);
    if (q == 0) {
      if (ops_ && ops_->failed(ep_))
        throw std::runtime_error("DataPlane: IpcComm: peer did not reach a collective (the generation failed)");
      return;
    }
    if (q != kHipNotReady) hip_check(q, "hipStreamQuery");
    if (!ops_) {
      void* c = cell_.comm.load();
      if (!c || cell_.failed())
        throw std::runtime_error("DataPlane: ncclRemoteError: the communicator was aborted during a collective");
      int st = 0;
      if (a.async_error(c, &st) == 0 && st != 0 && st != kNcclInProgress) {
        abort();
        throw std::runtime_error(std::string("DataPlane: ncclRemoteError: ") + (a.errstr ? a.errstr(st) : "async error"));
      }
    } else if (ops_->failed(ep_)) {
      (void)a.stream_sync(stream_);  // (bounded: the endpoint's waits end once it failed)
      throw std::runtime_error("DataPlane: IpcComm: peer did not reach a collective (the generation failed)");
    }
    if (now_s() > t_end) {
      abort();
      throw std::runtime_error("DataPlane: ncclRemoteError: a collective did not complete within " +
                               std::to_string(timeout_s_) + " s (a peer is gone)");
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// ---------------------------------------------------------------- membership
// Each member's registration tag: the create revision of its registry key (a new
// process incarnation registers anew), so a record published for an earlier
// incarnation of the same member list is never taken for this formation's.
static std::vector<int64_t> member_tags(KvClient& kv, const std::string& service,
                                        const std::vector<std::string>& members) {
  const std::string pfx = std::string(kServicesPrefix) + "/" + service + "/";
  RangeOpts o;
  o.end = prefix_range_end(pfx);
  const RangeResult r = kv.get(pfx, o);
  std::vector<int64_t> tags(members.size(), 0);
  for (const auto& kv1 : r.kvs) {
    Node n;
    try {
      n = node_from_json(kv1.value);
    } catch (...) {
      continue;
    }
    const std::string id = n.address + ":" + std::to_string(n.port);
    for (size_t i = 0; i < members.size(); ++i)
      if (members[i] == id) tags[i] = std::max(tags[i], kv1.create_revision);
  }
  return tags;
}

std::vector<std::string> DataPlane::alive_nodes() {
  const auto ctx = Context::with_timeout(Context::background(), (int64_t)(timeout_s_ * 1000));
  std::set<std::string> ids;
  for (const auto& n : reg_->nodes(ctx, service_)) ids.insert(n.address + ":" + std::to_string(n.port));
  return {ids.begin(), ids.end()};
}

std::vector<std::string> DataPlane::wait_nodes(int world) {
  const double t_end = now_s() + timeout_s_;
  for (;;) {
    auto nodes = alive_nodes();
    if ((int)nodes.size() >= world) {
      nodes.resize((size_t)world);
      return nodes;
    }
    if (now_s() > t_end)
      throw std::runtime_error("DataPlane: only " + std::to_string(nodes.size()) + " of " + std::to_string(world) +
                               " data-plane nodes of " + service_ + " registered");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

// Every member puts <key_pfx><itself> and waits (bounded) for `world` keys.
void DataPlane::store_barrier(const std::string& key_pfx, int world) {
  kv_->put(key_pfx + me_, "1");
  const double t_end = now_s() + timeout_s_;
  for (;;) {
    RangeOpts o;
    o.end = prefix_range_end(key_pfx);
    if ((int)kv_->get(key_pfx, o).kvs.size() >= world) return;
    if (now_s() > t_end)
      throw std::runtime_error("DataPlane: ncclRemoteError: a member did not reach the formation barrier " + key_pfx);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

// Rendezvous: the proposal's first node publishes {members, tags, uid | nonce}
// under .../<gen>/<itself>; every member takes the record with the lowest create
// revision among those still current (their members' registrations are the ones
// in force), so survivors whose views differed still converge on one member list
// -- or learn they were left out.
int DataPlane::form(uint64_t gen, const std::vector<std::string>& proposal) {
  Api& a = need();
  if (std::find(proposal.begin(), proposal.end(), me_) == proposal.end())
    throw std::runtime_error("DataPlane: " + me_ + " is not in the proposal for generation " + std::to_string(gen));
  destroy_comm();
  const std::string pfx = std::string(kStorePrefix) + "/_ptype/nccl/" + service_ + "/" + std::to_string(gen) + "/";
  if (proposal[0] == me_) {
    std::string secret;
    if (!ops_) {
      NcclUid mine{};
      nccl_check(a.get_uid(&mine), "ncclGetUniqueId");
      secret = hex(&mine, sizeof mine);
    } else {  // IPC: a nonce names this formation's segments (no uid)
      std::random_device rd;
      const uint64_t r = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
      secret = hex(&r, sizeof r);
    }
    const std::vector<int64_t> tags = member_tags(*kv_, service_, proposal);
    JValue rec;
    rec.kind = JValue::kObject;
    rec.obj.emplace_back(ops_ ? "nonce" : "uid", JValue::string(secret));
    JValue ms, ts;
    ms.kind = ts.kind = JValue::kArray;
    for (size_t i = 0; i < proposal.size(); ++i) {
      ms.arr.push_back(JValue::string(proposal[i]));
      ts.arr.push_back(JValue::integer(tags[i]));
    }
    rec.obj.emplace_back("members", ms);
    rec.obj.emplace_back("tags", ts);
    kv_->put(pfx + me_, json_dump(rec));
  }
  std::string secret;
  std::vector<std::string> members;
  const double t_end = now_s() + timeout_s_;
  for (bool got = false; !got;) {
    RangeOpts o;
    o.end = prefix_range_end(pfx);
    o.sort_target = kSortCreate;
    o.sort_order = kSortAscend;
    const RangeResult r = kv_->get(pfx, o);
    for (const auto& kv1 : r.kvs) {
      JValue v;
      try {
        v = json_parse(kv1.value);
      } catch (...) {
        continue;  // (a barrier key of this generation, not a record)
      }
      const JValue* u = v.get(ops_ ? "nonce" : "uid");
      const JValue* ms = v.get("members");
      const JValue* ts = v.get("tags");
      std::vector<std::string> theirs;
      std::vector<int64_t> their_tags;
      if (ms)
        for (const auto& m : ms->arr) theirs.push_back(m.str);
      if (ts)
        for (const auto& t : ts->arr) their_tags.push_back(t.i);
      if (!u || theirs.empty() || their_tags != member_tags(*kv_, service_, theirs))
        continue;  // an earlier incarnation's record (or a member gone since): not this formation's
      secret = u->str;
      members = theirs;
      got = true;
      break;
    }
    if (got) break;
    if (now_s() > t_end)
      throw std::runtime_error("DataPlane: no record of generation " + std::to_string(gen) + " of " + service_);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  const auto it = std::find(members.begin(), members.end(), me_);
  if (it == members.end())
    throw std::runtime_error("DataPlane: excluded: " + me_ + " was left out of generation " + std::to_string(gen));
  const int rank = (int)(it - members.begin());
  if (device_ < 0) throw std::runtime_error("DataPlane: no device (set_device before form)");
  hip_check(a.set_device(device_), "hipSetDevice");
  if (!stream_) hip_check(a.stream_create(&stream_, 1 /* hipStreamNonBlocking */), "hipStreamCreateWithFlags");
  if (!ops_) form_rccl(secret, rank, (int)members.size());
  else form_ipc(pfx, secret, rank, (int)members.size());
  rank_ = rank;
  gen_ = gen;
  members_ = members;
  if (nodes0_.empty()) nodes0_ = members;  // the original ring (ring adoption, buddies)
  if (rank == 0 && gen >= 2) {  // generation gen - 2's records are nobody's any more (best effort)
    try {
      const std::string old = std::string(kStorePrefix) + "/_ptype/nccl/" + service_ + "/" + std::to_string(gen - 2) + "/";
      int64_t deleted = 0;
      (void)kv_->del(old, prefix_range_end(old), &deleted, 2000);
    } catch (const std::exception&) {
    }
  }
  return rank;
}

// ncclCommInitRank, bounded: it blocks in RCCL's bootstrap until every rank of the
// record arrives -- a member that died between the record and its init would hang
// it.  The init runs on a helper thread; past timeout_s the caller gets
// a rank failure, and a late completion is aborted by the helper itself.
void DataPlane::form_rccl(const std::string& uid_hex, int rank, int world) {
  Api& a = need();
  NcclUid uid{};
  if (!unhex(uid_hex, &uid, sizeof uid)) throw std::runtime_error("DataPlane: malformed unique id record");
  struct Init {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    int rc = 0;
    void* comm = nullptr;
  };
  auto st = std::make_shared<Init>();
  const int dev = device_;
  std::thread([st, uid, world, rank, dev] {
    Api& a2 = api();
    (void)a2.set_device(dev);
    void* c = nullptr;
    const int rc = a2.init_rank(&c, world, uid, rank);
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->abandoned) {
      if (rc == 0 && c) (void)a2.abort(c);
      return;
    }
    st->rc = rc;
    st->comm = c;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  if (!st->cv.wait_for(lk, std::chrono::duration<double>(timeout_s_), [&] { return st->done; })) {
    st->abandoned = true;
    throw std::runtime_error("DataPlane: ncclRemoteError: ncclCommInitRank did not complete within " +
                             std::to_string(timeout_s_) + " s (a member of the record is gone)");
  }
  nccl_check(st->rc, "ncclCommInitRank");
  (void)a;
  cell_.install(st->comm);
}

// IPC: segment names follow from the record's nonce; members meet at a store
// barrier once every segment exists, connect, meet again (every mapping done) and
// seal (the names leave /dev/shm; the mappings stay).
void DataPlane::form_ipc(const std::string& pfx, const std::string& nonce, int rank, int world) {
  if (!cap_bytes_) throw std::runtime_error("DataPlane: IPC transport without a region capacity");
  auto name_of = [&](int r) { return "ptype-dp-" + nonce + "-" + std::to_string(r); };
  char err[512] = {0};
  void* ep = ops_->open(device_, world, rank, cap_bytes_, timeout_s_, name_of(rank).c_str(), err, sizeof err);
  if (!ep) throw std::runtime_error(std::string("DataPlane: IPC transport open failed: ") + err);
  try {
    store_barrier(pfx + "ipc-open/" + nonce + "/", world);
    std::vector<std::string> names;
    std::vector<const char*> cn;
    for (int r = 0; r < world; ++r) names.push_back(name_of(r));
    for (auto& n : names) cn.push_back(n.c_str());
    if (ops_->connect(ep, cn.data(), world, err, sizeof err) != 0)
      throw std::runtime_error(std::string("DataPlane: ncclRemoteError: IPC connect failed: ") + err);
    store_barrier(pfx + "ipc-conn/" + nonce + "/", world);
    ops_->seal(ep);
  } catch (...) {
    ops_->abort(ep);
    ops_->release(ep);
    throw;
  }
  ep_ = ep;
  ep_failed_ = false;
}

// The next generation's proposal after a failed one: wait (at most grace_s)
// until the lease-based membership has dropped somebody of `current` (a dead
// node's 2 s registry lease lapsing), then the survivors in their old order, so
// ranks stay dense and ordered.
std::vector<std::string> DataPlane::settle(const std::vector<std::string>& current, double grace_s) {
  const double t_end = now_s() + grace_s;
  std::vector<std::string> live = alive_nodes();
  auto all_alive = [&](const std::vector<std::string>& l) {
    for (const auto& n : current)
      if (std::find(l.begin(), l.end(), n) == l.end()) return false;
    return true;
  };
  while (all_alive(live) && now_s() < t_end) {
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    live = alive_nodes();
  }
  std::vector<std::string> proposal;
  for (const auto& n : current)
    if (std::find(live.begin(), live.end(), n) != live.end()) proposal.push_back(n);
  if (std::find(proposal.begin(), proposal.end(), me_) == proposal.end()) {
    proposal.push_back(me_);
    std::sort(proposal.begin(), proposal.end());
  }
  return proposal;
}

// ---------------------------------------------------------------- placement (ring adoption)
// Every surviving original node owns its own original rank first, then adopts
// each dead original rank whose next surviving successor (in original ring
// order) it is.  Actors of live ranks never move.
std::map<std::string, std::vector<int>> DataPlane::placement(const std::vector<std::string>& members) const {
  const std::set<std::string> alive(members.begin(), members.end());
  std::map<std::string, std::vector<int>> own;
  const int W0 = (int)nodes0_.size();
  for (int r = 0; r < W0; ++r)
    if (alive.count(nodes0_[(size_t)r])) own[nodes0_[(size_t)r]].push_back(r);
  for (int r = 0; r < W0; ++r) {
    if (alive.count(nodes0_[(size_t)r])) continue;
    for (int k = 1; k < W0; ++k) {
      const std::string& succ = nodes0_[(size_t)((r + k) % W0)];
      if (alive.count(succ)) {
        own[succ].push_back(r);
        break;
      }
    }
  }
  return own;
}

std::vector<int> DataPlane::blocks() const {
  const auto own = placement(members_);
  const auto it = own.find(me_);
  return it == own.end() ? std::vector<int>{} : it->second;
}

std::string DataPlane::buddy(const std::string& node) const {
  const std::set<std::string> alive(members_.begin(), members_.end());
  const auto it = std::find(nodes0_.begin(), nodes0_.end(), node);
  if (it == nodes0_.end()) return node;
  const size_t i = (size_t)(it - nodes0_.begin()), W0 = nodes0_.size();
  for (size_t k = 1; k < W0; ++k) {
    const std::string& n = nodes0_[(i + k) % W0];
    if (alive.count(n)) return n;
  }
  return node;
}

std::vector<int> DataPlane::lost_blocks(const std::vector<std::string>& before,
                                        const std::vector<std::string>& after) const {
  const auto own = placement(before);
  const std::set<std::string> stay(after.begin(), after.end());
  std::vector<int> lost;
  for (const auto& kv1 : own)
    if (!stay.count(kv1.first)) lost.insert(lost.end(), kv1.second.begin(), kv1.second.end());
  std::sort(lost.begin(), lost.end());
  return lost;
}

std::vector<int> DataPlane::replica_blocks() const {
  if (buddy(me_) == me_) return {};
  for (const auto& n : members_)
    if (n != me_ && buddy(n) == me_) return placement(members_)[n];
  return {};
}

std::vector<int> DataPlane::replicate(uintptr_t state, size_t bytes, uintptr_t recv, size_t recv_bytes) {
  const std::string dst = buddy(me_);
  if (dst == me_) {  // alone: nothing could adopt these blocks
    replicas_.clear();
    return {};
  }
  std::string src;
  for (const auto& n : members_)
    if (n != me_ && buddy(n) == me_) src = n;
  auto idx = [&](const std::string& n) { return (int)(std::find(members_.begin(), members_.end(), n) - members_.begin()); };
  const int d = idx(dst), s = src.empty() ? -1 : idx(src);
  sendrecv(state, bytes, d, recv, s >= 0 ? recv_bytes : 0, s);
  replicas_ = s >= 0 ? placement(members_)[src] : std::vector<int>{};
  return replicas_;
}

DataPlane::Recovery DataPlane::recover(double grace_s) {
  const std::vector<std::string> before = members_;
  const std::vector<int> old_blocks = blocks();
  const std::vector<int> held = replicas_;
  abort();
  form(gen_ + 1, settle(members_, grace_s));
  Recovery out;
  out.lost = lost_blocks(before, members_);
  out.members = members_;
  out.blocks = blocks();
  for (int r : out.blocks) {
    const auto k = std::find(old_blocks.begin(), old_blocks.end(), r);
    out.kept_from.push_back(k == old_blocks.end() ? -1 : (int)(k - old_blocks.begin()));
    out.from_replica.push_back(k == old_blocks.end() && std::find(held.begin(), held.end(), r) != held.end());
  }
  replicas_.clear();  // the ring changed: replicas are re-taken by the next replicate()
  return out;
}

// ---------------------------------------------------------------- collectives of the control plane
int DataPlane::async_error() const {
  if (ops_) return (!ep_ || ep_failed_.load() || ops_->failed(ep_)) ? 1 : 0;
  void* c = cell_.comm.load();
  if (!c) return -1;
  int st = 0;
  nccl_check(api().async_error(c, &st), "ncclCommGetAsyncError");
  return st;
}

void DataPlane::ensure_scratch(size_t bytes) {
  Api& a = need();
  if (scratch_bytes_ >= bytes) return;
  if (scratch_) (void)a.hfree(scratch_);
  scratch_ = nullptr;
  hip_check(a.hmalloc(&scratch_, bytes), "hipMalloc");
  scratch_bytes_ = bytes;
}

std::vector<uint64_t> DataPlane::allreduce_max(const std::vector<uint64_t>& v) {
  Api& a = need();
  if (v.empty()) return {};
  hip_check(a.set_device(device_), "hipSetDevice");
  ensure_scratch(v.size() * 8);
  hip_check(a.memcpy_(scratch_, v.data(), v.size() * 8, kHipH2D), "hipMemcpy");
  allreduce_max_dev((uintptr_t)scratch_, v.size(), (uintptr_t)stream_);
  wait_stream();
  std::vector<uint64_t> out(v.size());
  hip_check(a.memcpy_(out.data(), scratch_, v.size() * 8, kHipD2H), "hipMemcpy");
  return out;
}

void DataPlane::allreduce_max_dev(uintptr_t dev, size_t n, uintptr_t stream) {
  Api& a = need();
  if (ops_) {
    if (!ep_ || ep_failed_) throw std::runtime_error("DataPlane: IpcComm: peer failure (the generation was aborted)");
    char err[512] = {0};
    if (ops_->allreduce_max(ep_, (uint64_t*)dev, (int)n, (void*)stream, err, sizeof err) != 0)
      throw std::runtime_error(std::string("DataPlane: IpcComm: peer ") + err);
    return;
  }
  void* c = live_comm();
  const int rc = a.allreduce((const void*)dev, (void*)dev, n, kNcclUint64, kNcclMax, c, (void*)stream);
  cell_.leave();
  nccl_check(rc, "ncclAllReduce");
}

void DataPlane::sendrecv(uintptr_t send, size_t sbytes, int dst, uintptr_t recv, size_t rbytes, int src) {
  Api& a = need();
  hip_check(a.set_device(device_), "hipSetDevice");
  if (!ops_) {
    void* c = live_comm();
    int rc = a.group_start();
    if (rc == 0 && dst >= 0 && sbytes) rc = a.send((const void*)send, sbytes, kNcclInt8, dst, c, stream_);
    if (rc == 0 && src >= 0 && rbytes) rc = a.recv((void*)recv, rbytes, kNcclInt8, src, c, stream_);
    const int rc2 = a.group_end();
    cell_.leave();
    nccl_check(rc ? rc : rc2, "ncclSend/ncclRecv");
    wait_stream();
    return;
  }
  // IPC: an all-to-all with two used regions, staged and cut into pieces of the
  // region capacity -- every member runs the same number of ops (the agreed max)
  const std::vector<uint64_t> m = allreduce_max({dst >= 0 ? sbytes : 0, src >= 0 ? rbytes : 0});
  const uint64_t total = std::max(m[0], m[1]);
  const int R = size();
  const uint64_t piece = std::max<uint64_t>(16, ops_->cap(ep_) / 16 * 16);
  ensure_scratch((size_t)(2 * R * piece));
  char* S = (char*)scratch_;
  char* D = S + R * piece;
  std::vector<size_t> sn((size_t)R), rn((size_t)R);
  for (uint64_t off = 0; off < total; off += piece) {
    std::fill(sn.begin(), sn.end(), 0);
    std::fill(rn.begin(), rn.end(), 0);
    if (dst >= 0 && off < sbytes) {
      sn[(size_t)dst] = (size_t)std::min<uint64_t>(piece, sbytes - off);
      hip_check(a.memcpy_(S + (size_t)dst * piece, (const char*)send + off, sn[(size_t)dst], kHipD2D), "hipMemcpy");
    }
    if (src >= 0 && off < rbytes) rn[(size_t)src] = (size_t)std::min<uint64_t>(piece, rbytes - off);
    char err[512] = {0};
    if (ops_->alltoallv(ep_, S, D, (size_t)piece, sn.data(), rn.data(), stream_, err, sizeof err) != 0)
      throw std::runtime_error(std::string("DataPlane: IpcComm: peer ") + err);
    wait_stream();
    if (src >= 0 && rn[(size_t)src])
      hip_check(a.memcpy_((char*)recv + off, D + (size_t)src * piece, rn[(size_t)src], kHipD2D), "hipMemcpy");
  }
}

void DataPlane::barrier() { (void)allreduce_max({1}); }

uintptr_t DataPlane::engine_comm_ref() {
  if (!ops_) return 0;
  if (!ep_) throw std::runtime_error("DataPlane: ncclRemoteError: no IPC generation formed");
  return (uintptr_t)ops_->engine_ref(ep_);
}

// ---------------------------------------------------------------- Send watchdog
void DataPlane::set_watchdog(double timeout_s) {
  std::lock_guard<std::mutex> lk(wd_mu_);
  wd_timeout_s_ = timeout_s;
  if (timeout_s > 0 && !wd_thread_.joinable()) wd_thread_ = std::thread([this] { watchdog_loop(); });
}

void DataPlane::begin_send() {
  std::lock_guard<std::mutex> lk(wd_mu_);
  if (wd_timeout_s_ > 0) host_deadline_ = now_s() + wd_timeout_s_;
}

void DataPlane::end_send() {
  std::lock_guard<std::mutex> lk(wd_mu_);
  host_deadline_ = 0;
}

void DataPlane::arm(uintptr_t stream) {
  Api& a = need();
  if (wd_timeout_s_ <= 0) return;
  void* ev = nullptr;
  hip_check(a.event_create(&ev, 2 /* hipEventDisableTiming */), "hipEventCreateWithFlags");
  hip_check(a.event_record(ev, (void*)stream), "hipEventRecord");
  std::lock_guard<std::mutex> lk(wd_mu_);
  armed_.emplace_back(ev, now_s() + wd_timeout_s_);
  if (armed_.size() > 64) {  // completed events are dropped by the thread; bound the backlog anyway
    std::vector<std::pair<void*, double>> keep;
    for (auto& e : armed_)
      if (a.event_query(e.first) == kHipNotReady) keep.push_back(e);
      else (void)a.event_destroy(e.first);
    armed_.swap(keep);
  }
}

std::string DataPlane::watchdog_failed() const {
  std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(wd_mu_));
  return wd_failed_;
}

void DataPlane::reset_watchdog() {
  std::lock_guard<std::mutex> lk(wd_mu_);
  for (auto& e : armed_) (void)api().event_destroy(e.first);
  armed_.clear();
  host_deadline_ = 0;
  wd_failed_.clear();
}

// Marks the generation failed and aborts it: RCCL -- the cell is poisoned first,
// so an engine between two enqueues raises instead of using the communicator,
// and the abort waits for any enqueue in flight; host waits see the poison.
void DataPlane::fail_generation(const std::string& why) {
  {
    std::lock_guard<std::mutex> lk(wd_mu_);
    if (!wd_failed_.empty()) return;
    wd_failed_ = why;
  }
  abort();
}

void DataPlane::watchdog_loop() {
  Api& a = api();
  std::unique_lock<std::mutex> lk(wd_mu_);
  while (!wd_stop_) {
    wd_cv_.wait_for(lk, std::chrono::milliseconds(50));
    if (wd_stop_) break;
    if (!wd_failed_.empty()) continue;
    const double now = now_s();
    std::string why;
    if (host_deadline_ > 0 && now > host_deadline_)
      why = "a Send did not return within " + std::to_string(wd_timeout_s_) + " s";
    std::vector<std::pair<void*, double>> keep;
    for (auto& e : armed_) {
      if (a.event_query(e.first) != kHipNotReady) {
        (void)a.event_destroy(e.first);
        continue;
      }
      if (now > e.second && why.empty())
        why = "a Send's device work did not complete within " + std::to_string(wd_timeout_s_) + " s";
      keep.push_back(e);
    }
    armed_.swap(keep);
    if (!why.empty()) {
      lk.unlock();
      fail_generation(why);
      lk.lock();
    }
  }
}

}  // namespace ptype
