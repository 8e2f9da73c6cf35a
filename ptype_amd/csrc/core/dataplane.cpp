// Data-plane communicator lifecycle (dataplane.hpp).
#include "dataplane.hpp"

#include <dlfcn.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <set>
#include <stdexcept>
#include <thread>

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
  }
  Api() {
    bind_all(RTLD_DEFAULT);
    for (const char* lib : {"librccl.so", "librccl.so.1", "libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"}) {
      if (ok()) break;
      void* h = dlopen(lib, RTLD_NOW | RTLD_NOLOAD);  // only what the process already loaded
      if (h) bind_all(h);
    }
  }
  bool ok() const {
    return get_uid && init_rank && abort && async_error && allreduce && send && recv && group_start && group_end &&
           set_device && hmalloc && hfree && memcpy_ && stream_create && stream_sync && stream_query && stream_destroy;
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
constexpr int kNcclUint64 = 5, kNcclInt8 = 0, kNcclMax = 2;
constexpr int kHipH2D = 1, kHipD2H = 2;

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

void DataPlane::set_device(int device) {
  if (comm_.load()) throw std::runtime_error("DataPlane: the device is fixed while a communicator exists");
  if (stream_ && device != device_) {
    (void)api().set_device(device_);
    (void)api().stream_destroy(stream_);
    stream_ = nullptr;
  }
  device_ = device;
}

DataPlane::~DataPlane() {
  Api& a = api();
  if (!a.ok() || device_ < 0) return;
  (void)a.set_device(device_);
  destroy_comm();
  if (scratch_) (void)a.hfree(scratch_);
  if (stream_) (void)a.stream_destroy(stream_);
}

void DataPlane::destroy_comm() {
  // ncclCommAbort, not Destroy: a communicator of a generation that may have lost
  // a member must not wait for it (Destroy flushes outstanding work).  Another
  // thread (a Send watchdog) may abort while this one waits in wait_stream().
  if (void* c = comm_.exchange(nullptr)) (void)api().abort(c);
}

// A host wait for this object's stream that a dead peer cannot hang: poll the
// stream and the communicator's async error; past timeout_s (or once another
// thread aborted) the communicator is aborted -- its kernels return -- and the
// wait raises a peer failure (parallel/elastic.py is_rank_failure).
void DataPlane::wait_stream(void* comm) {
  Api& a = need();
  const double t_end = now_s() + timeout_s_;
  for (int spin = 0;; ++spin) {
    const int q = a.stream_query(stream_);
    if (q == 0) return;
    if (q != 600 /* hipErrorNotReady */) hip_check(q, "hipStreamQuery");
    int st = 0;
    if (comm_.load() != comm)
      throw std::runtime_error("DataPlane: ncclRemoteError: the communicator was aborted during a collective");
    if (a.async_error(comm, &st) == 0 && st != 0 && st != 7 /* ncclInProgress */) {
      destroy_comm();
      throw std::runtime_error(std::string("DataPlane: ncclRemoteError: ") + (a.errstr ? a.errstr(st) : "async error"));
    }
    if (now_s() > t_end) {
      destroy_comm();
      throw std::runtime_error("DataPlane: ncclRemoteError: a collective did not complete within " +
                               std::to_string(timeout_s_) + " s (a peer is gone)");
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

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

// Rendezvous: the proposal's first node draws the unique id and publishes
// {uid, members, tags} under .../<gen>/<itself>; every member takes the record
// with the lowest create revision among those still current (their members'
// registrations are the ones in force), so survivors whose views differed still
// converge on one member list -- or learn they were left out.
int DataPlane::form(uint64_t gen, const std::vector<std::string>& proposal) {
  Api& a = need();
  if (std::find(proposal.begin(), proposal.end(), me_) == proposal.end())
    throw std::runtime_error("DataPlane: " + me_ + " is not in the proposal for generation " + std::to_string(gen));
  destroy_comm();
  const std::string pfx = std::string(kStorePrefix) + "/_ptype/nccl/" + service_ + "/" + std::to_string(gen) + "/";
  if (proposal[0] == me_) {
    NcclUid mine{};
    nccl_check(a.get_uid(&mine), "ncclGetUniqueId");
    const std::vector<int64_t> tags = member_tags(*kv_, service_, proposal);
    JValue rec;
    rec.kind = JValue::kObject;
    rec.obj.emplace_back("uid", JValue::string(hex(&mine, sizeof mine)));
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
  NcclUid uid{};
  std::vector<std::string> members;
  const double t_end = now_s() + timeout_s_;
  for (bool got = false; !got;) {
    RangeOpts o;
    o.end = prefix_range_end(pfx);
    o.sort_target = kSortCreate;
    o.sort_order = kSortAscend;
    const RangeResult r = kv_->get(pfx, o);
    for (const auto& kv1 : r.kvs) {
      const JValue v = json_parse(kv1.value);
      const JValue* u = v.get("uid");
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
      if (!unhex(u->str, &uid, sizeof uid)) throw std::runtime_error("DataPlane: malformed unique id record");
      members = theirs;
      got = true;
      break;
    }
    if (got) break;
    if (now_s() > t_end)
      throw std::runtime_error("DataPlane: no unique id of generation " + std::to_string(gen) + " of " + service_);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  const auto it = std::find(members.begin(), members.end(), me_);
  if (it == members.end())
    throw std::runtime_error("DataPlane: excluded: " + me_ + " was left out of generation " + std::to_string(gen));
  const int rank = (int)(it - members.begin());
  if (device_ < 0) throw std::runtime_error("DataPlane: no device (set_device before form)");
  hip_check(a.set_device(device_), "hipSetDevice");
  if (!stream_) hip_check(a.stream_create(&stream_, 1 /* hipStreamNonBlocking */), "hipStreamCreateWithFlags");
  void* comm = nullptr;
  nccl_check(a.init_rank(&comm, (int)members.size(), uid, rank), "ncclCommInitRank");
  comm_.store(comm);
  rank_ = rank;
  gen_ = gen;
  members_ = members;
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

std::vector<std::string> DataPlane::recover(double grace_s) {
  abort();
  form(gen_ + 1, settle(members_, grace_s));
  return members_;  // the winning record's list (it may differ from this member's proposal)
}

int DataPlane::async_error() const {
  void* c = comm_.load();
  if (!c) return -1;
  int st = 0;
  nccl_check(api().async_error(c, &st), "ncclCommGetAsyncError");
  return st;
}

void DataPlane::abort() {
  if (!api().ok()) return;
  (void)api().set_device(device_);
  destroy_comm();
}

void* DataPlane::live_comm() const {
  void* c = comm_.load();
  if (!c) throw std::runtime_error("DataPlane: ncclRemoteError: no communicator (aborted or never formed)");
  return c;
}

std::vector<uint64_t> DataPlane::allreduce_max(const std::vector<uint64_t>& v) {
  Api& a = need();
  void* c = live_comm();
  if (v.empty()) return {};
  hip_check(a.set_device(device_), "hipSetDevice");
  if (scratch_words_ < v.size()) {
    if (scratch_) (void)a.hfree(scratch_);
    scratch_ = nullptr;
    hip_check(a.hmalloc(&scratch_, v.size() * 8), "hipMalloc");
    scratch_words_ = v.size();
  }
  hip_check(a.memcpy_(scratch_, v.data(), v.size() * 8, kHipH2D), "hipMemcpy");
  nccl_check(a.allreduce(scratch_, scratch_, v.size(), kNcclUint64, kNcclMax, c, stream_), "ncclAllReduce");
  wait_stream(c);
  std::vector<uint64_t> out(v.size());
  hip_check(a.memcpy_(out.data(), scratch_, v.size() * 8, kHipD2H), "hipMemcpy");
  return out;
}

void DataPlane::allreduce_max_dev(uintptr_t dev, size_t n, uintptr_t stream) {
  Api& a = need();
  nccl_check(a.allreduce((const void*)dev, (void*)dev, n, kNcclUint64, kNcclMax, live_comm(), (void*)stream),
             "ncclAllReduce");
}

void DataPlane::sendrecv(uintptr_t send, size_t sbytes, int dst, uintptr_t recv, size_t rbytes, int src) {
  Api& a = need();
  void* c = live_comm();
  hip_check(a.set_device(device_), "hipSetDevice");
  nccl_check(a.group_start(), "ncclGroupStart");
  if (dst >= 0 && sbytes) nccl_check(a.send((const void*)send, sbytes, kNcclInt8, dst, c, stream_), "ncclSend");
  if (src >= 0 && rbytes) nccl_check(a.recv((void*)recv, rbytes, kNcclInt8, src, c, stream_), "ncclRecv");
  nccl_check(a.group_end(), "ncclGroupEnd");
  wait_stream(c);
}

void DataPlane::barrier() { (void)allreduce_max({1}); }

}  // namespace ptype
