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
           set_device && hmalloc && hfree && memcpy_ && stream_create && stream_sync && stream_destroy;
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
  Api& a = need();
  hip_check(a.set_device(device_), "hipSetDevice");
  hip_check(a.stream_create(&stream_, 1 /* hipStreamNonBlocking */), "hipStreamCreateWithFlags");
}

DataPlane::~DataPlane() {
  Api& a = api();
  if (!a.ok()) return;
  (void)a.set_device(device_);
  destroy_comm();
  if (scratch_) (void)a.hfree(scratch_);
  if (stream_) (void)a.stream_destroy(stream_);
}

void DataPlane::destroy_comm() {
  // ncclCommAbort, not Destroy: a communicator of a generation that may have lost
  // a member must not wait for it (Destroy flushes outstanding work)
  if (comm_) (void)api().abort(comm_);
  comm_ = nullptr;
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

int DataPlane::form(uint64_t gen, const std::vector<std::string>& members) {
  Api& a = need();
  const auto it = std::find(members.begin(), members.end(), me_);
  if (it == members.end()) throw std::runtime_error("DataPlane: " + me_ + " is not a member of generation " +
                                                    std::to_string(gen));
  const int rank = (int)(it - members.begin());
  destroy_comm();
  const std::string key = std::string(kStorePrefix) + "/_ptype/nccl/" + service_ + "/" + std::to_string(gen) + "/uid";
  NcclUid uid{};
  if (rank == 0) {  // rank 0 draws the id and publishes it with the member list
    nccl_check(a.get_uid(&uid), "ncclGetUniqueId");
    JValue rec;
    rec.kind = JValue::kObject;
    rec.obj.emplace_back("uid", JValue::string(hex(&uid, sizeof uid)));
    JValue ms;
    ms.kind = JValue::kArray;
    for (const auto& m : members) ms.arr.push_back(JValue::string(m));
    rec.obj.emplace_back("members", ms);
    kv_->put(key, json_dump(rec));
  } else {  // everyone else reads it from the replicated store
    const double t_end = now_s() + timeout_s_;
    bool got = false;
    while (!got) {
      RangeOpts o;
      const RangeResult r = kv_->get(key, o);
      if (!r.kvs.empty()) {
        const JValue v = json_parse(r.kvs[0].value);
        const JValue* u = v.get("uid");
        const JValue* ms = v.get("members");
        std::vector<std::string> theirs;
        if (ms)
          for (const auto& m : ms->arr) theirs.push_back(m.str);
        if (!u || theirs != members)
          throw std::runtime_error("DataPlane: generation " + std::to_string(gen) + " was published for another member list");
        got = unhex(u->str, &uid, sizeof uid);
        if (!got) throw std::runtime_error("DataPlane: malformed unique id record");
        break;
      }
      if (now_s() > t_end)
        throw std::runtime_error("DataPlane: no unique id of generation " + std::to_string(gen) + " of " + service_);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }
  hip_check(a.set_device(device_), "hipSetDevice");
  void* comm = nullptr;
  nccl_check(a.init_rank(&comm, (int)members.size(), uid, rank), "ncclCommInitRank");
  comm_ = comm;
  rank_ = rank;
  gen_ = gen;
  members_ = members;
  return rank;
}

std::vector<std::string> DataPlane::settle(const std::vector<std::string>& current, double grace_s) {
  const double t_end = now_s() + std::max(timeout_s_, 4 * grace_s);
  std::vector<std::string> last = alive_nodes();
  double since = now_s();
  for (;;) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const auto nodes = alive_nodes();
    if (nodes != last) {
      last = nodes;
      since = now_s();
    }
    // a lost member shows up as a lapsed lease; stable for grace_s and changed: the next generation
    if (last != current && std::find(last.begin(), last.end(), me_) != last.end() && now_s() - since >= grace_s)
      return last;
    if (now_s() > t_end) {
      if (std::find(last.begin(), last.end(), me_) != last.end()) return last;  // (unchanged: re-form as is)
      throw std::runtime_error("DataPlane: this node is not registered any more");
    }
  }
}

std::vector<std::string> DataPlane::recover(double grace_s) {
  abort();
  const auto members = settle(members_, grace_s);
  form(gen_ + 1, members);
  return members;
}

int DataPlane::async_error() const {
  if (!comm_) return -1;
  int st = 0;
  nccl_check(api().async_error(comm_, &st), "ncclCommGetAsyncError");
  return st;
}

void DataPlane::abort() {
  if (!api().ok()) return;
  (void)api().set_device(device_);
  destroy_comm();
}

std::vector<uint64_t> DataPlane::allreduce_max(const std::vector<uint64_t>& v) {
  Api& a = need();
  if (!comm_) throw std::runtime_error("DataPlane: no communicator (aborted or never formed)");
  if (v.empty()) return {};
  hip_check(a.set_device(device_), "hipSetDevice");
  if (scratch_words_ < v.size()) {
    if (scratch_) (void)a.hfree(scratch_);
    scratch_ = nullptr;
    hip_check(a.hmalloc(&scratch_, v.size() * 8), "hipMalloc");
    scratch_words_ = v.size();
  }
  hip_check(a.memcpy_(scratch_, v.data(), v.size() * 8, kHipH2D), "hipMemcpy");
  nccl_check(a.allreduce(scratch_, scratch_, v.size(), kNcclUint64, kNcclMax, comm_, stream_), "ncclAllReduce");
  hip_check(a.stream_sync(stream_), "hipStreamSynchronize");
  std::vector<uint64_t> out(v.size());
  hip_check(a.memcpy_(out.data(), scratch_, v.size() * 8, kHipD2H), "hipMemcpy");
  return out;
}

void DataPlane::sendrecv(uintptr_t send, size_t sbytes, int dst, uintptr_t recv, size_t rbytes, int src) {
  Api& a = need();
  if (!comm_) throw std::runtime_error("DataPlane: no communicator (aborted or never formed)");
  hip_check(a.set_device(device_), "hipSetDevice");
  nccl_check(a.group_start(), "ncclGroupStart");
  if (dst >= 0 && sbytes) nccl_check(a.send((const void*)send, sbytes, kNcclInt8, dst, comm_, stream_), "ncclSend");
  if (src >= 0 && rbytes) nccl_check(a.recv((void*)recv, rbytes, kNcclInt8, src, comm_, stream_), "ncclRecv");
  nccl_check(a.group_end(), "ncclGroupEnd");
  hip_check(a.stream_sync(stream_), "hipStreamSynchronize");
}

void DataPlane::barrier() { (void)allreduce_max({1}); }

}  // namespace ptype
