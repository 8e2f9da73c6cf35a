// Node-local cross-process path to GPU actors: the persistent dispatcher's
// request/reply rings in a POSIX shared-memory segment.
//
// The reference reaches another process's service over TCP net/rpc even on the
// same host (cluster/rpc.go:272-285, rpc.DialHTTP; the calculator example runs
// client and server as two processes, example/calculator/run).  Here a server
// process that hosts GPU actors places the dispatcher's rings in shared memory
// registered with HIP (the GPU polls them exactly as it polls its own process's
// rings), and exports its device methods (name -> method id + argument fields)
// in the segment header.  A client process on the node maps the segment and
// publishes calls directly: no socket, no gob, no server thread on the path.
// The server's launcher thread sleeps on a process-shared futex that clients
// poke when the dispatcher wave has parked itself.
//
// Layout: [ShmHeader, 16 KB][ServerCtrl, 4 KB][RingSlot x ring][ReplySlot x ring][u64 owner x ring]
//         [RingTaker x kRingTakers] (ringproto.hpp: who holds which sequence numbers)
//         [XLane x kXLanes][XReply x kXLanes] (GPU peer lanes and their reply slots)
//
// Request ring placement: by default the ring the dispatcher
// polls is NOT the segment's RingSlot area but fine-grained memory on the
// server's GPU.  The server exports it as a dma-buf and hands the fd to client
// processes over an abstract unix socket (SCM_RIGHTS; same uid only); a client
// maps it with plain mmap -- no HIP in the client -- and writes requests through
// the BAR, so the polling wave's tag and payload reads stay in HBM instead of
// crossing PCIe twice per call.  Replies, the owner words and the control block
// stay in host memory (the client polls them).  PTYPE_XPROC_RING=host keeps the
// ring in the segment (either side).
#pragma once
#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "records.hpp"
#include "ringproto.hpp"

namespace ptype {

constexpr uint64_t kShmMagic = 0x35736d6570797470ull;  // "ptypems5" (GPU peer lanes in the segment)
constexpr int kShmMaxMethods = 32;

// GPU peer lanes: a GPU in ANOTHER process calls this
// server's actors without any host on the path.  The server keeps kXLanes
// single-producer lanes (XLane) and their 16-B reply slots (XReply) in THIS
// segment -- host shared memory that the server and every calling process map
// and register with HIP, so each GPU reaches them through its own process's
// mapping.  A calling process registers one lane (XLaneReg: its process token);
// from then on the caller's kernel writes a request into the lane and spins on
// the lane's reply slot, which the persistent dispatcher fills with one 16-B
// store.  A lane carries one call at a time (the caller waits for each reply),
// so it needs no sequence taking, owners or rescue: seq + 1 in req_tag
// publishes, `served` acknowledges.
//
// Crash safety: no process ever touches memory another process
// owns.  Round 4's lanes lived in the server's HBM and the reply slots in the
// caller's (both imported by IPC handle), and an import of a killed process's
// HBM faults the GPU of the survivor (profiles/r4_ipc_kill_faults.md).  Pages
// of a shared segment stay mapped for as long as any survivor maps them, so a
// dead server costs its callers a timeout (kStatusNotDelivered) and a dead
// caller costs the server nothing: its lane is reclaimed once quiet.
constexpr int kXLanes = 64;
// Lane life cycle: Free -> (caller) Requested -> (server: lane reset) Ready ->
// (caller) Releasing -> (server: no request in flight, lane reset) Free.  A dead
// caller's lane takes the same server-side path; the caller may register again.
enum XLaneState : uint32_t {
  kXLaneFree = 0,
  kXLaneRequested = 1,
  kXLaneReady = 2,
  kXLaneFailed = 3,
  kXLaneReleasing = 4,
};
struct XLaneReg {
  std::atomic<uint64_t> token;  // the caller's process token (ring_self_token); 0: free
  std::atomic<uint32_t> state;
  int32_t device;               // the caller's HIP device ordinal (diagnostics)
  uint64_t pad[2];
};
struct alignas(128) XLane {  // in the segment; one per wave lane of the dispatcher
  uint64_t req_tag;  // caller: seq + 1 once the request below is out (release)
  uint64_t served;   // dispatcher: req_tag of the last request answered
  uint64_t w0;       // actor | method << 32 | flags << 48 (MsgRecord word 0)
  int64_t a0, a1, a2;
  uint64_t pad[10];
};
static_assert(sizeof(XLane) == 128, "XLane layout");
struct alignas(64) XReply {  // in the segment: lane i's reply {value, reply_tag(seq, status)}
  uint64_t value;
  uint64_t tag;
  uint64_t pad[6];
};
static_assert(sizeof(XReply) == 64, "XReply layout");

struct ShmMethod {
  char name[96];  // "Service.Method"
  uint32_t method, actor, n_fields, pad;
  char fields[3][32];
  char actor_field[32];
};

struct alignas(64) ShmHeader {
  uint64_t magic;
  uint32_t ring;
  int32_t owner_pid;
  std::atomic<uint64_t> next_seq;  // request sequence, shared by every publisher
  std::atomic<uint32_t> wake;      // futex word: 1 = a publisher found the dispatcher parked
  std::atomic<uint32_t> n_methods;
  ShmMethod methods[kShmMaxMethods];
  // device-memory request ring (0: the ring is the segment's own RingSlot area)
  uint32_t req_dev;
  int32_t ipc_device;     // the server's HIP device ordinal
  uint64_t req_dev_off;   // offset of the ring in the dma-buf
  uint64_t req_dev_bytes;
  char req_sock[64];      // abstract unix socket handing out the dma-buf fd
  // GPU peer lanes (the XLane / XReply areas of the segment)
  uint32_t xl_valid, xl_lanes;
  XLaneReg xregs[kXLanes];
};
static_assert(sizeof(ShmHeader) <= 16384, "ShmHeader too large");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics must be lock-free");

constexpr size_t kShmHeaderBytes = 16384, kShmCtrlBytes = 4096;

inline size_t shm_lanes_offset(uint32_t ring) {  // 128-B aligned
  const size_t o = kShmHeaderBytes + kShmCtrlBytes + (size_t)ring * (sizeof(RingSlot) + sizeof(ReplySlot) + sizeof(uint64_t)) +
                   (size_t)kRingTakers * sizeof(RingTaker);
  return (o + 127) & ~(size_t)127;
}
inline size_t shm_bytes(uint32_t ring) {
  return shm_lanes_offset(ring) + (size_t)kXLanes * (sizeof(XLane) + sizeof(XReply));
}

struct ShmView {
  ShmHeader* hdr = nullptr;
  ServerCtrl* ctrl = nullptr;
  RingSlot* req = nullptr;
  ReplySlot* rep = nullptr;
  std::atomic<uint64_t>* owner = nullptr;
  RingTaker* takers = nullptr;
  XLane* xl = nullptr;     // GPU peer lanes
  XReply* xrep = nullptr;  // their reply slots
  bool bar = false;  // `req` is device memory written through a BAR mapping
};

inline ShmView shm_view(void* base, uint32_t ring) {
  char* p = static_cast<char*>(base);
  ShmView v;
  v.hdr = reinterpret_cast<ShmHeader*>(p);
  v.ctrl = reinterpret_cast<ServerCtrl*>(p + kShmHeaderBytes);
  v.req = reinterpret_cast<RingSlot*>(p + kShmHeaderBytes + kShmCtrlBytes);
  v.rep = reinterpret_cast<ReplySlot*>(reinterpret_cast<char*>(v.req) + (size_t)ring * sizeof(RingSlot));
  v.owner = reinterpret_cast<std::atomic<uint64_t>*>(reinterpret_cast<char*>(v.rep) + (size_t)ring * sizeof(ReplySlot));
  v.takers = reinterpret_cast<RingTaker*>(reinterpret_cast<char*>(v.owner) + (size_t)ring * sizeof(uint64_t));
  v.xl = reinterpret_cast<XLane*>(p + shm_lanes_offset(ring));
  v.xrep = reinterpret_cast<XReply*>(reinterpret_cast<char*>(v.xl) + (size_t)kXLanes * sizeof(XLane));
  return v;
}

// Process-shared futex on a 32-bit word of the segment.
void shm_futex_wake(std::atomic<uint32_t>* w);
void shm_futex_wait(std::atomic<uint32_t>* w, uint32_t expect, int64_t timeout_us);

// A mapping of a named segment (creator: O_CREAT + ftruncate; others: attach).
class ShmSegment {
 public:
  static std::shared_ptr<ShmSegment> create(const std::string& name, size_t bytes);
  static std::shared_ptr<ShmSegment> attach(const std::string& name);  // nullptr if absent
  ~ShmSegment();
  void* base() const { return base_; }
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }
  void unlink_on_close() { unlink_ = true; }
  // Remove the name now (every peer has attached): the mappings stay valid, and a
  // process killed later leaves nothing behind in /dev/shm.
  void unlink_now();

 private:
  std::string name_;
  void* base_ = nullptr;
  size_t size_ = 0;
  bool unlink_ = false;
};

// Whether a server places its request ring on the device (PTYPE_XPROC_RING != host).
bool xproc_device_ring_enabled();

// Server side: hands `fd` to every same-uid process that connects to the
// abstract unix socket `name` (one thread; stops on destruction).
class FdHandoff {
 public:
  FdHandoff(const std::string& name, int fd);
  ~FdHandoff();
  FdHandoff(const FdHandoff&) = delete;
  FdHandoff& operator=(const FdHandoff&) = delete;
  uint64_t handed() const { return handed_.load(); }

 private:
  void loop();
  int listen_fd_ = -1, fd_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> handed_{0};
  std::thread thread_;
};

// Client side of FdHandoff: the fd (owned by the caller), or -1 with `why` set.
int shm_receive_fd(const std::string& name, std::string* why = nullptr);

// Client side: the server's device request ring mapped into this process.
class DevRingMap {
 public:
  // nullptr if the header names no device ring or any step fails (`why` says which)
  static std::shared_ptr<DevRingMap> attach(const ShmHeader* h, std::string* why = nullptr);
  ~DevRingMap();
  RingSlot* req() const { return req_; }

 private:
  void* map_ = nullptr;
  size_t len_ = 0;
  RingSlot* req_ = nullptr;
};

// Attach to a dispatcher segment: the view (with the device ring mapped when the
// server placed it there) and the mapping that keeps it alive.  Throws when the
// server's ring is on the device and cannot be mapped here.
ShmView shm_attach_view(const std::shared_ptr<ShmSegment>& seg, std::shared_ptr<DevRingMap>* devmap);

// Publish one request into the segment's ring and wait for its reply (any
// process).  `poke` is called when the dispatcher is not running.
ReplyRecord shm_call(const ShmView& v, const MsgRecord& m, double timeout_s);

// A CPU stand-in for the GPU's persistent dispatcher on a segment of its own:
// the same protocol (requests strictly in sequence order, 16-B reply tag +
// value), stateless handlers only (Calculator.Multiply, Echo; anything else
// answers kStatusNoMethod).  For GPU-less hosts and the ring-protocol tests
// (liveness with stopped and killed callers).
class HostDispatcher {
 public:
  HostDispatcher(const std::string& name, uint32_t ring);
  ~HostDispatcher();
  HostDispatcher(const HostDispatcher&) = delete;
  HostDispatcher& operator=(const HostDispatcher&) = delete;
  const std::string& name() const { return seg_->name(); }
  uint64_t processed() const { return processed_.load(); }
  uint64_t noops() const { return noops_.load(); }  // rescued numbers (method 0) answered

 private:
  void loop();
  std::shared_ptr<ShmSegment> seg_;
  ShmView v_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> processed_{0}, noops_{0};
  std::thread thread_;
};

// port -> segment locator written by a listening net/rpc server with
// shared-memory device methods ("/ptype-port-<port>").
void shm_locator_publish(int port, const std::string& segment);
void shm_locator_remove(int port);
std::string shm_locator_lookup(int port);  // "" if none or its owner is gone

}  // namespace ptype
