// GPU-initiated remote call: a kernel on this GPU
// calls an actor served by ANOTHER process's persistent dispatcher -- on this
// GPU or a peer over xGMI -- with no host on the call's path.
//
// The reference's remote Call is one request/reply to a remote node
// (cluster/rpc.go:59-67, dialled at :272-285).  Here the caller process
// attaches to the server's shared-memory segment (shmring.hpp), imports its
// GPU peer-lane array with hipIpcOpenMemHandle, and registers one lane: the
// lane's reply slot is 16 B of fine-grained memory in THIS process's HBM whose
// IPC handle the server imports.  Then a call is, inside a kernel:
//
//   store w0, a0, a1, a2 into the lane (remote stores through the import)
//   system fence; store req_tag = seq + 1        (publish)
//   spin on the LOCAL reply slot until its tag names seq (bounded by a timeout)
//
// and the server's dispatcher wave, which polls its lanes in HBM next to its
// request ring, runs the handler and writes {value, tag} into the caller's slot
// with one 16-B store.  One lane carries one call at a time; a process that
// needs more concurrency registers more lanes.  If the server dies, the caller's
// spin ends at its timeout with kStatusNotDelivered.
#pragma once
#include <chrono>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "shmring.hpp"

namespace ptype {

__device__ __forceinline__ uint64_t xc_ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void xc_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// n calls in sequence from one lane of one wave (the rest of the wave idles):
// call k publishes seq0 + k and waits for its reply before the next.  ticks[k]
// = publish -> reply seen, s_memrealtime ticks (100 MHz).
__global__ __launch_bounds__(64) void xcall_kernel(XLane* __restrict__ lane, const uint64_t* __restrict__ reply,
                                                   uint64_t seq0, const uint32_t* __restrict__ actor,
                                                   const uint16_t* __restrict__ method, uint16_t method_uniform,
                                                   const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
                                                   const int64_t* __restrict__ a2, int64_t n,
                                                   int64_t* __restrict__ out_val, int32_t* __restrict__ out_st,
                                                   uint64_t* __restrict__ ticks, uint64_t timeout_ticks,
                                                   uint64_t* __restrict__ done) {
  if (threadIdx.x != 0) return;
  uint64_t k = 0;
  for (; k < (uint64_t)n; ++k) {
    const uint64_t seq = seq0 + k;
    const uint64_t m = method ? method[k] : method_uniform;
    const uint64_t w0 = (uint64_t)actor[k] | (m << 32) | ((uint64_t)kFlagValid << 48);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    xc_st(&lane->w0, w0);
    xc_st(reinterpret_cast<uint64_t*>(&lane->a0), (uint64_t)(a0 ? a0[k] : 0));
    xc_st(reinterpret_cast<uint64_t*>(&lane->a1), (uint64_t)(a1 ? a1[k] : 0));
    xc_st(reinterpret_cast<uint64_t*>(&lane->a2), (uint64_t)(a2 ? a2[k] : 0));
    __threadfence_system();
    xc_st(&lane->req_tag, seq + 1);
    int32_t status = kStatusNotDelivered;
    int64_t value = 0;
    for (;;) {
      const uint64_t tag = xc_ld(reply + 1);
      if (reply_tag_is(tag, seq)) {
        const int64_t v = (int64_t)xc_ld(reply);
        if (xc_ld(reply + 1) != tag) continue;  // the value belongs to this tag only if it still carries it
        value = v;
        status = (int32_t)(tag & 0xff);
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) break;
      __builtin_amdgcn_s_sleep(1);
    }
    out_val[k] = value;
    out_st[k] = status;
    if (ticks) ticks[k] = __builtin_amdgcn_s_memrealtime() - t0;
    if (status == kStatusNotDelivered) {  // the lane is out of step now: stop here
      ++k;
      break;
    }
  }
  *done = k;
}

class PeerLane {
 public:
  // Attach to the dispatcher segment `shm_name` (same node) and register a lane
  // whose reply slot lives on `device` (this process's GPU).
  PeerLane(const std::string& shm_name, int device, double timeout_s = 10.0) : device_(device) {
    seg_ = ShmSegment::attach(shm_name);
    if (!seg_) throw std::runtime_error("peer lane: no dispatcher segment " + shm_name);
    hdr_ = static_cast<ShmHeader*>(seg_->base());
    if (seg_->size() < sizeof(ShmHeader) || __atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) != kShmMagic)
      throw std::runtime_error("peer lane: segment " + shm_name + " is not a ptype dispatcher");
    if (!hdr_->xl_valid) throw std::runtime_error("peer lane: the server exports no GPU lanes");
    PT_HIP_CHECK(hipSetDevice(device_));
    hipIpcMemHandle_t h;
    memcpy(&h, hdr_->xl_ipc, sizeof h);
    void* p = nullptr;
    PT_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    peer_ = static_cast<XLane*>(p);
    PT_HIP_CHECK(hipExtMallocWithFlags((void**)&reply_, 4096, hipDeviceMallocFinegrained));
    PT_HIP_CHECK(hipMemset(reply_, 0, 4096));
    PT_HIP_CHECK(hipMalloc((void**)&done_, 64));
    PT_HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t rh;
    PT_HIP_CHECK(hipIpcGetMemHandle(&rh, reply_));
    const uint64_t me = ring_self_token();
    for (int i = 0; i < kXLanes && lane_ < 0; ++i) {
      uint64_t z = 0;
      if (hdr_->xregs[i].token.compare_exchange_strong(z, me)) lane_ = i;
    }
    if (lane_ < 0) throw std::runtime_error("peer lane: all lanes of the server are taken");
    XLaneReg& g = hdr_->xregs[lane_];
    memcpy(g.reply_ipc, &rh, sizeof rh);
    g.device = device_;
    g.state.store(kXLaneRequested, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {  // the server's waker admits the lane (imports the reply slot)
      hdr_->wake.store(1, std::memory_order_release);
      shm_futex_wake(&hdr_->wake);
      const uint32_t st = g.state.load(std::memory_order_acquire);
      if (st == kXLaneReady) break;
      if (st == kXLaneFailed) {
        release();
        throw std::runtime_error("peer lane: the server could not import the reply slot");
      }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
        release();
        throw std::runtime_error("peer lane: registration timed out");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }

  ~PeerLane() {
    try {
      release();
    } catch (...) {
    }
  }

  // n calls in one kernel on `stream` (columns are device pointers; method
  // column optional).  Returns how many completed (the rest after a timeout
  // are kStatusNotDelivered and the lane is retired).
  int64_t call(uintptr_t actor, uintptr_t method, int method_uniform, uintptr_t a0, uintptr_t a1, uintptr_t a2,
               int64_t n, uintptr_t out_val, uintptr_t out_st, uintptr_t ticks, double timeout_s, uintptr_t stream) {
    if (lane_ < 0) throw std::runtime_error("peer lane: closed");
    if (n <= 0) return 0;
    PT_HIP_CHECK(hipSetDevice(device_));
    hdr_->wake.store(1, std::memory_order_release);  // a parked dispatcher relaunches (its waker polls anyway)
    shm_futex_wake(&hdr_->wake);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(xcall_kernel, dim3(1), dim3(64), 0, s, peer_ + lane_, (const uint64_t*)reply_, seq_,
                       (const uint32_t*)actor, (const uint16_t*)method, (uint16_t)method_uniform,
                       (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2, n, (int64_t*)out_val,
                       (int32_t*)out_st, (uint64_t*)ticks, (uint64_t)(timeout_s * 1e8), done_);
    PT_HIP_CHECK(hipGetLastError());
    uint64_t done = 0;
    PT_HIP_CHECK(hipMemcpyAsync(&done, done_, sizeof done, hipMemcpyDeviceToHost, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
    seq_ += done;
    if ((int64_t)done < n || (done && last_status_failed(out_st, done, s))) retire();
    return (int64_t)done;
  }

  int lane() const { return lane_; }
  uint64_t calls() const { return seq_; }
  // the lane as a relay slot: the peer's lane (imported) and this process's reply
  // slot; the caller must not also call() through it (PeerRelay owns the sequence)
  XLane* peer_lane() const { return lane_ >= 0 ? peer_ + lane_ : nullptr; }
  uint64_t* reply_slot() const { return reply_; }

 private:
  bool last_status_failed(uintptr_t out_st, uint64_t done, hipStream_t s) {
    int32_t st = 0;
    PT_HIP_CHECK(hipMemcpyAsync(&st, (const int32_t*)out_st + (done - 1), sizeof st, hipMemcpyDeviceToHost, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
    return st == kStatusNotDelivered;
  }
  void retire() { release(); }
  // Two-phase release: the lane goes Releasing, the server's waker
  // closes its import of our reply slot once no request is in flight and marks
  // the lane Free -- only then is the slot freed here.  If the server does not
  // answer within the bound (it died, or a handler is stuck), the 4 KB slot is
  // leaked rather than freed under a possible late reply store.
  void release() {
    bool acked = true;
    if (lane_ >= 0) {
      XLaneReg& g = hdr_->xregs[lane_];
      g.state.store(kXLaneReleasing, std::memory_order_release);
      const auto t0 = std::chrono::steady_clock::now();
      acked = false;
      for (;;) {
        hdr_->wake.store(1, std::memory_order_release);
        shm_futex_wake(&hdr_->wake);
        if (g.state.load(std::memory_order_acquire) == kXLaneFree) {
          acked = true;
          break;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > release_wait_s_) break;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
      lane_ = -1;
    }
    if (peer_) (void)hipIpcCloseMemHandle(peer_);
    peer_ = nullptr;
    if (reply_) {
      if (acked) (void)hipFree(reply_);
      else ++leaked_slots_;
      reply_ = nullptr;
    }
    if (done_) (void)hipFree(done_);
    done_ = nullptr;
  }

 public:
  static uint64_t leaked_slots() { return leaked_slots_; }

 private:
  double release_wait_s_ = 2.0;
  static inline uint64_t leaked_slots_ = 0;
  int device_;
  std::shared_ptr<ShmSegment> seg_;
  ShmHeader* hdr_ = nullptr;
  XLane* peer_ = nullptr;
  uint64_t* reply_ = nullptr;
  uint64_t* done_ = nullptr;
  int lane_ = -1;
  uint64_t seq_ = 0;
};

// Handler-initiated remote calls: n peer lanes on another process's dispatcher,
// handed to THIS process's dispatcher as a relay table.  A kMethodRelay request
// it serves (server.hpp relay_calls) is forwarded from the dispatcher wave
// through a lane -- publish into the peer's HBM, spin on the local reply slot --
// and the remote actor's reply returned as the call's own.  Reference: a server
// handler that itself dials and Calls another node (cluster/rpc.go:59-67).
class PeerRelay {
 public:
  PeerRelay(const std::string& shm_name, int device, int n_lanes, double timeout_s) : device_(device) {
    if (n_lanes < 1 || n_lanes > kRelayMax) throw std::invalid_argument("PeerRelay: 1..64 lanes");
    for (int i = 0; i < n_lanes; ++i) lanes_.push_back(std::make_shared<PeerLane>(shm_name, device, 10.0));
    RelayTable t{};
    for (int i = 0; i < n_lanes; ++i) t.lanes[i] = RelayLane{lanes_[(size_t)i]->peer_lane(), lanes_[(size_t)i]->reply_slot(), 0, 0};
    t.n = (uint32_t)n_lanes;
    t.timeout_ticks = (uint64_t)(timeout_s * 1e8);
    PT_HIP_CHECK(hipSetDevice(device_));
    PT_HIP_CHECK(hipMalloc((void**)&table_, sizeof(RelayTable)));
    PT_HIP_CHECK(hipMemcpy(table_, &t, sizeof t, hipMemcpyHostToDevice));
  }
  ~PeerRelay() {
    (void)hipSetDevice(device_);
    lanes_.clear();  // lanes first: their release waits for the peer to let go of the reply slots
    (void)hipFree(table_);
  }
  PeerRelay(const PeerRelay&) = delete;
  PeerRelay& operator=(const PeerRelay&) = delete;
  uintptr_t table() const { return (uintptr_t)table_; }
  int lanes() const { return (int)lanes_.size(); }

 private:
  int device_;
  std::vector<std::shared_ptr<PeerLane>> lanes_;
  RelayTable* table_ = nullptr;
};

}  // namespace ptype
