// GPU-initiated remote call: a kernel on this GPU
// calls an actor served by ANOTHER process's persistent dispatcher -- on this
// GPU or a peer over xGMI -- with no host on the call's path.
//
// The reference's remote Call is one request/reply to a remote node
// (cluster/rpc.go:59-67, dialled at :272-285).  Here the caller process maps
// the server's shared-memory segment (shmring.hpp), registers it with HIP, and
// claims one of the segment's peer lanes.  Then a call is, inside a kernel:
//
//   store w0, a0, a1, a2 into the lane
//   system fence; store req_tag = seq + 1        (publish)
//   spin on the lane's reply slot until its tag names seq (bounded by a timeout)
//
// and the server's dispatcher wave, which polls its lanes next to its request
// ring, runs the handler and writes {value, tag} into the reply slot with one
// 16-B store.  Lane and reply slot are host shared memory that each side
// reaches through its OWN mapping, so neither process ever touches memory the
// other owns: a dead server costs the caller its timeout (kStatusNotDelivered),
// a dead caller costs the server nothing (round 4 imported each
// side's HBM, and a killed peer's HBM faulted the survivor's GPU).  One lane
// carries one call at a time; a process that needs more concurrency registers
// more lanes.
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

// A peer's dispatcher segment mapped and registered with HIP in this process
// (its own mapping: it outlives the peer).
class PeerSegment {
 public:
  PeerSegment(const std::string& shm_name, int device) : device_(device) {
    seg_ = ShmSegment::attach(shm_name);
    if (!seg_) throw std::runtime_error("peer lane: no dispatcher segment " + shm_name);
    hdr_ = static_cast<ShmHeader*>(seg_->base());
    if (seg_->size() < sizeof(ShmHeader) || __atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) != kShmMagic)
      throw std::runtime_error("peer lane: segment " + shm_name + " is not a ptype dispatcher (or another version)");
    if (!hdr_->xl_valid) throw std::runtime_error("peer lane: the server exports no GPU lanes");
    if (seg_->size() < shm_bytes(hdr_->ring)) throw std::runtime_error("peer lane: segment too small");
    view_ = shm_view(seg_->base(), hdr_->ring);
    PT_HIP_CHECK(hipSetDevice(device_));
    PT_HIP_CHECK(hipHostRegister(seg_->base(), seg_->size(), hipHostRegisterMapped | hipHostRegisterPortable));
    char* dbase = nullptr;
    PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dbase, seg_->base(), 0));
    const char* hbase = static_cast<const char*>(seg_->base());
    dxl_ = reinterpret_cast<XLane*>(dbase + (reinterpret_cast<const char*>(view_.xl) - hbase));
    dxrep_ = reinterpret_cast<XReply*>(dbase + (reinterpret_cast<const char*>(view_.xrep) - hbase));
  }
  ~PeerSegment() {
    (void)hipSetDevice(device_);
    (void)hipHostUnregister(seg_->base());
  }
  PeerSegment(const PeerSegment&) = delete;
  PeerSegment& operator=(const PeerSegment&) = delete;
  ShmHeader* hdr() const { return hdr_; }
  XLane* dev_lane(int i) const { return dxl_ + i; }
  XReply* dev_reply(int i) const { return dxrep_ + i; }
  const ShmView& view() const { return view_; }
  void wake() const {
    hdr_->wake.store(1, std::memory_order_release);
    shm_futex_wake(&hdr_->wake);
  }

 private:
  int device_;
  std::shared_ptr<ShmSegment> seg_;
  ShmHeader* hdr_ = nullptr;
  ShmView view_;
  XLane* dxl_ = nullptr;
  XReply* dxrep_ = nullptr;
};

class PeerLane {
 public:
  // Attach to the dispatcher segment `shm_name` (same node) and register a lane.
  PeerLane(const std::string& shm_name, int device, double timeout_s = 10.0)
      : PeerLane(std::make_shared<PeerSegment>(shm_name, device), device, timeout_s) {}
  PeerLane(std::shared_ptr<PeerSegment> seg, int device, double timeout_s) : device_(device), seg_(std::move(seg)) {
    ShmHeader* h = seg_->hdr();
    PT_HIP_CHECK(hipSetDevice(device_));
    PT_HIP_CHECK(hipMalloc((void**)&done_, 64));
    const uint64_t me = ring_self_token();
    for (int i = 0; i < kXLanes && lane_ < 0; ++i) {
      uint64_t z = 0;
      if (h->xregs[i].token.compare_exchange_strong(z, me)) lane_ = i;
    }
    if (lane_ < 0) throw std::runtime_error("peer lane: all lanes of the server are taken");
    XLaneReg& g = h->xregs[lane_];
    g.device = device_;
    g.state.store(kXLaneRequested, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {  // the server's waker resets the lane and admits it
      seg_->wake();
      const uint32_t st = g.state.load(std::memory_order_acquire);
      if (st == kXLaneReady) break;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
        release();
        throw std::runtime_error("peer lane: registration timed out (is the server alive?)");
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
  // are kStatusNotDelivered and the lane is released: register a new one).
  int64_t call(uintptr_t actor, uintptr_t method, int method_uniform, uintptr_t a0, uintptr_t a1, uintptr_t a2,
               int64_t n, uintptr_t out_val, uintptr_t out_st, uintptr_t ticks, double timeout_s, uintptr_t stream) {
    if (lane_ < 0) throw std::runtime_error("peer lane: closed");
    if (n <= 0) return 0;
    PT_HIP_CHECK(hipSetDevice(device_));
    seg_->wake();  // a parked dispatcher relaunches (its waker polls anyway)
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(xcall_kernel, dim3(1), dim3(64), 0, s, seg_->dev_lane(lane_),
                       reinterpret_cast<const uint64_t*>(seg_->dev_reply(lane_)), seq_, (const uint32_t*)actor,
                       (const uint16_t*)method, (uint16_t)method_uniform, (const int64_t*)a0, (const int64_t*)a1,
                       (const int64_t*)a2, n, (int64_t*)out_val, (int32_t*)out_st, (uint64_t*)ticks,
                       (uint64_t)(timeout_s * 1e8), done_);
    PT_HIP_CHECK(hipGetLastError());
    uint64_t done = 0;
    PT_HIP_CHECK(hipMemcpyAsync(&done, done_, sizeof done, hipMemcpyDeviceToHost, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
    seq_ += done;
    if ((int64_t)done < n || (done && last_status_failed(out_st, done, s))) release();
    return (int64_t)done;
  }

  int lane() const { return lane_; }
  uint64_t calls() const { return seq_; }
  // the lane as a relay slot (its device addresses); the caller must not also
  // call() through it (the relaying dispatcher owns the sequence)
  XLane* peer_lane() const { return lane_ >= 0 ? seg_->dev_lane(lane_) : nullptr; }
  XReply* reply_slot() const { return lane_ >= 0 ? seg_->dev_reply(lane_) : nullptr; }

 private:
  bool last_status_failed(uintptr_t out_st, uint64_t done, hipStream_t s) {
    int32_t st = 0;
    PT_HIP_CHECK(hipMemcpyAsync(&st, (const int32_t*)out_st + (done - 1), sizeof st, hipMemcpyDeviceToHost, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
    return st == kStatusNotDelivered;
  }
  // The lane goes Releasing; the server's waker resets and frees it once no
  // request is in flight (a dead server never does -- nothing to wait for then:
  // the lane lives in shared memory, not in either process's allocations).
  void release() {
    if (lane_ >= 0) {
      XLaneReg& g = seg_->hdr()->xregs[lane_];
      g.state.store(kXLaneReleasing, std::memory_order_release);
      seg_->wake();
      lane_ = -1;
    }
    if (done_) (void)hipFree(done_);
    done_ = nullptr;
  }

  int device_;
  std::shared_ptr<PeerSegment> seg_;
  uint64_t* done_ = nullptr;
  int lane_ = -1;
  uint64_t seq_ = 0;
};

// Handler-initiated remote calls: n peer lanes on another process's dispatcher,
// handed to THIS process's dispatcher as a relay table.  A kMethodRelay request
// it serves is published by the dispatcher wave into a free lane and parked
// there; the wave keeps serving, and the remote actor's reply, when it lands,
// completes the call (server.hpp relay_post / relay_poll).  Reference: a server
// handler that itself dials and Calls another node (cluster/rpc.go:59-67), one
// goroutine per request (example/calculator/server/server.go:16-20).
class PeerRelay {
 public:
  PeerRelay(const std::string& shm_name, int device, int n_lanes, double timeout_s) : device_(device) {
    if (n_lanes < 1 || n_lanes > kRelayMax) throw std::invalid_argument("PeerRelay: 1..64 lanes");
    seg_ = std::make_shared<PeerSegment>(shm_name, device);
    for (int i = 0; i < n_lanes; ++i) lanes_.push_back(std::make_shared<PeerLane>(seg_, device, 10.0));
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
    lanes_.clear();
    (void)hipFree(table_);
  }
  PeerRelay(const PeerRelay&) = delete;
  PeerRelay& operator=(const PeerRelay&) = delete;
  uintptr_t table() const { return (uintptr_t)table_; }
  int lanes() const { return (int)lanes_.size(); }
  // slot words {seq, suspect} per lane as the device table holds them (written back when the wave parks)
  std::vector<uint64_t> slots() const {
    RelayTable t{};
    PT_HIP_CHECK(hipMemcpy(&t, table_, sizeof t, hipMemcpyDeviceToHost));
    std::vector<uint64_t> v;
    for (uint32_t i = 0; i < t.n; ++i) {
      v.push_back(t.lanes[i].seq);
      v.push_back(t.lanes[i].suspect);
    }
    return v;
  }

 private:
  int device_;
  std::shared_ptr<PeerSegment> seg_;
  std::vector<std::shared_ptr<PeerLane>> lanes_;
  RelayTable* table_ = nullptr;
};

}  // namespace ptype
