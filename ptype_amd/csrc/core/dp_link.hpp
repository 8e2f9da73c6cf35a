// What the control plane's DataPlane (dataplane.hpp, module _core, g++) and the
// device runtime's engines (module _hip, hipcc) share at run time -- header-only
// and layout-stable, so neither module links the other:
//
//   CommCell         the live RCCL communicator of a data-plane generation.  The
//                    DataPlane owns it; an engine brackets every RCCL enqueue with
//                    enter() / leave() and polls `poisoned` in its host waits.  A
//                    Send watchdog (any thread) retires the cell: poison, wait for
//                    the enqueues in flight to leave, THEN ncclCommAbort -- an engine
//                    never touches a freed communicator (the abort race).
//   DpTransportOps   a non-RCCL transport the DataPlane drives through a C table the
//                    device runtime fills (IpcComm: shared-memory segments between
//                    the processes of one GPU): the same form / abort / settle /
//                    next-generation code runs over RCCL or over IpcComm.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <thread>

namespace ptype {

struct CommCell {
  std::atomic<void*> comm{nullptr};  // ncclComm_t of the generation in force
  std::atomic<int> users{0};         // enqueues in flight (enter .. leave)
  std::atomic<int> poisoned{0};      // the generation failed: no new enqueue, host waits end

  // The communicator for one enqueue, or nullptr once poisoned / retired (the
  // caller raises a rank failure).  Every non-null return pairs with leave().
  void* enter() {
    users.fetch_add(1, std::memory_order_acq_rel);
    void* c = poisoned.load(std::memory_order_acquire) ? nullptr : comm.load(std::memory_order_acquire);
    if (!c) users.fetch_sub(1, std::memory_order_acq_rel);
    return c;
  }
  void leave() { users.fetch_sub(1, std::memory_order_acq_rel); }
  bool failed() const { return poisoned.load(std::memory_order_acquire) != 0; }
  // Poison, wait (at most wait_s) for the enqueues in flight, and hand back the
  // communicator to abort (once: later calls return nullptr).  An enqueue stuck in
  // RCCL past wait_s (a group connecting to a dead peer) is aborted underneath:
  // the alternative is a hang.
  void* retire(double wait_s) {
    poisoned.store(1, std::memory_order_release);
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(wait_s);
    while (users.load(std::memory_order_acquire) > 0 && std::chrono::steady_clock::now() < t_end)
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    return comm.exchange(nullptr, std::memory_order_acq_rel);
  }
  // a fresh generation
  void install(void* c) {
    comm.store(c, std::memory_order_release);
    poisoned.store(0, std::memory_order_release);
  }
};

constexpr uint32_t kDpTransportAbi = 1;

// Non-RCCL transport, one endpoint per process (h: opaque).  Every call that can
// fail returns 0 on success and writes a message into err otherwise.
struct DpTransportOps {
  uint32_t abi;
  void* (*open)(int device, int world, int rank, uint64_t cap_bytes, double timeout_s, const char* name, char* err,
                size_t errlen);
  int (*connect)(void* h, const char* const* names, int count, char* err, size_t errlen);  // every rank's name
  void (*seal)(void* h);  // after EVERY rank connected: remove this rank's name
  // element-wise MAX of n device words, in place, enqueued on stream
  int (*allreduce_max)(void* h, uint64_t* dev, int n, void* stream, char* err, size_t errlen);
  // regions `stride` bytes apart: send_bytes[q] of region q to peer q, recv_bytes[p] into region p
  int (*alltoallv)(void* h, const void* src, void* dst, size_t stride, const size_t* send_bytes,
                   const size_t* recv_bytes, void* stream, char* err, size_t errlen);
  int (*failed)(void* h);     // nonzero once a collective failed (a peer missed it) or abort() ran
  void (*abort)(void* h);     // fail every pending and later collective of this endpoint at once
  uint64_t (*cap)(void* h);   // bytes per peer region one op moves at most
  void* (*engine_ref)(void* h);  // a new reference for the engines (the binding adopts it)
  void (*release)(void* h);      // the DataPlane's reference
};

}  // namespace ptype
