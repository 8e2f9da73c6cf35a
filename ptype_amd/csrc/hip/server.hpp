// Persistent device dispatcher: the latency path of `Client.Call` on a GPU actor
// (SURVEY C10 / K3 persistent form, K8 fused).
//
// Reference: each net/rpc call is one TCP round trip into a goroutine that runs
// the handler (cluster/rpc.go:59-67 -> stdlib net/rpc server, registered at
// example/calculator/server/server.go:16-20).  Here the host publishes a 64-B
// request slot into a ring; ONE resident
// wave polls the ring with relaxed system-scope loads + s_sleep, runs up to 64
// consecutive requests per poll (one per lane) through the same compiled-in
// handler table as the batch path, and writes reply slots back as single 16-B
// system-scope stores.  No kernel launch per call.  In-process, the request
// ring is fine-grained DEVICE memory the host writes through its BAR mapping
// (polls and payload reads stay on the GPU: p50 RTT 4.0-4.5 -> 3.1 us,
// profiles/r1_ring_placement_ab.txt); for other processes the same device ring
// is exported as a dma-buf they map (shmring.hpp), with replies in host shm.
//
// Liveness: the kernel exits when the host sets `stop`, when it has been idle
// for `idle_ticks`, or after `max_ticks` (a hard bound so nothing can hang the
// GPU).  Exit uses a Dekker-style hand-off on `state` so a request published
// while the kernel retires is never stranded: the kernel stores STOPPED,
// re-checks the ring, and resumes only by CAS(STOPPED->RUNNING); the host, after
// publishing, relaunches only by CAS(STOPPED->LAUNCHING).
#pragma once
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include "common.hpp"
#include "tune.hpp"
#include "handlers.hpp"
#include "ringproto.hpp"
#include "shmring.hpp"

namespace ptype {

// Whether the host CPU can read and write `p` directly (device memory mapped
// through the BAR): the pointer's accessible agents include a CPU agent.  The
// module links libhsa-runtime64.so.1, which resolves (RUNPATH, same soname) to
// the HSA runtime torch's HIP already loaded -- one runtime in the process.
inline bool cpu_can_access(const void* p);

inline hsa_status_t find_cpu_agent(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// Open device allocation `p` to the host CPU (large-BAR mapping) and confirm it.
inline bool open_to_cpu(const void* p) {
  hsa_agent_t cpu{};
  hsa_iterate_agents(find_cpu_agent, &cpu);
  if (!cpu.handle) return false;
  const hsa_status_t st = hsa_amd_agents_allow_access(1, &cpu, nullptr, p);
  if (st != HSA_STATUS_SUCCESS) {
    if (getenv("PTYPE_DEBUG")) fprintf(stderr, "ptype: hsa_amd_agents_allow_access -> %d\n", (int)st);
    return false;
  }
  // (the pointer's accessible-agent list does not name the CPU for device
  // memory even after this succeeds; success is the runtime's mapping promise)
  cpu_can_access(p);  // debug report only
  return true;
}

inline bool cpu_can_access(const void* p) {
  const bool dbg = getenv("PTYPE_DEBUG") != nullptr;
  hsa_amd_pointer_info_t info{};
  info.size = sizeof(info);
  uint32_t n = 0;
  hsa_agent_t* agents = nullptr;
  const hsa_status_t st = hsa_amd_pointer_info(p, &info, malloc, &n, &agents);
  if (st != HSA_STATUS_SUCCESS) {
    if (dbg) fprintf(stderr, "ptype: hsa_amd_pointer_info -> %d\n", (int)st);
    return false;
  }
  bool cpu = false;
  for (uint32_t i = 0; i < n; ++i) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(agents[i], HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU)
      cpu = true;
  }
  free(agents);
  if (dbg) fprintf(stderr, "ptype: ring %p type %d, %u accessible agents, cpu %d\n", p, (int)info.type, n, (int)cpu);
  return cpu;
}

// ServerState / ServerCtrl live in records.hpp (shared with the cross-process client).

__device__ __forceinline__ uint64_t sys_ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16 aligned bytes in ONE system-coherent vector store (what sys_st emits for 8 B,
// `sc0 sc1`, at dwordx4 width): a single write to host memory, not two.
__device__ __forceinline__ void sys_st16(uint64_t* p, uint64_t lo, uint64_t hi) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const u64x2 v{lo, hi};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

// How the wave polls the ring (tune poll_lanes / poll_full / poll_sleep, tune.hpp):
// slots whose tag is read per trip (= most requests taken per batch), whether the
// head slot's message is read in the same trip (checksum-validated), and how
// many s_sleep(1) pauses separate empty polls.  Measured on MI355X
// (tools/latency_sweep.py, profiles/r1_latency_sweep.jsonl): reading the head
// slot whole in every poll saves the second round trip but costs more than it
// saves -- p50 6.0 us vs 4.0-4.2 us with tag-only polls (the device's reads of
// the line the host is writing slow the host's publish) -- so it is off.
struct PollConfig {
  uint32_t lanes = 64;
  uint32_t full = 0;
  uint32_t sleep = 1;
};

// GPU peer lanes (shmring.hpp XLane, in the segment): lane l of the wave serves
// XLane l.  A request is pending when req_tag == served + 1; the reply goes into
// the lane's reply slot (XReply l, also in the segment) as one 16-B store, then
// `served` acknowledges.  Returns the number of lanes served (wave-uniform).
__device__ __forceinline__ unsigned serve_xlanes(XLane* __restrict__ xl, XReply* __restrict__ xrep, uint32_t nx,
                                                 int64_t* __restrict__ state, uint32_t n_state,
                                                 uint64_t delay_ticks) {
  const unsigned lane = lane_id();
  bool ready = false;
  uint64_t t = 0;
  if (xl && lane < nx) {
    t = sys_ld(&xl[lane].req_tag);
    ready = t != 0 && t == sys_ld(&xl[lane].served) + 1;
  }
  const uint64_t m = __ballot(ready);
  if (!m) return 0;
  if (ready) {  // payload loads ordered after the tag load (the branch waits for it)
    XLane* L = &xl[lane];
    const uint64_t w0 = sys_ld(&L->w0);
    MsgRecord msg;
    msg.actor = (uint32_t)w0;
    msg.method = (uint16_t)(w0 >> 32);
    msg.flags = (uint16_t)(w0 >> 48);
    msg.a0 = (int64_t)sys_ld(reinterpret_cast<const uint64_t*>(&L->a0));
    msg.a1 = (int64_t)sys_ld(reinterpret_cast<const uint64_t*>(&L->a1));
    msg.a2 = (int64_t)sys_ld(reinterpret_cast<const uint64_t*>(&L->a2));
    const ReplyRecord r = run_handler(msg, state, n_state, delay_ticks);
    sys_st16(reinterpret_cast<uint64_t*>(&xrep[lane]), (uint64_t)r.value, reply_tag(t - 1, (uint32_t)r.status));
    __threadfence_system();
    sys_st(&L->served, t);
  }
  return (unsigned)__popcll(m);
}

// Relay table (kMethodRelay): one GPU peer lane of ANOTHER server per relay slot
// -- its lane and reply slot in that server's segment (mapped and registered by
// this process), the lane's next sequence and whether a timed-out call on it is
// still unanswered.  Built by PeerRelay (xcall.hpp).  While the dispatcher wave
// runs, slot l's words live in lane l's registers (RelayRegs); they are written
// back when the wave parks or the table is replaced.
struct RelayLane {
  XLane* lane;
  XReply* reply;
  uint64_t seq;      // the sequence of the lane's next call
  uint64_t suspect;  // 1: call `seq` timed out -- the slot is reused once its late reply lands
};
constexpr int kRelayMax = 64;
struct RelayTable {
  RelayLane lanes[kRelayMax];
  uint32_t n;  // slots in use
  uint32_t pad;
  uint64_t timeout_ticks;
};

// Asynchronous relays: the wave never waits on a peer.  A relayed
// request takes a free slot, is published into the peer's lane, and parks there
// (pend = its ring sequence + 1) while the wave goes on serving its ring, its own
// peer lanes and other relays; every trip polls the parked slots' reply words,
// and a reply (or the slot's deadline) completes the ring request it belongs to.
// A timed-out call fails that call only: the slot is suspect until the late reply
// lands (then free again), never retired.  A peer that died leaves its slots
// suspect -- their memory is this process's mapping of the peer's segment, so
// nothing faults.
struct RelayRegs {
  uint64_t seq = 0, pend = 0, deadline = 0;
  XLane* x = nullptr;
  XReply* rp = nullptr;
  bool suspect = false;
  uint32_t cont = 0;  // kMethodCoordPrime: the local actor + 1 whose continuation runs on the reply
  int64_t cont_n = 0;  // ... and its candidate
};
// slot words through memory-side atomics: the wave may be relaunched on another
// XCD, whose L2 could hold a line of the table from an earlier run
__device__ __forceinline__ uint64_t relay_ld(uint64_t* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void relay_st(uint64_t* p, uint64_t v) {
  (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ RelayRegs relay_load(RelayTable* rt) {
  RelayRegs g;
  const unsigned lane = lane_id();
  if (!rt || lane >= (unsigned)relay_ld(reinterpret_cast<uint64_t*>(&rt->n)) % 0x100000000ull) return g;
  RelayLane* L = &rt->lanes[lane];
  g.x = reinterpret_cast<XLane*>(relay_ld(reinterpret_cast<uint64_t*>(&L->lane)));
  g.rp = reinterpret_cast<XReply*>(relay_ld(reinterpret_cast<uint64_t*>(&L->reply)));
  g.seq = relay_ld(&L->seq);
  g.suspect = relay_ld(&L->suspect) != 0;
  return g;
}
__device__ __forceinline__ void relay_store(RelayTable* rt, const RelayRegs& g) {
  if (!rt || !g.x) return;
  RelayLane* L = &rt->lanes[lane_id()];
  relay_st(&L->seq, g.seq);
  relay_st(&L->suspect, g.suspect ? 1ull : 0ull);
}

// Complete parked relays whose reply landed or whose deadline passed (their ring
// replies written here); clear suspect slots whose late reply landed.  Returns
// the number of ring requests completed (wave-uniform).
__device__ __forceinline__ unsigned relay_poll(RelayRegs& g, ReplySlot* __restrict__ rep, uint64_t ring_mask,
                                               uint64_t now, int64_t* __restrict__ state, uint32_t n_state) {
  bool fin = false;
  if (g.pend || g.suspect) {
    const uint64_t tag = sys_ld(&g.rp->tag);
    bool got = reply_tag_is(tag, g.seq);
    int64_t v = 0;
    if (got) {
      v = (int64_t)sys_ld(&g.rp->value);
      got = sys_ld(&g.rp->tag) == tag;  // the value belongs to this tag only if it still carries it
    }
    if (g.pend) {
      const uint64_t seq = g.pend - 1;
      if (got) {
        uint32_t st = (uint32_t)(tag & 0xff);
        if (g.cont) {  // the coordinator's continuation: tally a prime into its own state
          const uint32_t a = g.cont - 1;
          if (!state || a >= n_state) {
            v = 0, st = kStatusNoActor;
          } else if (st == kStatusOk) {
            const bool prime = g.cont_n >= 2 && v == g.cont_n;  // no divisor in [2, isqrt(n)]
            unsigned long long* sp = reinterpret_cast<unsigned long long*>(state + a);
            v = prime ? (int64_t)atomicAdd(sp, 1ull) + 1
                      : (int64_t)__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          g.cont = 0;
        }
        sys_st16(reinterpret_cast<uint64_t*>(&rep[seq & ring_mask]), (uint64_t)v, reply_tag(seq, st));
        g.seq += 1;
        g.pend = 0;
        fin = true;
      } else if (now > g.deadline) {
        sys_st16(reinterpret_cast<uint64_t*>(&rep[seq & ring_mask]), 0ull, reply_tag(seq, kStatusNotDelivered));
        g.suspect = true;  // the peer may still answer call g.seq
        g.pend = 0;
        g.cont = 0;
        fin = true;
      }
    } else if (got) {  // a suspect slot's late reply: the lane is in step again
      g.seq += 1;
      g.suspect = false;
    }
  }
  return (unsigned)__popcll(__ballot(fin));
}

// Relayed ring requests wait for a slot in a FIFO in device memory (one entry of
// 5 words per ring slot: every entry is a ring request not yet answered, so the
// ring's size bounds it), so the ring head never stops behind a relay: requests
// after it are served at once (other callers unaffected).  The
// queue is empty whenever the wave parks (a queued relay is work in flight).
struct RelayQueue {
  uint64_t* q = nullptr;  // [ring][5]: ring seq, w0..w3
  uint64_t mask = 0;      // ring - 1
  uint64_t head = 0, tail = 0;  // wave-uniform
};
__device__ __forceinline__ uint64_t q_ld(const uint64_t* p) {  // another lane's store: past the L1
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Queue this trip's relayed requests (lanes < n flagged in `relayed_mask`, ring
// sequence head + lane), then let every free slot take the next queued request
// in order and publish it into its peer lane.  With no slot parked and requests
// still queued, no slot can free (every one is suspect: the peer stopped
// answering), so the queued requests fail at once (kStatusNotDelivered) -- a dead
// peer never holds them until their callers' timeouts.  Returns the ring
// requests failed here (wave-uniform).
__device__ __forceinline__ unsigned relay_dispatch(RelayRegs& g, RelayQueue& rq, uint64_t relayed_mask,
                                                   uint64_t head, uint64_t w0, uint64_t w1, uint64_t w2,
                                                   uint64_t w3, uint64_t timeout_ticks, uint64_t now,
                                                   ReplySlot* __restrict__ rep, uint64_t ring_mask) {
  const unsigned lane = lane_id();
  const uint64_t below = (1ull << lane) - 1;
  if (relayed_mask) {
    if ((relayed_mask >> lane) & 1) {
      uint64_t* e = rq.q + ((rq.tail + (uint64_t)__popcll(relayed_mask & below)) & rq.mask) * 5;
      e[0] = head + lane, e[1] = w0, e[2] = w1, e[3] = w2, e[4] = w3;
    }
    rq.tail += (uint64_t)__popcll(relayed_mask);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the entries before any lane reads them
  }
  const uint64_t avail = rq.tail - rq.head;
  if (!avail) return 0;
  const uint64_t free_mask = __ballot(g.x != nullptr && !g.pend && !g.suspect);
  const uint64_t q = (uint64_t)__popcll(free_mask & below);
  if (((free_mask >> lane) & 1) && q < avail) {
    const uint64_t* e = rq.q + ((rq.head + q) & rq.mask) * 5;
    const uint64_t seq = q_ld(e), s0 = q_ld(e + 1), s1 = q_ld(e + 2), s2 = q_ld(e + 3), s3 = q_ld(e + 4);
    uint64_t rw0, r0, r1, r2;
    if ((uint16_t)(s0 >> 32) == kMethodCoordPrime) {
      // the coordinator's handler: it picks the worker and builds the PrimeCheck itself
      const int64_t n = (int64_t)s1;
      const uint64_t W = (uint64_t)((int64_t)s2 > 0 ? s2 : 1);
      uint64_t h = (uint64_t)n * 0x9e3779b97f4a7c15ull;
      h ^= h >> 29;
      const uint64_t worker = (uint64_t)s3 + h % W;
      int64_t lim = n > 3 ? (int64_t)sqrt((double)n) + 1 : n;
      while (lim > 2 && (lim - 1) * (lim - 1) > n) --lim;  // (double rounding) isqrt(n) + 1
      rw0 = (worker & 0xffffffffull) | ((uint64_t)kPrimeCheck << 32) | ((uint64_t)kFlagValid << 48);
      r0 = 2, r1 = (uint64_t)lim, r2 = (uint64_t)n;
      g.cont = (uint32_t)s0 + 1;
      g.cont_n = n;
    } else {
      // kMethodRelay: actor = the remote actor, a0 = the remote method, a1 / a2 = its arguments
      rw0 = (s0 & 0xffffffffull) | ((uint64_t)(uint16_t)s1 << 32) | ((uint64_t)kFlagValid << 48);
      r0 = s2, r1 = s3, r2 = 0;
      g.cont = 0;
    }
    sys_st(&g.x->w0, rw0);
    sys_st(reinterpret_cast<uint64_t*>(&g.x->a0), r0);
    sys_st(reinterpret_cast<uint64_t*>(&g.x->a1), r1);
    sys_st(reinterpret_cast<uint64_t*>(&g.x->a2), r2);
    __threadfence_system();
    sys_st(&g.x->req_tag, g.seq + 1);
    g.pend = seq + 1;
    g.deadline = now + timeout_ticks;
  }
  const uint64_t took = min((uint64_t)__popcll(free_mask), avail);
  rq.head += took;
  if (rq.tail == rq.head || __ballot(g.pend != 0)) return 0;
  const uint64_t left = rq.tail - rq.head;  // nothing parked, nothing can free: fail the rest
  for (uint64_t i = lane; i < left; i += kWave) {
    const uint64_t seq = q_ld(rq.q + ((rq.head + i) & rq.mask) * 5);
    sys_st16(reinterpret_cast<uint64_t*>(&rep[seq & ring_mask]), 0ull, reply_tag(seq, kStatusNotDelivered));
  }
  rq.head = rq.tail;
  return (unsigned)left;
}

__global__ __launch_bounds__(64) void persistent_dispatch_kernel(RingSlot* __restrict__ req,
                                                                 ReplySlot* __restrict__ rep, uint64_t ring_mask,
                                                                 ServerCtrl* __restrict__ ctrl, uint64_t head,
                                                                 int64_t* __restrict__ state, uint32_t n_state,
                                                                 uint64_t delay_ticks, uint64_t idle_ticks,
                                                                 uint64_t max_ticks, PollConfig poll,
                                                                 XLane* __restrict__ xl, XReply* __restrict__ xrep,
                                                                 uint32_t nx, uint64_t* __restrict__ relay_q) {
  const unsigned lane = lane_id();
  const uint64_t t_start = realtime_ticks();
  uint64_t last_work = t_start;
  uint64_t processed = 0;
  bool lifetime_exit = false;
  // tracing knobs are re-read on the idle path only, never between a request and its reply
  uint64_t trace_mask = sys_ld(&ctrl->trace_mask);
  TraceRec* trace = reinterpret_cast<TraceRec*>(sys_ld(&ctrl->trace_ring));
  unsigned idle_polls = 0, iters = 0;
  // GPU peer lanes are polled only while some are registered (re-read on the idle path)
  uint32_t nxl = xl ? (uint32_t)min<uint64_t>(sys_ld(&ctrl->xl_n), (uint64_t)nx) : 0u;
  // relay slots: lane l holds slot l (re-read on the idle path while none is parked)
  RelayTable* relay = reinterpret_cast<RelayTable*>(sys_ld(&ctrl->relay));
  RelayRegs rg = relay_load(relay);
  uint64_t relay_timeout = relay ? relay_ld(&relay->timeout_ticks) : 0;
  bool parked_any = __ballot(rg.suspect) != 0;  // wave-uniform: a relay is parked or a slot is suspect
  RelayQueue rq;
  rq.q = relay_q;
  rq.mask = ring_mask;
  for (;;) {
    // every poll is a PCIe round trip to host memory: the stop flag is read on
    // one poll in 16, not before every ring poll (that made a poll two trips)
    if ((++iters & 15) == 0 && sys_ld(&ctrl->stop) && !__ballot(rg.pend != 0) && rq.tail == rq.head) break;
    if (parked_any) {  // parked relays first: their replies may be waiting, and their slots the queue
      const uint64_t now = realtime_ticks();
      unsigned done = relay_poll(rg, rep, ring_mask, now, state, n_state);
      if (rq.tail != rq.head) done += relay_dispatch(rg, rq, 0, 0, 0, 0, 0, 0, relay_timeout, now, rep, ring_mask);
      processed += done;
      if (done) last_work = realtime_ticks();
      parked_any = __ballot(rg.pend != 0 || rg.suspect) != 0 || rq.tail != rq.head;
    }
    const uint64_t seq = head + lane;
    RingSlot* s = &req[seq & ring_mask];
    // Every poll is PCIe reads of host memory.  With `poll.full` the head slot is
    // read whole in the same trip as its tag and validated by its checksum, so a
    // lone call costs one round trip to be seen, not two.
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&s->msg);
    const bool spec = poll.full && lane == 0;
    uint64_t tag = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0, cs = 0;
    if (lane < poll.lanes) tag = sys_ld(&s->tag);
    if (spec) w0 = sys_ld(w), w1 = sys_ld(w + 1), w2 = sys_ld(w + 2), w3 = sys_ld(w + 3), cs = sys_ld(&s->csum);
    const bool ready = tag == seq + 1 && (!spec || cs == ring_csum(seq, w0, w1, w2, w3));
    const uint64_t m = __ballot(ready);
    unsigned n = (m == ~0ull) ? 64u : (unsigned)__builtin_ctzll(~m);
    if (nxl) {  // GPU peer lanes (the segment's host memory)
      const unsigned nxs = serve_xlanes(xl, xrep, nxl, state, n_state, delay_ticks);
      if (nxs) {
        processed += nxs;
        last_work = realtime_ticks();
        if (n == 0) continue;
      }
    }
    if (n == 0) {
      if ((++idle_polls & 3) == 0) {
        if ((idle_polls & 63) == 0) {
          trace_mask = sys_ld(&ctrl->trace_mask);
          trace = reinterpret_cast<TraceRec*>(sys_ld(&ctrl->trace_ring));
          if (xl) nxl = (uint32_t)min<uint64_t>(sys_ld(&ctrl->xl_n), (uint64_t)nx);
          RelayTable* r2 = reinterpret_cast<RelayTable*>(sys_ld(&ctrl->relay));
          if (r2 != relay && !__ballot(rg.pend != 0) && rq.tail == rq.head) {  // a new table: the old one keeps its slots' words
            relay_store(relay, rg);
            relay = r2;
            rg = relay_load(relay);
            relay_timeout = relay ? relay_ld(&relay->timeout_ticks) : 0;
            parked_any = __ballot(rg.suspect) != 0;
          }
        }
        if (lane == 0 && sys_ld(&ctrl->calib_req)) {  // clock calibration handshake
          sys_st(&ctrl->calib_ticks, realtime_ticks());
          __threadfence_system();
          sys_st(&ctrl->calib_req, 0);
        }
      }
      const uint64_t now = realtime_ticks();
      const bool parked = __ballot(rg.pend != 0) != 0 || rq.tail != rq.head;  // relays in flight: no exit
      const bool idle = idle_ticks && now - last_work > idle_ticks && !parked;
      lifetime_exit = now - t_start > max_ticks;
      if (idle || lifetime_exit) {
        for (uint64_t i = rq.head + lane; i < rq.tail; i += kWave) {  // (lifetime exit) queued relays fail now
          const uint64_t qs = q_ld(rq.q + (i & rq.mask) * 5);
          sys_st16(reinterpret_cast<uint64_t*>(&rep[qs & ring_mask]), 0ull, reply_tag(qs, kStatusNotDelivered));
        }
        rq.head = rq.tail;
        relay_store(relay, rg);  // (a lifetime exit with parked relays: their callers time out)
        int resume = 0;
        if (lane == 0) {
          sys_st(&ctrl->resume_head, head);
          __threadfence_system();
          sys_st(&ctrl->state, kStopped);
          __threadfence_system();
          bool pending = sys_ld(&req[head & ring_mask].tag) == head + 1;
          const uint32_t nxp = xl ? (uint32_t)min<uint64_t>(sys_ld(&ctrl->xl_n), (uint64_t)nx) : 0u;
          for (uint32_t k = 0; k < nxp && !pending; ++k) {
            const uint64_t t = sys_ld(&xl[k].req_tag);
            pending = t != 0 && t == sys_ld(&xl[k].served) + 1;
          }
          if (!lifetime_exit && pending) {
            uint64_t expected = kStopped;
            resume = __hip_atomic_compare_exchange_strong(&ctrl->state, &expected, (uint64_t)kRunning,
                                                          __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_SYSTEM)
                         ? 1
                         : 0;
          }
        }
        resume = __shfl(resume, 0);
        if (resume) {
          last_work = realtime_ticks();
          continue;
        }
        if (lane == 0) {
          __hip_atomic_fetch_add(lifetime_exit ? &ctrl->exits_lifetime : &ctrl->exits_idle, 1ull,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_fetch_add(&ctrl->processed, processed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
      }
      for (uint32_t k = 0; k < poll.sleep; ++k) __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t t_seen = realtime_ticks();
    if (lane < n && !spec) {  // ordered after this lane's tag read (it returned; the branch depends on it)
      w0 = sys_ld(w), w1 = sys_ld(w + 1), w2 = sys_ld(w + 2), w3 = sys_ld(w + 3);
    }
    const bool relayed = lane < n && relay != nullptr &&
                         ((uint16_t)(w0 >> 32) == kMethodRelay || (uint16_t)(w0 >> 32) == kMethodCoordPrime);
    const uint64_t rmask = __ballot(relayed);
    if (rmask) {  // queued for a relay slot (the free ones publish now); the ring moves on
      processed += relay_dispatch(rg, rq, rmask, head, w0, w1, w2, w3, relay_timeout, t_seen, rep, ring_mask);
      parked_any = true;
    }
    if (lane < n && !relayed) {
      MsgRecord msg;
      msg.actor = (uint32_t)w0;
      msg.method = (uint16_t)(w0 >> 32);
      msg.flags = (uint16_t)(w0 >> 48);
      msg.a0 = (int64_t)w1;
      msg.a1 = (int64_t)w2;
      msg.a2 = (int64_t)w3;
      const ReplyRecord r = run_handler(msg, state, n_state, delay_ticks);
      // value + tag in ONE 16-B store (one PCIe write that lands whole): the
      // host that sees the tag sees the value, so no fence and no second write
      ReplySlot* o = &rep[seq & ring_mask];
      sys_st16(reinterpret_cast<uint64_t*>(o), (uint64_t)r.value, reply_tag(seq, (uint32_t)r.status));
      if (trace_mask && trace) {  // after the reply is out: off the request's critical path
        const uint64_t t_done = realtime_ticks();
        TraceRec* tr = &trace[seq & trace_mask];
        sys_st(&tr->seq, seq);
        sys_st(&tr->t_pub_ns, sys_ld(&s->t_pub_ns));
        sys_st(&tr->t_seen_ticks, t_seen);
        sys_st(&tr->t_done_ticks, t_done);
      }
    }
    head += n;
    processed += (uint64_t)__popcll(__ballot(lane < n && !relayed));
    last_work = realtime_ticks();
  }
  relay_store(relay, rg);
  if (lane == 0) {
    sys_st(&ctrl->resume_head, head);
    __threadfence_system();
    sys_st(&ctrl->state, kStopped);
    __hip_atomic_fetch_add(&ctrl->processed, processed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

class DeviceServer {
 public:
  // `shm_name` non-empty: the rings live in a POSIX shared-memory segment of that
  // name (registered with HIP), so other processes on the node can publish calls
  // (shmring.hpp); a launcher thread relaunches the parked wave on their poke.
  DeviceServer(int device, uint32_t ring, uintptr_t state, uint32_t n_state, uint64_t delay_us, double idle_ms,
               double max_s, const std::string& shm_name = "")
      : device_(device), ring_(ring), state_((int64_t*)state), n_state_(n_state) {
    if (ring == 0 || (ring & (ring - 1))) throw std::invalid_argument("ring size must be a power of two");
    pub_actor_.assign(ring_, 0);
    pub_ns_.assign(ring_, 0);
    delay_ticks_ = delay_us * 100;  // s_memrealtime runs at 100 MHz
    idle_ticks_ = (uint64_t)(idle_ms * 1e5);
    max_ticks_ = (uint64_t)(max_s * 1e8);
    PT_HIP_CHECK(hipSetDevice(device_));
    if (shm_name.empty()) {
      const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
      // Request ring in fine-grained DEVICE memory that the host writes through
      // its BAR mapping: the wave's polls and payload reads stay on the GPU
      // instead of crossing PCIe (tools/ring_latency_probe.hip: ping-pong floor
      // 2.14 vs 2.38 us, and a call's payload read is a second round trip).
      // Replies and the control block (host-polled; CAS hand-off) stay in host
      // memory.  A device the CPU cannot map keeps the ring in pinned host memory.
      {
        if (hipExtMallocWithFlags((void**)&req_, sizeof(RingSlot) * ring_, hipDeviceMallocFinegrained) == hipSuccess) {
          if (open_to_cpu(req_)) {
            req_on_device_ = true;
          } else {
            PT_HIP_CHECK(hipFree(req_));
            req_ = nullptr;
          }
        } else {
          if (getenv("PTYPE_DEBUG")) fprintf(stderr, "ptype: fine-grained device ring allocation failed\n");
          (void)hipGetLastError();
          req_ = nullptr;
        }
      }
      if (req_on_device_) {
        PT_HIP_CHECK(hipMemset(req_, 0, sizeof(RingSlot) * ring_));
        PT_HIP_CHECK(hipDeviceSynchronize());
        dreq_ = req_;
      } else {
        PT_HIP_CHECK(hipHostMalloc((void**)&req_, sizeof(RingSlot) * ring_, fl));
        memset((void*)req_, 0, sizeof(RingSlot) * ring_);
        PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dreq_, req_, 0));
      }
      PT_HIP_CHECK(hipHostMalloc((void**)&rep_, sizeof(ReplySlot) * ring_, fl));
      PT_HIP_CHECK(hipHostMalloc((void**)&ctrl_, sizeof(ServerCtrl), fl));
      memset((void*)rep_, 0, sizeof(ReplySlot) * ring_);
      memset((void*)ctrl_, 0, sizeof(ServerCtrl));
      PT_HIP_CHECK(hipHostGetDevicePointer((void**)&drep_, rep_, 0));
      PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dctrl_, ctrl_, 0));
      owner_mem_.reset(new std::atomic<uint64_t>[ring_]);
      owner_ = owner_mem_.get();
      takers_mem_.reset(new RingTaker[kRingTakers]);
      takers_ = takers_mem_.get();
      for (uint32_t i = 0; i < kRingTakers; ++i) {
        takers_[i].token.store(0, std::memory_order_relaxed);
        takers_[i].range.store(0, std::memory_order_relaxed);
        takers_[i].state.store(kTakerIdle, std::memory_order_relaxed);
      }
      seq_ = &local_seq_;
    } else {
      seg_ = ShmSegment::create(shm_name, shm_bytes(ring_));
      const ShmView v = shm_view(seg_->base(), ring_);
      hdr_ = v.hdr;
      req_ = v.req;
      rep_ = v.rep;
      ctrl_ = v.ctrl;
      owner_ = v.owner;
      takers_ = v.takers;  // zero-filled with the new segment
      seq_ = &hdr_->next_seq;
      PT_HIP_CHECK(hipHostRegister(seg_->base(), seg_->size(), hipHostRegisterMapped | hipHostRegisterPortable));
      registered_ = true;
      char* dbase = nullptr;
      PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dbase, seg_->base(), 0));
      const char* hbase = static_cast<const char*>(seg_->base());
      dreq_ = reinterpret_cast<RingSlot*>(dbase + (reinterpret_cast<const char*>(req_) - hbase));
      drep_ = reinterpret_cast<ReplySlot*>(dbase + (reinterpret_cast<const char*>(rep_) - hbase));
      dctrl_ = reinterpret_cast<ServerCtrl*>(dbase + (reinterpret_cast<const char*>(ctrl_) - hbase));
      if (xproc_device_ring_enabled()) export_device_ring();
      export_xlanes();
    }
    for (uint32_t i = 0; i < ring_; ++i) owner_[i].store(i, std::memory_order_relaxed);
    stream_ = dedicated_stream(device_);  // the persistent dispatcher runs here
    PT_HIP_CHECK(hipMalloc((void**)&relay_q_, (size_t)ring_ * 5 * sizeof(uint64_t)));  // relay FIFO (relay_dispatch)
    if (hdr_) {  // publish the segment only once fully initialised
      hdr_->ring = ring_;
      hdr_->owner_pid = (int32_t)getpid();
      __atomic_store_n(&hdr_->magic, kShmMagic, __ATOMIC_RELEASE);
      waker_ = std::thread([this] { waker_loop(); });
    }
  }

  ~DeviceServer() {
    try {
      close();
    } catch (...) {
    }
  }

  bool ring_on_device() const { return req_on_device_; }
  int stream_priority() const {  // the dispatcher stream's priority (dedicated_stream)
    int p = 0;
    return hipStreamGetPriority(stream_, &p) == hipSuccess ? p : -99;
  }  // request ring in device memory (host writes via BAR)

  void close() {
    if (closed_.exchange(true)) return;
    if (hdr_) {
      hdr_->wake.store(2);
      shm_futex_wake(&hdr_->wake);
      if (waker_.joinable()) waker_.join();
    }
    __atomic_store_n(&ctrl_->stop, 1ull, __ATOMIC_SEQ_CST);
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
    (void)hipFree(relay_q_);
    relay_q_ = nullptr;
    xl_ = nullptr;
    if (seg_) {
      handoff_.reset();  // no new client maps the ring (mapped ones keep the buffer alive)
      if (dmabuf_fd_ >= 0) (void)hsa_amd_portable_close_dmabuf(dmabuf_fd_);
      if (req_on_device_) (void)hipFree(req_);
      if (registered_) (void)hipHostUnregister(seg_->base());
      seg_.reset();  // unmaps + unlinks the segment
    } else {
      if (req_on_device_) (void)hipFree(req_);
      else (void)hipHostFree(req_);
      (void)hipHostFree(rep_);
      (void)hipHostFree(ctrl_);
    }
    if (trace_) (void)hipHostFree(trace_);
  }

  // Export a device method to same-node client processes (segment header table).
  void export_method(const std::string& name, uint32_t method, uint32_t actor, const std::vector<std::string>& fields,
                     const std::string& actor_field) {
    if (!hdr_) throw std::runtime_error("export_method: server has no shared-memory segment");
    std::lock_guard<std::mutex> g(launch_mu_);
    const uint32_t n = hdr_->n_methods.load();
    if (n >= (uint32_t)kShmMaxMethods) throw std::runtime_error("export_method: method table full");
    ShmMethod& m = hdr_->methods[n];
    memset(&m, 0, sizeof m);
    strncpy(m.name, name.c_str(), sizeof m.name - 1);
    m.method = method;
    m.actor = actor;
    m.n_fields = (uint32_t)std::min<size_t>(fields.size(), 3);
    for (uint32_t k = 0; k < m.n_fields; ++k) strncpy(m.fields[k], fields[k].c_str(), sizeof m.fields[k] - 1);
    strncpy(m.actor_field, actor_field.c_str(), sizeof m.actor_field - 1);
    hdr_->n_methods.store(n + 1, std::memory_order_release);
  }

  std::string shm_name() const { return seg_ ? seg_->name() : std::string(); }
  bool xlanes_exported() const { return xl_ != nullptr; }
  // kMethodRelay calls of this dispatcher go through `table` (a device RelayTable,
  // xcall.hpp PeerRelay; 0 turns relaying off).  Takes effect at the wave's next
  // launch or idle poll.
  void set_relay(uintptr_t table) { __atomic_store_n(&ctrl_->relay, (uint64_t)table, __ATOMIC_SEQ_CST); }
  uint64_t ring_fds_handed() const { return handoff_ ? handoff_->handed() : 0; }  // client processes that mapped the ring

  // Publish n requests and wait for all replies (any thread).
  void call(const MsgRecord* in, ReplyRecord* out, int n, double timeout_s) {
    if (closed_) throw std::runtime_error("device server closed");
    int done = 0;
    while (done < n) {
      const int batch = std::min<int>({n - done, (int)(ring_ / 2), (int)kRingMaxTake});
      const RingRefs r = refs();
      // one taker entry names the batch's numbers until every reply is read
      RingTicket t = ring_take(r, (uint32_t)batch, timeout_s);
      RingTicketGuard guard{r, t};
      for (int i = 0; i < batch; ++i) publish(r, t.seq + (uint64_t)i, in[done + i], timeout_s);
      ensure_running();
      for (int i = 0; i < batch; ++i) out[done + i] = wait(t.seq + (uint64_t)i, timeout_s);
      done += batch;
    }
  }

  // ---- tracing (device timestamp ring, enqueue -> dispatch -> reply)
  void enable_trace(uint32_t capacity) {
    if (capacity == 0 || (capacity & (capacity - 1))) throw std::invalid_argument("trace capacity: power of two");
    std::lock_guard<std::mutex> g(launch_mu_);
    if (!trace_) {
      const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
      PT_HIP_CHECK(hipHostMalloc((void**)&trace_, sizeof(TraceRec) * capacity, fl));
      memset((void*)trace_, 0, sizeof(TraceRec) * capacity);
      PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dtrace_, trace_, 0));
      trace_cap_ = capacity;
    }
    __atomic_store_n(&ctrl_->trace_ring, (uint64_t)(uintptr_t)dtrace_, __ATOMIC_SEQ_CST);
    __atomic_store_n(&ctrl_->trace_mask, (uint64_t)(trace_cap_ - 1), __ATOMIC_SEQ_CST);
  }
  void disable_trace() { __atomic_store_n(&ctrl_->trace_mask, 0ull, __ATOMIC_SEQ_CST); }
  // Copy of the trace ring (unordered; seq identifies each record).
  std::vector<TraceRec> trace_records() const {
    std::vector<TraceRec> v;
    if (!trace_) return v;
    v.resize(trace_cap_);
    memcpy(v.data(), (const void*)trace_, sizeof(TraceRec) * trace_cap_);
    return v;
  }
  // Host steady-clock ns <-> device ticks: the running dispatcher stamps its
  // clock while the host brackets the handshake.  Returns {host_ns, ticks, err_ns}.
  std::vector<uint64_t> calibrate(double timeout_s = 2.0) {
    ensure_running();
    const uint64_t t0 = now_ns();
    __atomic_store_n(&ctrl_->calib_req, 1ull, __ATOMIC_SEQ_CST);
    while (__atomic_load_n(&ctrl_->calib_req, __ATOMIC_ACQUIRE)) {
      ensure_running();
      if ((now_ns() - t0) * 1e-9 > timeout_s) throw std::runtime_error("device server: calibration timeout");
    }
    const uint64_t t1 = now_ns();
    return {(t0 + t1) / 2, __atomic_load_n(&ctrl_->calib_ticks, __ATOMIC_ACQUIRE), (t1 - t0) / 2};
  }
  // Host-measured round trip of every call, log2(ns) buckets.
  std::vector<uint64_t> rtt_histogram() const {
    std::vector<uint64_t> h(kRttBuckets);
    for (int i = 0; i < kRttBuckets; ++i) h[i] = rtt_hist_[i].load(std::memory_order_relaxed);
    return h;
  }
  static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

  uint64_t processed() const { return __atomic_load_n(&ctrl_->processed, __ATOMIC_ACQUIRE); }
  uint64_t launches() const { return launches_.load(); }
  uint64_t exits_idle() const { return __atomic_load_n(&ctrl_->exits_idle, __ATOMIC_ACQUIRE); }
  uint64_t exits_lifetime() const { return __atomic_load_n(&ctrl_->exits_lifetime, __ATOMIC_ACQUIRE); }
  bool running() const { return __atomic_load_n(&ctrl_->state, __ATOMIC_ACQUIRE) == kRunning; }

  static int submit_c(void* ctx, const MsgRecord* req, ReplyRecord* rep, int n) {
    try {
      static_cast<DeviceServer*>(ctx)->call(req, rep, n, 30.0);
      return 0;
    } catch (...) {
      return -1;
    }
  }

 private:
  RingRefs refs() {
    RingRefs r;
    r.req = req_;
    r.rep = rep_;
    r.owner = owner_;
    r.takers = takers_;
    r.next_seq = seq_;
    r.ring = ring_;
    r.bar = req_on_device_;
    r.poke = [this] { ensure_running(); };
    return r;
  }

  // Claim the next sequence number's slot and publish (ringproto.hpp protocol).
  void publish(const RingRefs& r, uint64_t seq, const MsgRecord& m, double timeout_s) {
    if (!ring_claim(r, seq, timeout_s))
      throw std::runtime_error("device server: request slot not free in time (left for rescue)");
    const uint32_t idx = (uint32_t)(seq & (ring_ - 1));
    const uint64_t t = now_ns();
    pub_actor_[idx] = m.actor;  // host-side copies: the ring may be device memory (slow to read back)
    pub_ns_[idx] = t;
    ring_write(r, seq, m, t);
  }

  ReplyRecord wait(uint64_t seq, double timeout_s) {
    const uint32_t idx = (uint32_t)(seq & (ring_ - 1));
    const uint32_t actor = pub_actor_[idx];
    const uint64_t t_pub = pub_ns_[idx];
    int64_t value = 0;
    uint32_t status = 0;
    // a timed-out call keeps its slot busy until the late reply lands (no reuse
    // while the dispatcher may still read the request)
    if (!ring_wait(refs(), seq, timeout_s, &value, &status)) throw std::runtime_error("device server: reply timeout");
    ReplyRecord r;
    r.value = value;
    r.status = (int32_t)status;
    r.actor = actor;
    const uint64_t rtt = now_ns() - t_pub;
    int b = rtt ? 63 - __builtin_clzll(rtt) : 0;
    rtt_hist_[b < kRttBuckets ? b : kRttBuckets - 1].fetch_add(1, std::memory_order_relaxed);
    return r;
  }

  // Cross-process request ring in device memory (shmring.hpp):
  // fine-grained HBM that this process writes through its BAR mapping, client
  // processes through an mmap of its dma-buf (fd handed over a unix socket).  (No
  // IPC handle: an import of this process's HBM would fault its importer's GPU
  // once this process died.)  Any failure leaves the segment's ring.
  void export_device_ring() {
    const size_t bytes = sizeof(RingSlot) * ring_;
    RingSlot* d = nullptr;
    const auto dbg = [](const char* what, int st) {
      if (getenv("PTYPE_DEBUG")) fprintf(stderr, "ptype: device ring export: %s -> %d\n", what, st);
    };
    if (hipExtMallocWithFlags((void**)&d, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
      (void)hipGetLastError();
      return dbg("hipExtMallocWithFlags", -1);
    }
    int fd = -1;
    uint64_t off = 0;
    hsa_status_t st = HSA_STATUS_ERROR;
    if (!open_to_cpu(d) || (st = hsa_amd_portable_export_dmabuf(d, bytes, &fd, &off)) != HSA_STATUS_SUCCESS) {
      dbg("open_to_cpu / hsa_amd_portable_export_dmabuf", (int)st);
      (void)hipFree(d);
      return;
    }
    static std::atomic<uint32_t> counter{0};
    const std::string sock = "ptype-ring-" + std::to_string(getpid()) + "-" + std::to_string(counter.fetch_add(1));
    try {
      handoff_.reset(new FdHandoff(sock, fd));
    } catch (const std::exception& e) {
      dbg(e.what(), -1);
      (void)hsa_amd_portable_close_dmabuf(fd);
      (void)hipFree(d);
      return;
    }
    PT_HIP_CHECK(hipMemset(d, 0, bytes));
    PT_HIP_CHECK(hipDeviceSynchronize());
    dmabuf_fd_ = fd;
    req_ = d;
    dreq_ = d;
    req_on_device_ = true;
    hdr_->ipc_device = device_;
    hdr_->req_dev_off = off;
    hdr_->req_dev_bytes = bytes;
    memset(hdr_->req_sock, 0, sizeof hdr_->req_sock);
    strncpy(hdr_->req_sock, sock.c_str(), sizeof hdr_->req_sock - 1);
    hdr_->req_dev = 1;  // published with the magic (release) at the end of construction
  }

  // Same-node clients poke the futex when they find the wave parked.  With GPU
  // peer lanes registered the loop also wakes every millisecond: it admits new
  // lane registrations and relaunches a parked wave for a pending lane request
  // (a GPU caller cannot poke a futex).
  void waker_loop() {
    while (!closed_) {
      shm_futex_wait(&hdr_->wake, 0, xl_live_ ? 1000 : 2000);
      const uint32_t w = hdr_->wake.exchange(0);
      if (closed_ || w == 2) break;
      if (xl_) admit_xlanes();
      if (w || (xl_live_ && xlane_pending())) ensure_running();
    }
  }

  // ---- GPU peer lanes (shmring.hpp): the segment's XLane / XReply areas, which
  // this process registered with HIP along with the rest of the segment
  void export_xlanes() {
    const ShmView v = shm_view(seg_->base(), ring_);
    hxl_ = v.xl;
    hxrep_ = v.xrep;
    const char* hbase = static_cast<const char*>(seg_->base());
    char* dbase = nullptr;
    PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dbase, seg_->base(), 0));
    xl_ = reinterpret_cast<XLane*>(dbase + (reinterpret_cast<const char*>(hxl_) - hbase));
    xrep_ = reinterpret_cast<XReply*>(dbase + (reinterpret_cast<const char*>(hxrep_) - hbase));
    hdr_->xl_lanes = kXLanes;
    hdr_->xl_valid = 1;
  }

  // Requested lanes are reset and marked ready; released lanes and lanes of dead
  // callers are reset and freed once quiet (served == req_tag: the wave has
  // answered every request it took -- a reset under a request still running
  // would let its late `served` store confuse the next holder).  A lane with a
  // request in flight is retried at the next waker pass.
  void admit_xlanes() {
    uint32_t live = 0;
    for (int i = 0; i < kXLanes; ++i) {
      XLaneReg& g = hdr_->xregs[i];
      const uint32_t st = g.state.load(std::memory_order_acquire);
      const uint64_t tok = g.token.load(std::memory_order_acquire);
      const bool gone = st == kXLaneFree || st == kXLaneReleasing || !tok || !ring_token_alive(tok);
      if (gone) {
        if (st == kXLaneFree) continue;
        if (!xlane_quiet(i)) {
          ++live;  // keep polling: the wave must finish (and the waker relaunch it for) the request
          continue;
        }
        xlane_reset(i);
        uint64_t t = tok;
        g.token.compare_exchange_strong(t, 0);
        g.state.store(kXLaneFree, std::memory_order_release);
        continue;
      }
      ++live;
      if (st != kXLaneRequested) continue;
      if (!xlane_quiet(i)) continue;  // a previous holder's request is still running
      xlane_reset(i);
      g.state.store(kXLaneReady, std::memory_order_release);
    }
    xl_live_ = live;
    uint64_t top = 0;  // lanes the wave polls: up to the highest registered one
    for (int i = 0; i < kXLanes; ++i) {
      const uint32_t st = hdr_->xregs[i].state.load(std::memory_order_acquire);
      if (st == kXLaneReady || st == kXLaneReleasing || !xlane_quiet(i)) top = (uint64_t)i + 1;
    }
    __atomic_store_n(&ctrl_->xl_n, top, __ATOMIC_SEQ_CST);
  }

  // No request of lane i in flight: the wave answered everything published there.
  bool xlane_quiet(int i) const {
    const uint64_t t = __atomic_load_n(&hxl_[i].req_tag, __ATOMIC_ACQUIRE);
    return t == 0 || __atomic_load_n(&hxl_[i].served, __ATOMIC_ACQUIRE) == t;
  }

  // Reset lane i and its reply slot (host memory): sequence restarts at 0.
  void xlane_reset(int i) {
    __atomic_store_n(&hxl_[i].served, 0ull, __ATOMIC_RELAXED);
    __atomic_store_n(&hxl_[i].req_tag, 0ull, __ATOMIC_RELAXED);
    __atomic_store_n(&hxrep_[i].value, 0ull, __ATOMIC_RELAXED);
    __atomic_store_n(&hxrep_[i].tag, 0ull, __ATOMIC_RELEASE);
  }

  bool xlane_pending() const {
    for (int i = 0; i < kXLanes; ++i) {
      const uint64_t t = __atomic_load_n(&hxl_[i].req_tag, __ATOMIC_ACQUIRE);
      if (t && t == __atomic_load_n(&hxl_[i].served, __ATOMIC_ACQUIRE) + 1) return true;
    }
    return false;
  }

  void ensure_running() {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    for (;;) {
      uint64_t s = __atomic_load_n(&ctrl_->state, __ATOMIC_SEQ_CST);
      if (s == kRunning) return;
      if (s == kStopped) {
        uint64_t exp = kStopped;
        if (__atomic_compare_exchange_n(&ctrl_->state, &exp, (uint64_t)kLaunching, false, __ATOMIC_SEQ_CST,
                                        __ATOMIC_SEQ_CST)) {
          std::lock_guard<std::mutex> g(launch_mu_);
          const uint64_t head = __atomic_load_n(&ctrl_->resume_head, __ATOMIC_ACQUIRE);
          __atomic_store_n(&ctrl_->state, (uint64_t)kRunning, __ATOMIC_SEQ_CST);
          (void)hipSetDevice(device_);
          hipLaunchKernelGGL(persistent_dispatch_kernel, dim3(1), dim3(64), 0, stream_, dreq_, drep_,
                             (uint64_t)(ring_ - 1), dctrl_, head, state_, n_state_, delay_ticks_, idle_ticks_,
                             max_ticks_, poll_, xl_, xrep_, xl_ ? (uint32_t)kXLanes : 0u, relay_q_);
          PT_HIP_CHECK(hipGetLastError());
          launches_.fetch_add(1);
          return;
        }
      }
      std::this_thread::yield();
    }
  }

  int device_;
  uint32_t ring_;
  int64_t* state_;
  uint32_t n_state_;
  uint64_t delay_ticks_ = 0, idle_ticks_ = 0, max_ticks_ = 0;
  PollConfig poll_ = [] {
    PollConfig p;
    const Tune t = tune();
    auto pick = [](int v, uint32_t d) { return v >= 0 ? (uint32_t)v : d; };
    p.lanes = std::min<uint32_t>(64, std::max<uint32_t>(1, pick(t.poll_lanes, p.lanes)));
    p.full = pick(t.poll_full, p.full);
    p.sleep = pick(t.poll_sleep, p.sleep);
    return p;
  }();
  RingSlot* req_ = nullptr;
  bool req_on_device_ = false;     // request ring in fine-grained device memory (host writes via BAR)
  std::vector<uint32_t> pub_actor_;  // per slot: actor / publish time of the call this process published
  std::vector<uint64_t> pub_ns_;
  ReplySlot* rep_ = nullptr;
  ServerCtrl* ctrl_ = nullptr;
  RingSlot* dreq_ = nullptr;
  ReplySlot* drep_ = nullptr;
  ServerCtrl* dctrl_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::atomic<uint64_t> local_seq_{0};
  std::atomic<uint64_t>* seq_ = nullptr;
  std::unique_ptr<std::atomic<uint64_t>[]> owner_mem_;
  std::unique_ptr<RingTaker[]> takers_mem_;
  RingTaker* takers_ = nullptr;
  std::atomic<uint64_t>* owner_ = nullptr;
  std::shared_ptr<ShmSegment> seg_;
  std::unique_ptr<FdHandoff> handoff_;
  int dmabuf_fd_ = -1;
  ShmHeader* hdr_ = nullptr;
  bool registered_ = false;
  std::thread waker_;
  std::atomic<uint64_t> launches_{0};
  std::mutex launch_mu_;
  std::atomic<bool> closed_{false};
  static constexpr int kRttBuckets = 40;
  std::atomic<uint64_t> rtt_hist_[kRttBuckets] = {};
  TraceRec* trace_ = nullptr;
  TraceRec* dtrace_ = nullptr;
  uint32_t trace_cap_ = 0;
  uint64_t* relay_q_ = nullptr;       // relayed requests waiting for a relay slot (device FIFO)
  XLane* xl_ = nullptr;               // GPU peer lanes (the segment's, device address)
  XReply* xrep_ = nullptr;            // their reply slots (device address)
  XLane* hxl_ = nullptr;              // the same two areas, host addresses
  XReply* hxrep_ = nullptr;
  std::atomic<uint32_t> xl_live_{0};  // registered lanes (the waker polls while any)
};

}  // namespace ptype
