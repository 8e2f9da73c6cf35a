// Native epoch engine: the whole chunk-pipelined Send of ActorExchange in one
// host call.
//
// Per chunk: route kernels on the compute stream -> event -> ncclAllToAll of the
// request slots on the engine's comm stream -> event -> dispatch on the compute
// stream -> event -> ncclAllToAll of the reply slots -> event -> completion.
// Chunk k's collectives overlap chunk k+1's route and chunk k-1's dispatch; the
// host only enqueues (~10 us per step instead of ~100 us of Python per chunk,
// which made a multi-GPU step host-bound -- measured with tools/host_overhead.py).
//
// RCCL is called directly on the communicator the control plane's DataPlane
// formed (csrc/core/dataplane.hpp), through its CommCell (dp_link.hpp); the entry
// points are resolved at run time from the librccl torch loaded, so this module
// links no second copy.
// Every rank issues the same collectives in the same order (the pipeline is
// deterministic in the chunk count, which ActorExchange agrees collectively).
#pragma once
#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "mailbox.hpp"
#include "packed.hpp"
#include "tune.hpp"
#include "dp_link.hpp"

namespace ptype {

void launch_route(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                  int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R,
                  int64_t C, int nargs, bool mc, uintptr_t sendbuf, uintptr_t perm, uintptr_t route, uintptr_t hist,
                  uintptr_t lb, uintptr_t stats, int rank_self, const std::vector<uintptr_t>& direct,
                  uint32_t affine_w, uintptr_t stream);
void launch_dispatch(uintptr_t recv, int R, int64_t C, int nargs, bool mc, uintptr_t reply, uintptr_t state,
                     uint32_t n_state, uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank,
                     const std::vector<uintptr_t>& outbox, uint64_t outbox_cap, const std::vector<uintptr_t>& direct,
                     int self, uintptr_t stream);
void launch_local_send(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                       int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                       uint32_t affine_w, uintptr_t state, uint32_t n_state, uint64_t delay_ticks,
                       const std::vector<uintptr_t>& outbox, uint64_t outbox_cap, uintptr_t out_val, uintptr_t out_st,
                       uintptr_t stats, uintptr_t checksum, uintptr_t stream, uintptr_t m_dev = 0);
void launch_outbox_advance(uintptr_t count, uint64_t cap, uintptr_t epoch_m, int64_t j, uintptr_t stream);
void launch_outbox_seal(uintptr_t actor, uint64_t cap, uintptr_t count, uintptr_t stream);
void launch_pack_replies(uintptr_t v2, int R, int64_t C, uintptr_t reply, int vb, uintptr_t stats,
                         int64_t expected_per_rank, uintptr_t stream);
void launch_complete(uintptr_t rep, int64_t C, uintptr_t perm, int64_t M, uintptr_t out_val, uintptr_t out_st,
                     uintptr_t checksum, bool direct, uintptr_t stream, uintptr_t failed = 0);
int64_t wire_req_words(int64_t C, int nargs, bool mc);
int64_t wire_rep_words(int64_t C);
// wire format v3 (packed.hpp / packed.hip)
void launch_packed_meta(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                        int method_uniform, int64_t M, uint32_t n_dir, uint32_t affine_w, uintptr_t meta,
                        uintptr_t stream);
void launch_route_packed(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                         int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                         int R, int64_t C, const PackedLayout& L, uintptr_t sendbuf, uintptr_t perm, uintptr_t route,
                         uintptr_t hist, uintptr_t stats, int rank_self, const std::vector<uintptr_t>& direct,
                         uint32_t affine_w, uintptr_t stream, bool prepped = false);
int64_t route_prep(uintptr_t actor, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R,
                   uintptr_t route, uintptr_t hist, uint32_t affine_w, uintptr_t stream, int64_t* P_out,
                   const MetaCols* mc = nullptr, const CapFold* cf = nullptr);
void launch_dispatch_packed(uintptr_t recv, int R, int64_t C, const PackedLayout& L, uintptr_t reply, uintptr_t state,
                            uint32_t n_state, uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank,
                            const std::vector<uintptr_t>& outbox, uint64_t outbox_cap,
                            const std::vector<uintptr_t>& direct, int self, uintptr_t stream);
void launch_complete_sx(uintptr_t rep, int64_t C, int R, int vb, uintptr_t perm, int64_t M, uintptr_t out_val,
                        uintptr_t out_st, uintptr_t stream, uintptr_t failed, uintptr_t zero, int64_t zero_words);
void launch_complete_packed(uintptr_t rep, int64_t C, int R, int vb, uintptr_t perm, int64_t M, uintptr_t out_val,
                            uintptr_t out_st, uintptr_t checksum, bool direct, uintptr_t stream, uintptr_t failed = 0,
                            uintptr_t zero = 0, int64_t zero_words = 0);

// ---- RCCL entry points (from the library torch loaded)
namespace engine_detail {
typedef int (*AllToAllFn)(const void*, void*, size_t, int, void*, hipStream_t);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef int (*SendFn)(const void*, size_t, int, int, void*, hipStream_t);
typedef int (*RecvFn)(void*, size_t, int, int, void*, hipStream_t);
typedef int (*GroupFn)();
typedef const char* (*ErrStrFn)(int);
constexpr int kNcclInt8 = 0;    // ncclDataType_t ncclInt8
constexpr int kNcclUint64 = 5;  // ncclDataType_t ncclUint64
constexpr int kNcclMax = 2;     // ncclRedOp_t ncclMax

struct Rccl {
  AllToAllFn alltoall = nullptr;
  AllReduceFn allreduce = nullptr;
  SendFn send = nullptr;
  RecvFn recv = nullptr;
  GroupFn group_start = nullptr, group_end = nullptr;
  ErrStrFn errstr = nullptr;
  void bind(void* h) {
    alltoall = (AllToAllFn)dlsym(h, "ncclAllToAll");
    allreduce = (AllReduceFn)dlsym(h, "ncclAllReduce");
    send = (SendFn)dlsym(h, "ncclSend");
    recv = (RecvFn)dlsym(h, "ncclRecv");
    group_start = (GroupFn)dlsym(h, "ncclGroupStart");
    group_end = (GroupFn)dlsym(h, "ncclGroupEnd");
    errstr = (ErrStrFn)dlsym(h, "ncclGetErrorString");
  }
  Rccl() {
    bind(RTLD_DEFAULT);
    if (!alltoall)
      for (const char* lib : {"librccl.so", "librccl.so.1"}) {
        void* h = dlopen(lib, RTLD_NOW | RTLD_NOLOAD);
        if (!h) continue;
        bind(h);
        if (alltoall) break;
      }
  }
  bool p2p() const { return send && recv && group_start && group_end; }
};
inline Rccl& rccl() {
  static Rccl r;
  return r;
}
}  // namespace engine_detail
using engine_detail::rccl;

// One RCCL enqueue on the data plane's CommCell (csrc/core/dp_link.hpp): the
// communicator of the generation in force, or a peer-failure error once the
// DataPlane (or its Send watchdog) retired it -- never a freed communicator.
struct CellUse {
  CommCell* c;
  void* comm;
  explicit CellUse(CommCell* cell) : c(cell), comm(cell ? cell->enter() : nullptr) {
    if (!comm) throw std::runtime_error("ncclRemoteError: the data-plane generation was aborted");
  }
  ~CellUse() { c->leave(); }
  CellUse(const CellUse&) = delete;
  CellUse& operator=(const CellUse&) = delete;
};
using engine_detail::kNcclInt8;
using engine_detail::kNcclMax;
using engine_detail::kNcclUint64;

// In-process stand-in for an R-rank communicator (tests only): R engines of one
// process, each driven by its own host thread and stream on the same GPU, run
// the exact multi-rank pipeline -- slot geometry, per-peer offsets, direct
// completion of the own slot, reply routing -- with the all-to-all done as
// R x R device copies ordered by events.  What RCCL adds on a real node (the
// xGMI transport) is the only part it does not exercise.
//
// Loopback mode (bench/profiling only): ONE driving rank stands for every rank of
// a symmetric R-rank node -- each rank sends the same traffic pattern, so what
// rank q would send this rank is exactly what this rank sends q (recv = send, one
// copy) and the all-reduce is the identity.  The rank runs the full R-rank kernel
// pipeline with an HBM-speed interconnect: the compute side of an R-GPU step.
// link_gbps > 0 also models the interconnect: after each loopback copy, one wave
// holds the comm stream for the time the off-rank bytes (R - 1 peer regions)
// would take at that per-rank egress bandwidth, so chunk-pipelining choices can
// be compared against an xGMI-like all-to-all (compute contention from RCCL's
// own kernels is not modelled).
static __global__ void fake_link_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

// Loopback exact-size all-to-all as ONE launch: region q's first sizes[q] bytes
// (a multiple of 16) from src + q * stride to dst + q * stride.
struct RegionSizes {
  uint32_t n[64];
};
static __global__ __launch_bounds__(256) void fake_copy_regions_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                                size_t stride16, RegionSizes sz) {
  const uint32_t q = blockIdx.y, n16 = sz.n[q] / 16;
  const uint4* s = src + (size_t)q * stride16;
  uint4* d = dst + (size_t)q * stride16;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) d[i] = s[i];
}

// The data plane's collectives when they are not RCCL's: the engines drive a
// HostComm through these calls, one rank's view at a time (`r`).  Two
// implementations: FakeComm (R ranks of ONE process, host threads) and IpcComm
// (ipc_comm.hpp: one rank per PROCESS, shared-memory segments every rank maps, every
// collective stream-ordered on the device).
class HostComm {
 public:
  virtual ~HostComm() = default;
  virtual int size() const = 0;
  // loopback: one driving rank stands for a symmetric node (recv = send, identity all-reduce)
  virtual bool loopback() const { return false; }
  // whether allreduce_max is stream-ordered on the device (no host wait inside it)
  virtual bool device_side() const { return false; }
  // recv_r[q] = send_q[r], `bytes` per peer region
  virtual void alltoall(int r, const void* src, void* dst, size_t bytes, hipStream_t s) = 0;
  // regions `stride` bytes apart; send_bytes[q] of region q go to peer q, which
  // lands recv_bytes[.] in its region r (nullptr: whole regions)
  virtual void alltoallv(int r, const void* src, void* dst, size_t stride, const size_t* send_bytes,
                         const size_t* recv_bytes, hipStream_t s) = 0;
  // element-wise max of n u64 over the ranks, in place
  virtual void allreduce_max(int r, uint64_t* dev, int n, hipStream_t s) = 0;
  // throws when an earlier collective failed (a peer missed it); called at every Send
  virtual void check() const {}
  // device address of a word that is nonzero once a collective of this comm has
  // failed (nullptr: collectives cannot fail softly).  The completion kernels read
  // it in stream order: the replies of a failed op answer kStatusNotDelivered
  // instead of whatever the unwritten regions decode to.
  virtual const uint64_t* device_failed() const { return nullptr; }
};

class FakeComm : public HostComm {
 public:
  explicit FakeComm(int R, bool loopback = false, double link_gbps = 0.0)
      : R_(R), loopback_(loopback), link_gbps_(link_gbps), slots_(R) {
    if (R < 1 || R > 64) throw std::invalid_argument("FakeComm: 1 <= R <= 64");
    for (auto& sl : slots_) {
      PT_HIP_CHECK(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
      PT_HIP_CHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
  }
  ~FakeComm() {
    for (auto& sl : slots_) {
      (void)hipEventDestroy(sl.ready);
      (void)hipEventDestroy(sl.done);
    }
  }
  int size() const override { return R_; }
  bool loopback() const override { return loopback_; }

  void alltoall(int r, const void* src, void* dst, size_t bytes, hipStream_t s) override {
    alltoallv(r, src, dst, bytes, nullptr, nullptr, s);
  }
  // Only the first `recv_bytes[q]` of region q move (in-process copies: the
  // receiver's sizes are all it needs).  Loopback: this rank stands for all, recv = send.
  void alltoallv(int r, const void* src, void* dst, size_t stride, const size_t* send_bytes, const size_t* recv_bytes,
                 hipStream_t s) override {
    (void)send_bytes;
    if (loopback_) {
      size_t off_rank = 0;
      if (!recv_bytes) {
        PT_HIP_CHECK(hipMemcpyAsync(dst, src, stride * R_, hipMemcpyDeviceToDevice, s));
        off_rank = stride * (R_ - 1);
      } else {
        RegionSizes sz{};
        size_t biggest = 0;
        for (int q = 0; q < R_; ++q) {
          if (recv_bytes[q] % 16 || stride % 16 || recv_bytes[q] > 0xffffffffu)
            throw std::invalid_argument("FakeComm: regions must be 16-B multiples below 4 GB");
          sz.n[q] = (uint32_t)recv_bytes[q];
          biggest = std::max(biggest, recv_bytes[q]);
          if (q != r) off_rank += recv_bytes[q];
        }
        const unsigned gx = (unsigned)std::min<size_t>(std::max<size_t>((biggest / 16 + 255) / 256, 1), 1024);
        hipLaunchKernelGGL(fake_copy_regions_kernel, dim3(gx, R_), dim3(256), 0, s, (const uint4*)src, (uint4*)dst,
                           stride / 16, sz);
        PT_HIP_CHECK(hipGetLastError());
      }
      if (link_gbps_ > 0) {
        const double secs = (double)off_rank / (link_gbps_ * 1e9);
        const uint64_t ticks = (uint64_t)std::min(secs * 1e8, 1e7);  // at most 100 ms
        hipLaunchKernelGGL(fake_link_kernel, dim3(1), dim3(64), 0, s, ticks);
        PT_HIP_CHECK(hipGetLastError());
      }
      return;
    }
    slots_[r].src = src;
    slots_[r].dst = dst;
    PT_HIP_CHECK(hipEventRecord(slots_[r].ready, s));
    barrier();
    for (int q = 0; q < R_; ++q) {
      PT_HIP_CHECK(hipStreamWaitEvent(s, slots_[q].ready, 0));
      const size_t n = recv_bytes ? recv_bytes[q] : stride;
      if (n)
        PT_HIP_CHECK(hipMemcpyAsync((char*)dst + (size_t)q * stride, (const char*)slots_[q].src + (size_t)r * stride, n,
                                    hipMemcpyDeviceToDevice, s));
    }
    PT_HIP_CHECK(hipEventRecord(slots_[r].done, s));
    barrier();
    for (int q = 0; q < R_; ++q) PT_HIP_CHECK(hipStreamWaitEvent(s, slots_[q].done, 0));  // senders' buffers read
    barrier();
  }

  // element-wise max of n u64 on every rank (host-synchronous, like the engine's use)
  void allreduce_max(int r, uint64_t* dev, int n, hipStream_t s) override {
    if (loopback_) return;  // every rank holds the same maxima
    slots_[r].host.assign(n, 0);
    PT_HIP_CHECK(hipMemcpyAsync(slots_[r].host.data(), dev, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
    barrier();
    std::vector<uint64_t> m(n, 0);
    for (int q = 0; q < R_; ++q)
      for (int k = 0; k < n; ++k) m[k] = std::max(m[k], slots_[q].host[k]);
    barrier();
    PT_HIP_CHECK(hipMemcpyAsync(dev, m.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    PT_HIP_CHECK(hipStreamSynchronize(s));
  }

 private:
  void barrier() {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t gen = gen_;
    if (++arrived_ == R_) {
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    if (!cv_.wait_for(lk, std::chrono::seconds(60), [&] { return gen_ != gen; }))
      throw std::runtime_error("FakeComm: a rank did not reach the collective within 60 s");
  }
  struct Slot {
    const void* src = nullptr;
    void* dst = nullptr;
    hipEvent_t ready{}, done{};
    std::vector<uint64_t> host;
  };
  int R_;
  bool loopback_;
  double link_gbps_;
  std::vector<Slot> slots_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  uint64_t gen_ = 0;
};

struct EngineBufs {
  uintptr_t send, recv, reply, back, perm, src, route, hist, lb, ws;
};

struct EngineSend {  // one Send: the batch, the registry, the outputs
  uintptr_t actor, a0, a1, a2, method_col;
  int method_uniform;
  int64_t M;
  uintptr_t table;
  uint64_t cap;
  uintptr_t dir;
  uint32_t n_dir, affine_w;
  int nargs;
  bool mc;
  uintptr_t out_val, out_st, state;
  uint32_t n_state;
  uint64_t delay_ticks;
  std::vector<uintptr_t> outbox;
  uint64_t outbox_cap;
  bool direct;
  uintptr_t checksum;
  uintptr_t stream;  // the caller's compute stream
  bool packed;       // wire format v3 for this Send (needs collectives; not under graph capture)
  uintptr_t mailboxes = 0;  // Mailboxes*: deliver on receipt through the HBM mailboxes (no direct)
  bool ordered = false;     // the batch may carry ordered methods (actor-sharded rings, ordered drain)
  uintptr_t m_dev = 0;      // u64 on the device: the batch's real length (<= M), read by the kernel (local path)
};

class EpochEngine {
 public:
  // `C`: per-peer slot capacity the buffers were allocated for.  `adaptive`: with
  // wire v3, each Send's slots are sized by the busiest bucket of the node,
  // agreed in the same all-reduce as the layout (never above `C`).
  // `c_fixed` (0: C): the capacity of Sends that do not adapt (wire v2).
  EpochEngine(int device, uintptr_t comm, int R, int rank, int64_t C, int64_t max_chunk, int chunks,
              std::shared_ptr<HostComm> fake = nullptr, bool adaptive = false, int64_t c_fixed = 0)
      : device_(device), cell_(reinterpret_cast<CommCell*>(comm)), fake_(std::move(fake)), R_(R), rank_(rank), C_(C), C_alloc_(C),
        C_fixed_(c_fixed > 0 && c_fixed <= C ? c_fixed : C), max_chunk_(max_chunk), chunks_(chunks),
        adaptive_(adaptive) {
    if (R < 1 || chunks < 1 || max_chunk < 1) throw std::invalid_argument("EpochEngine: bad geometry");
    if (fake_ && (cell_ || fake_->size() != R || rank < 0 || rank >= R))
      throw std::invalid_argument("EpochEngine: fake communicator must match R and replace comm");
    if (cell_ && !rccl().alltoall) throw std::runtime_error("EpochEngine: ncclAllToAll not found in the process");
    PT_HIP_CHECK(hipSetDevice(device_));
    int lo = 0, hi = 0;
    PT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    PT_HIP_CHECK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));  // comm first
    // Hand-off events keep the default system-scope release: RCCL may move a buffer
    // with peer reads / writes over xGMI, which must see (and not be hidden by) this
    // GPU's L2 contents.
    const unsigned ev_flags = hipEventDisableTiming;
    for (int i = 0; i < kMaxBufs; ++i)
      for (hipEvent_t* e : {&ev_route_[i], &ev_req_[i], &ev_disp_[i], &ev_rep_[i]})
        PT_HIP_CHECK(hipEventCreateWithFlags(e, ev_flags));
    PT_HIP_CHECK(hipEventCreateWithFlags(&ev_meta_out_, hipEventDisableTiming));
    // Cross-stream hand-offs use events unless tune stream_sync=1 (see handoff()).
    int wv = 0;
    if (tune().stream_sync == 1 &&
        hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, device_) == hipSuccess && wv) {
      if (getenv("PTYPE_HANG_DIAG")) {
        // diagnosis: the words in pinned host memory, readable while a queue is stuck
        PT_HIP_CHECK(hipHostMalloc((void**)&flags_host_, sizeof(flag_seq_), hipHostMallocMapped));
        memset((void*)flags_host_, 0, sizeof(flag_seq_));
        PT_HIP_CHECK(hipHostGetDevicePointer((void**)&flags_dev_, flags_host_, 0));
      } else {
        PT_HIP_CHECK(hipMalloc(&flags_dev_, sizeof(flag_seq_)));
        PT_HIP_CHECK(hipMemset(flags_dev_, 0, sizeof(flag_seq_)));
      }
      use_values_ = true;
    }
    // the agreement vector: the v3 column maxima, then (exact-size exchange) the
    // node's count matrix [src rank][dst rank][chunk] -- one all-reduce(MAX) carries
    // both, since every rank fills only its own row
    agree_words_ = kMetaWords + (int64_t)R * R * chunks;
    PT_HIP_CHECK(hipMalloc(&meta_dev_, agree_words_ * sizeof(uint64_t)));
    PT_HIP_CHECK(hipMalloc(&capfold_dev_, kCapFoldWords * sizeof(unsigned)));  // column totals + ticket, self-resetting
    PT_HIP_CHECK(hipMemset(capfold_dev_, 0, kCapFoldWords * sizeof(unsigned)));

    PT_HIP_CHECK(hipHostMalloc(&meta_host_, agree_words_ * sizeof(uint64_t), hipHostMallocDefault));
  }
  ~EpochEngine() {  // no synchronisation: a collective stuck on a dead peer must not hang the owner
    (void)hipSetDevice(device_);
    for (int i = 0; i < kMaxBufs; ++i)
      for (hipEvent_t e : {ev_route_[i], ev_req_[i], ev_disp_[i], ev_rep_[i]}) (void)hipEventDestroy(e);
    (void)hipEventDestroy(ev_meta_out_);
    (void)hipStreamDestroy(comm_stream_);
    (void)hipFree(meta_dev_);
    (void)hipFree(capfold_dev_);
    if (mb_stage_) (void)hipFree(mb_stage_);

    (void)hipHostFree(meta_host_);
    if (flags_host_) (void)hipHostFree(flags_host_);
    else if (flags_dev_) (void)hipFree(flags_dev_);
  }

  // Wire format of the last Send: v3 layout (S == 0: v2) and the words this rank
  // put on each request / reply all-to-all per chunk (all peers, padded slots).
  struct WireInfo {
    PackedLayout layout{};
    int64_t req_words = 0, rep_words = 0;
    int64_t C = 0;        // per-peer slot capacity this Send used
    int64_t C_alloc = 0;  // what the buffers hold
    bool adapted = false; // C was sized from the agreed busiest bucket (meta[kMetaCap])
    bool exact = false;   // regions moved at their used size (counts all-to-all + grouped send / recv)
    uint64_t meta[kMetaWords] = {};
  };
  const WireInfo& last_wire() const { return wire_; }
  bool stream_values() const { return use_values_; }  // hand-offs via stream wait-value packets
  // Hang diagnosis (PTYPE_HANG_DIAG with tune stream_sync=1): for every
  // (hand-off, buffer set) word its last signalled sequence and, when the words
  // live in pinned host memory, the value the GPU has written so far; plus
  // whether the compute / comm streams have drained (hipStreamQuery).
  std::vector<int64_t> hang_state(uintptr_t compute_stream) const {
    std::vector<int64_t> v;
    for (int k = 0; k < 4 * kMaxBufs; ++k) {
      v.push_back((int64_t)flag_seq_[k]);
      v.push_back(flags_host_ ? (int64_t)__atomic_load_n(&flags_host_[k], __ATOMIC_SEQ_CST) : -1);
    }
    v.push_back(hipStreamQuery(as_stream(compute_stream)) == hipSuccess ? 1 : 0);
    v.push_back(hipStreamQuery(comm_stream_) == hipSuccess ? 1 : 0);
    v.push_back(hipEventQuery(ev_meta_out_) == hipSuccess ? 1 : 0);
    for (int i = 0; i < kMaxBufs; ++i)  // 1: the chunk's route kernels completed, 0: not yet, -1: not marked
      v.push_back(diag_ev_[i] ? (hipEventQuery(diag_ev_[i]) == hipSuccess ? 1 : 0) : -1);
    return v;
  }
  void diag_mark(int i, hipStream_t s) {
    if (i >= kMaxBufs) return;
    if (!diag_ev_[i]) PT_HIP_CHECK(hipEventCreateWithFlags(&diag_ev_[i], hipEventDisableTiming));
    PT_HIP_CHECK(hipEventRecord(diag_ev_[i], s));
  }

  void set_bufs(int i, const EngineBufs& b) {
    if (i < 0 || i >= kMaxBufs) throw std::invalid_argument("EpochEngine: at most 8 buffer sets");
    bufs_[i] = b;
    nbufs_ = std::max(nbufs_, i + 1);
  }

  // host-side cost split of the enqueues (ns): kernels, collectives, stream/event ops
  struct HostProfile {
    uint64_t sends = 0, kernels_ns = 0, a2a_ns = 0, sync_ns = 0, total_ns = 0, meta_ns = 0;
  };
  HostProfile host_profile() const { return prof_; }
  void reset_host_profile() { prof_ = HostProfile(); }

  void send(const EngineSend& a) {
    if (fake_) fake_->check();  // an earlier collective's failure surfaces here (IpcComm: a peer missed one)
    const uint64_t t0 = now();
    send_impl(a);
    prof_.total_ns += now() - t0;
    ++prof_.sends;
  }

 private:
  static uint64_t now() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  struct Timed {  // adds the scope's duration to one profile bucket
    uint64_t& acc;
    uint64_t t0;
    explicit Timed(uint64_t& a) : acc(a), t0(now()) {}
    ~Timed() { acc += now() - t0; }
  };

  void send_impl(const EngineSend& in) {
    EngineSend a = in;
    const bool local = local_ && R_ == 1 && !collectives() && a.direct;
    if (a.packed || local) {  // exactly the columns the format names (as v2's scatter reads them)
      if (a.nargs < 2) a.a1 = 0;
      if (a.nargs < 3) a.a2 = 0;
    }
    if (local) {  // one destination: nothing to bucket or move
      if (a.M > max_chunk_ * chunks_) throw std::invalid_argument("EpochEngine: batch exceeds max_batch");
      Timed t(prof_.kernels_ns);
      wire_ = WireInfo();
      launch_local_send(a.actor, a.a0, a.a1, a.a2, a.method_col, a.method_uniform, a.M, a.table, a.cap, a.dir,
                        a.n_dir, a.affine_w, a.state, a.n_state, a.delay_ticks, a.outbox, a.outbox_cap, a.out_val,
                        a.out_st, bufs_[0].ws, a.checksum, a.stream, a.m_dev);
      return;
    }
    if (a.m_dev) throw std::invalid_argument("EpochEngine: a device-counted batch needs the single-rank local path");
    if (a.M > max_chunk_ * chunks_) throw std::invalid_argument("EpochEngine: batch exceeds max_batch");
    if (nbufs_ < 1) throw std::runtime_error("EpochEngine: buffers not set");
    const hipStream_t cs = as_stream(a.stream);
    packed_ = a.packed && collectives();  // v3 only where bytes cross a collective
    C_ = packed_ && adaptive_ && nbufs_ >= chunks_ ? C_alloc_ : C_fixed_;
    wire_.adapted = false;
    // exact-size exchange (SURVEY X1 + X2): needs every chunk's counts before the
    // agreement (adaptive mode preps all chunks) and RCCL's p2p calls
    exact_ = packed_ && adaptive_ && nbufs_ >= chunks_ && (fake_ || rccl().p2p());
    if (packed_) agree_layout(a, cs);
    wire_.C = C_;
    wire_.C_alloc = C_alloc_;
    const int64_t wq = packed_ ? packed_req_words(C_, L_.S) : wire_req_words(C_, a.nargs, a.mc);
    const int64_t wr = packed_ ? packed_rep_words(C_, L_.vb) : wire_rep_words(C_);
    if (packed_ && (wq > wire_req_words(C_, a.nargs, a.mc) || wr > wire_rep_words(C_)))
      throw std::logic_error("EpochEngine: packed regions exceed the v2 slot buffers");  // cannot happen (packed.hpp)
    wire_.layout = packed_ ? L_ : PackedLayout{};
    wire_.req_words = R_ * wq;
    wire_.rep_words = R_ * wr;
    wire_.exact = exact_;
    if (exact_) {  // what actually moves: the used prefixes, averaged over the chunks
      int64_t rq = 0, rp = 0;
      for (int i = 0; i < chunks_; ++i)
        for (int q = 0; q < R_; ++q) {
          rq += packed_req_words(std::min<int64_t>(send_count(i, q), C_), L_.S);
          rp += packed_rep_words(std::min<int64_t>(recv_count(i, q), C_), L_.vb);
        }
      wire_.req_words = rq / chunks_;
      wire_.rep_words = rp / chunks_;
    }
    const bool local_only = R_ == 1;
    const int n = chunks_;
    std::deque<int> pending;  // chunks whose replies are in flight
    int fwd = -1;
    for (int i = 0; i < n; ++i) {
      const int bi = i % nbufs_;
      while (!pending.empty() && pending.front() <= i - nbufs_) {  // buffer reuse: replies consumed first
        finish(a, pending.front(), cs, local_only);
        pending.pop_front();
      }
      route(a, i, bi, cs, local_only);
      if (flags_host_) diag_mark(i, cs);  // PTYPE_HANG_DIAG: did this chunk's route kernels finish?
      if (collectives()) {
        handoff(kRouted, bi, cs, comm_stream_);
        if (exact_) {
          for (int q = 0; q < R_; ++q) {
            xs_[q] = (size_t)packed_req_words(std::min<int64_t>(send_count(i, q), C_), L_.S) * 4;
            xr_[q] = (size_t)packed_req_words(std::min<int64_t>(recv_count(i, q), C_), L_.S) * 4;
          }
          a2av(bufs_[bi].send, bufs_[bi].recv, wq);
        } else {
          a2a(bufs_[bi].send, bufs_[bi].recv, wq);
        }
        signal(kReqIn, bi, comm_stream_);
      }
      if (fwd >= 0) {
        serve(a, fwd, cs, wr);
        pending.push_back(fwd);
      }
      fwd = i;
    }
    if (fwd >= 0) {
      serve(a, fwd, cs, wr);
      pending.push_back(fwd);
    }
    for (int j : pending) finish(a, j, cs, local_only);
  }

  // v3: column maxima of this rank's batch -> ncclAllReduce(MAX) over the node
  // -> host.  The one host wait of a packed Send: every rank derives the same
  // layout from the same agreed vector, so slot geometry stays equal-split.
  void agree_layout(const EngineSend& a, hipStream_t cs) {
    if (!fake_ && !rccl().allreduce) throw std::runtime_error("EpochEngine: ncclAllReduce not found in the process");
    const uint64_t t0 = now();
    // A separate width pass, and pass 1 of two chunks runs ahead (the width pass
    // fused into route pass 1 measured 1-3 % slower: profiles/r1_multirank_ab.txt).
    prepped_ = 0;
    // adaptive capacity needs every chunk's histograms before the agreement (a
    // buffer set per chunk keeps them until its scatter)
    const bool adapt = adaptive_ && nbufs_ >= chunks_;
    {
      Timed t(prof_.kernels_ns);
      // (adaptive: every chunk's pass 1 also folds its busiest column into
      // meta[kMetaCap] -- CapFold -- so no separate histogram pass runs)
      if (exact_)  // other ranks' rows of the count matrix must be zero for the MAX
        PT_HIP_CHECK(hipMemsetAsync(meta_dev_ + kMetaWords, 0, (agree_words_ - kMetaWords) * sizeof(uint64_t), cs));
      launch_packed_meta(a.actor, a.a0, a.a1, a.a2, a.method_col, a.method_uniform, a.M, a.n_dir, a.affine_w,
                         (uintptr_t)meta_dev_, (uintptr_t)cs);
      if (adapt) prep_all(a, cs);
    }
    // on the compute stream itself: the previous Send's collectives are complete
    // there already (its completions waited for them), and no cross-stream hop
    // sits on this, the one host wait of the Send
    const int64_t n_agree = exact_ ? agree_words_ : kMetaWords;
    if (fake_ && !fake_->loopback() && !fake_->device_side()) {  // in-process ranks: a host-synchronous MAX
      fake_->allreduce_max(rank_, meta_dev_, (int)n_agree, cs);
      PT_HIP_CHECK(hipMemcpy(meta_host_, meta_dev_, n_agree * sizeof(uint64_t), hipMemcpyDeviceToHost));
      for (int k = 0; k < kMetaWords; ++k) wire_.meta[k] = meta_host_[k];
      L_ = packed_layout(meta_host_);
      if (adapt) adapt_capacity();
      else prep_ahead(a, cs);
      prof_.meta_ns += now() - t0;
      return;
    }
    if (fake_ && !fake_->loopback()) fake_->allreduce_max(rank_, meta_dev_, (int)n_agree, cs);  // device-side (IpcComm)
    int rc = 0;
    if (!fake_) {
      CellUse u(cell_);
      rc = rccl().allreduce(meta_dev_, meta_dev_, n_agree, kNcclUint64, kNcclMax, u.comm, cs);
    }
    if (rc != 0)
      throw std::runtime_error(std::string("ncclAllReduce failed: ") +
                               (rccl().errstr ? rccl().errstr(rc) : std::to_string(rc)));
    PT_HIP_CHECK(hipMemcpyAsync(meta_host_, meta_dev_, n_agree * sizeof(uint64_t), hipMemcpyDeviceToHost, cs));
    PT_HIP_CHECK(hipEventRecord(ev_meta_out_, cs));
    if (!adapt) prep_ahead(a, cs);  // the GPU routes while the host waits for the agreement
    PT_HIP_CHECK(hipEventSynchronize(ev_meta_out_));
    for (int k = 0; k < kMetaWords; ++k) wire_.meta[k] = meta_host_[k];
    L_ = packed_layout(meta_host_);
    if (adapt) adapt_capacity();
    prof_.meta_ns += now() - t0;
  }

  // This Send's slot capacity: the node's busiest bucket, rounded up to 64 (at
  // least 64, at most what the buffers hold -- beyond that the excess overflows
  // into send_all's re-send rounds as before).
  void adapt_capacity() {
    const int64_t need = (int64_t)meta_host_[kMetaCap];
    int64_t c = ((need + 63) / 64) * 64;
    c = std::max<int64_t>(64, std::min<int64_t>(c, C_alloc_));
    C_ = c;
    wire_.adapted = true;
  }

  // Route pass 1 of chunk `chunk` folds its busiest bucket into meta[kMetaCap] and,
  // for the exact-size exchange, writes its per-destination totals into this
  // rank's row of the count matrix (X1: the same all-reduce then tells every rank
  // what each peer sends it -- no count all-to-all, no extra host wait).
  CapFold cap_fold(int chunk) const {
    CapFold f;
    f.tot = capfold_dev_;
    f.ticket = capfold_dev_ + kCapCopies * kMaxCapCols;
    f.meta = (unsigned long long*)meta_dev_;
    if (exact_) {
      f.counts = (unsigned long long*)meta_dev_ + kMetaWords + (size_t)rank_ * R_ * chunks_ + chunk;
      f.count_stride = (uint32_t)chunks_;
    }
    return f;
  }
  int64_t send_count(int chunk, int q) const {
    return (int64_t)meta_host_[kMetaWords + ((size_t)rank_ * R_ + q) * chunks_ + chunk];
  }
  int64_t recv_count(int chunk, int p) const {
    // loopback: this rank stands for every rank of a symmetric node (recv = send)
    if (fake_ && fake_->loopback()) return send_count(chunk, p);
    return (int64_t)meta_host_[kMetaWords + ((size_t)p * R_ + rank_) * chunks_ + chunk];
  }

  // Route pass 1 of every chunk, each folding its busiest bucket into the agreement.
  void prep_all(const EngineSend& a, hipStream_t cs) {
    for (int i = 0; i < chunks_; ++i) {
      const CapFold cf = cap_fold(i);
      const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M);
      int64_t P;
      prep_G_[i] = route_prep(off(a.actor, lo, 4), m_of(a, i), a.table, a.cap, a.dir, a.n_dir, R_, bufs_[i].route,
                              bufs_[i].hist, a.affine_w, (uintptr_t)cs, &P, nullptr, &cf);
    }
    prepped_ = chunks_;
  }

  // Pass 1 of the route (route words + histograms; layout-independent) for the
  // first two chunks, queued behind the agreement so the host's wake-up from the
  // wait (~10-20 us) is hidden behind device work.  Two, not all: every prep run
  // ahead delays the first all-to-all, which starts the comm-bound critical path.
  void prep_ahead(const EngineSend& a, hipStream_t cs) {
    if (nbufs_ < chunks_) return;
    Timed t(prof_.kernels_ns);
    const int n = std::min(chunks_, 2);
    for (int i = 0; i < n; ++i) {
      const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M);
      int64_t P;
      route_prep(off(a.actor, lo, 4), m_of(a, i), a.table, a.cap, a.dir, a.n_dir, R_, bufs_[i].route, bufs_[i].hist,
                 a.affine_w, (uintptr_t)cs, &P);
    }
    prepped_ = n;
  }

  int64_t m_of(const EngineSend& a, int i) const {
    const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M);
    return std::min<int64_t>(a.M, lo + max_chunk_) - lo;
  }
  static uintptr_t off(uintptr_t p, int64_t elems, int64_t size) { return p ? p + (uintptr_t)(elems * size) : 0; }

  std::vector<uintptr_t> direct_view(const EngineSend& a, int i, int bi) const {
    if (!a.direct) return {};
    const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M);
    return {bufs_[bi].src, off(a.out_val, lo, 8), off(a.out_st, lo, 4)};
  }

  void route(const EngineSend& a, int i, int bi, hipStream_t cs, bool local_only) {
    const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M), m = m_of(a, i);
    const bool write_perm = !(a.direct && local_only && !a.checksum);
    const EngineBufs& b = bufs_[bi];
    Timed t(prof_.kernels_ns);
    if (packed_) {
      launch_route_packed(off(a.actor, lo, 4), off(a.a0, lo, 8), off(a.a1, lo, 8), off(a.a2, lo, 8),
                          off(a.method_col, lo, 2), a.method_uniform, m, a.table, a.cap, a.dir, a.n_dir, R_, C_, L_,
                          b.send, write_perm ? b.perm : 0, b.route, b.hist, b.ws, rank_, direct_view(a, i, bi),
                          a.affine_w, (uintptr_t)cs, i < prepped_ && bi == i);
      return;
    }
    launch_route(off(a.actor, lo, 4), off(a.a0, lo, 8), off(a.a1, lo, 8), off(a.a2, lo, 8), off(a.method_col, lo, 2),
                 a.method_uniform, m, a.table, a.cap, a.dir, a.n_dir, R_, C_, a.nargs, a.mc, b.send,
                 write_perm ? b.perm : 0, b.route, b.hist, b.lb, b.ws, rank_, direct_view(a, i, bi), a.affine_w,
                 (uintptr_t)cs);
  }

  void serve(const EngineSend& a, int i, hipStream_t cs, int64_t wr) {
    const int bi = i % nbufs_;
    const EngineBufs& b = bufs_[bi];
    if (collectives()) await(cs, kReqIn, bi);
    const int64_t m = m_of(a, i);
    if (a.mailboxes) {  // K2 on receipt + K3: replies land in the reply regions
      Timed t(prof_.kernels_ns);
      const Mailboxes* mb = reinterpret_cast<const Mailboxes*>(a.mailboxes);
      ReplyView rv;
      rv.slots = (uint32_t*)b.reply;
      rv.rep_words = wr;  // words per source region
      rv.C = (uint32_t)C_;
      rv.n = (uint64_t)R_ * (uint64_t)C_;
      const uintptr_t src = collectives() ? b.recv : b.send;
      if (packed_) {  // v3 records in; the drain answers in v2 geometry into a staging set, packed below
        rv.slots = mb_stage(cs);
        rv.rep_words = wire_rep_words(C_);
        launch_mailbox_enqueue_slots_packed(mb->view(), src, R_, C_, L_, rv, std::max<int64_t>(1, m / R_),
                                            !a.ordered, (uintptr_t)cs);
      } else {
        launch_mailbox_enqueue_slots(mb->view(), src, R_, C_, a.nargs, a.mc, rv, std::max<int64_t>(1, m / R_),
                                     !a.ordered, (uintptr_t)cs);
      }
      OutboxView ob;
      if (a.outbox_cap) {
        ob.actor = (uint32_t*)a.outbox[0];
        ob.a0 = (int64_t*)a.outbox[1];
        ob.a1 = (int64_t*)a.outbox[2];
        ob.a2 = (int64_t*)a.outbox[3];
        ob.method = (uint16_t*)a.outbox[4];
        ob.count = (unsigned long long*)a.outbox[5];
        ob.cap = a.outbox_cap;
      }
      // (no fixed-method drain: other ranks' slots may carry other methods)
      launch_mailbox_drain(mb->view(), a.state, a.n_state, a.delay_ticks, ob, rv, a.ordered, (uintptr_t)cs, 0);
      if (packed_)
        launch_pack_replies((uintptr_t)rv.slots, R_, C_, b.reply, L_.vb, b.ws, std::max<int64_t>(1, m / R_),
                            (uintptr_t)cs);
    } else {
      Timed t(prof_.kernels_ns);
      if (packed_)
        launch_dispatch_packed(b.recv, R_, C_, L_, b.reply, a.state, a.n_state, a.delay_ticks, b.ws,
                               std::max<int64_t>(1, m / R_), a.outbox, a.outbox_cap, direct_view(a, i, bi), rank_,
                               (uintptr_t)cs);
      else
        launch_dispatch(collectives() ? b.recv : b.send, R_, C_, a.nargs, a.mc, b.reply, a.state, a.n_state, a.delay_ticks,
                        b.ws, std::max<int64_t>(1, m / R_), a.outbox, a.outbox_cap, direct_view(a, i, bi), rank_,
                        (uintptr_t)cs);
    }
    if (collectives()) {
      handoff(kServed, bi, cs, comm_stream_);
      if (exact_) {  // replies go back to whoever sent: sizes by the received counts
        for (int q = 0; q < R_; ++q) {
          xs_[q] = (size_t)packed_rep_words(std::min<int64_t>(recv_count(i, q), C_), L_.vb) * 4;
          xr_[q] = (size_t)packed_rep_words(std::min<int64_t>(send_count(i, q), C_), L_.vb) * 4;
        }
        a2av(b.reply, b.back, wr);
      } else {
        a2a(b.reply, b.back, wr);
      }
      signal(kRepIn, bi, comm_stream_);
    }
  }

  void finish(const EngineSend& a, int i, hipStream_t cs, bool local_only) {
    const int bi = i % nbufs_;
    if (collectives()) await(cs, kRepIn, bi);
    if (a.direct && local_only && !a.checksum) return;  // every reply was written by the own-slot dispatch
    Timed t(prof_.kernels_ns);
    const int64_t lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M), m = m_of(a, i);
    const EngineBufs& b = bufs_[bi];
    const uintptr_t failed = fake_ ? (uintptr_t)fake_->device_failed() : 0;
    if (packed_)
      launch_complete_packed(b.back, C_, R_, L_.vb, b.perm, m, off(a.out_val, lo, 8), off(a.out_st, lo, 4), a.checksum,
                             a.direct, (uintptr_t)cs, failed);
    else
      launch_complete(collectives() ? b.back : b.reply, C_, b.perm, m, off(a.out_val, lo, 8), off(a.out_st, lo, 4),
                      a.checksum, a.direct, (uintptr_t)cs, failed);
  }

  void record(hipEvent_t e, hipStream_t s) {
    Timed t(prof_.sync_ns);
    PT_HIP_CHECK(hipEventRecord(e, s));
  }
  void wait(hipStream_t s, hipEvent_t e) {
    Timed t(prof_.sync_ns);
    PT_HIP_CHECK(hipStreamWaitEvent(s, e, 0));
  }
  // Cross-stream hand-offs, 4 per chunk: route -> request all-to-all -> dispatch
  // -> reply all-to-all -> completion.
  //
  // Default: hipEventRecord on the producer stream + hipStreamWaitEvent on the
  // consumer (barrier-AND packets on HSA completion signals).
  //
  // Opt-in (tune stream_sync=1): a monotonic 64-bit sequence word per
  // (hand-off, buffer set) written by the producer stream (hipStreamWriteValue64)
  // and waited on by the consumer stream (hipStreamWaitValue64, a CP wait-value
  // packet).  Measured on gfx950 (tools/event_gap_bench.hip,
  // profiles/r1_event_gap.jsonl) a kernel -> other-stream kernel hop costs +3.6 us
  // this way vs +10.5 us with events, i.e. ~7 us per hop on a ~0.3 ms step.
  //
  // Why events are the default: a rocprofv3 --pmc pass over the RCCL path hung
  // with the wait-value hand-offs and completed with events.  A wait-value packet
  // blocks its hardware queue on a memory word that the runtime and tools know
  // nothing about; anything that serialises or re-orders dispatches across queues
  // (counter collection serialises kernels device-wide, and at N > 1 RCCL's and
  // torch's streams share the process's 4 hardware queues with ours) can hold the
  // producer's write-value packet behind the blocked waiter.  Host enqueue order
  // (every await enqueued after its signal) is NOT enough when two streams map to
  // one hardware queue in a different order than the host issued them, or when a
  // tool's queue interception releases packets one dispatch at a time.  Events
  // carry HSA signals that the runtime and profilers track, so they cannot
  // deadlock that way.  The gain of wait-value packets (~7 us per hop) is not
  // worth a hang at N = 8.
  enum Handoff { kRouted = 0, kReqIn = 1, kServed = 2, kRepIn = 3 };
  hipEvent_t& event_of(Handoff h, int bi) {
    return h == kRouted ? ev_route_[bi] : h == kReqIn ? ev_req_[bi] : h == kServed ? ev_disp_[bi] : ev_rep_[bi];
  }
  bool values_on(hipStream_t s) const {
    if (!use_values_) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone;
  }
  void signal(Handoff h, int bi, hipStream_t producer) {
    const int k = (int)h * kMaxBufs + bi;
    value_mode_[k] = values_on(producer);
    if (!value_mode_[k]) return record(event_of(h, bi), producer);
    Timed t(prof_.sync_ns);
    PT_HIP_CHECK(hipStreamWriteValue64(producer, flags_dev_ + k, ++flag_seq_[k], 0));
  }
  void await(hipStream_t waiter, Handoff h, int bi) {
    const int k = (int)h * kMaxBufs + bi;
    if (!value_mode_[k]) return wait(waiter, event_of(h, bi));
    Timed t(prof_.sync_ns);
    PT_HIP_CHECK(hipStreamWaitValue64(waiter, flags_dev_ + k, flag_seq_[k], hipStreamWaitValueGte, ~0ull));
  }
  void handoff(Handoff h, int bi, hipStream_t producer, hipStream_t waiter) {  // waiter runs after producer's work so far
    signal(h, bi, producer);
    await(waiter, h, bi);
  }

  void a2a(uintptr_t src, uintptr_t dst, int64_t words_per_peer) {
    Timed t(prof_.a2a_ns);
    if (fake_) {
      fake_->alltoall(rank_, (const void*)src, (void*)dst, (size_t)words_per_peer * 4, comm_stream_);
      return;
    }
    CellUse u(cell_);
    const int rc = rccl().alltoall((const void*)src, (void*)dst, (size_t)words_per_peer * 4, kNcclInt8, u.comm,
                                   comm_stream_);
    if (rc != 0)
      throw std::runtime_error(std::string("ncclAllToAll failed: ") +
                               (rccl().errstr ? rccl().errstr(rc) : std::to_string(rc)));
  }

  // X2: the regions' used prefixes (xs_ bytes to each peer, xr_ bytes from each)
  // as grouped ncclSend / ncclRecv; regions stay `stride_words` apart.
  void a2av(uintptr_t src, uintptr_t dst, int64_t stride_words) {
    Timed t(prof_.a2a_ns);
    const size_t stride = (size_t)stride_words * 4;
    if (fake_) {
      fake_->alltoallv(rank_, (const void*)src, (void*)dst, stride, xs_, xr_, comm_stream_);
      return;
    }
    auto check = [](int rc, const char* what) {
      if (rc != 0)
        throw std::runtime_error(std::string(what) + " failed: " +
                                 (rccl().errstr ? rccl().errstr(rc) : std::to_string(rc)));
    };
    CellUse u(cell_);
    check(rccl().group_start(), "ncclGroupStart");
    for (int q = 0; q < R_; ++q) {
      check(rccl().send((const char*)src + (size_t)q * stride, xs_[q], kNcclInt8, q, u.comm, comm_stream_), "ncclSend");
      check(rccl().recv((char*)dst + (size_t)q * stride, xr_[q], kNcclInt8, q, u.comm, comm_stream_), "ncclRecv");
    }
    check(rccl().group_end(), "ncclGroupEnd");
  }

  int device_;
  bool collectives() const { return cell_ != nullptr || fake_ != nullptr; }

  CommCell* cell_;  // the data plane's RCCL communicator (dp_link.hpp), or null
  std::shared_ptr<HostComm> fake_;
  int R_, rank_;
  int64_t C_, C_alloc_, C_fixed_, max_chunk_;
  int chunks_;
  bool adaptive_ = false;
  int64_t prep_G_[8] = {};  // route blocks of each chunk's pass 1 (kMaxBufs)
  static constexpr int kMaxBufs = 8;  // chunks in flight without waiting for buffer reuse
  EngineBufs bufs_[kMaxBufs]{};
  int nbufs_ = 0;
  hipStream_t comm_stream_ = nullptr;
  hipEvent_t ev_route_[kMaxBufs]{}, ev_req_[kMaxBufs]{}, ev_disp_[kMaxBufs]{}, ev_rep_[kMaxBufs]{};
  hipEvent_t ev_meta_out_{};
  bool use_values_ = false;              // hand-offs through stream wait-value packets (see handoff)
  uint64_t* flags_dev_ = nullptr;        // [4 hand-offs][kMaxBufs] sequence words
  uint64_t* flags_host_ = nullptr;       // the same words in pinned host memory (PTYPE_HANG_DIAG)
  hipEvent_t diag_ev_[8] = {};           // PTYPE_HANG_DIAG: after each chunk's route kernels
  uint64_t flag_seq_[4 * kMaxBufs] = {};  // last value written per word
  bool value_mode_[4 * kMaxBufs] = {};    // how the pending hand-off on that word was signalled
  uint64_t* meta_dev_ = nullptr;   // v3 column maxima (device, all-reduced in place)
  uint64_t* meta_host_ = nullptr;  // pinned copy the host derives the layout from
  unsigned* capfold_dev_ = nullptr;  // CapFold words: column totals [kCapCopies][kMaxCapCols] + ticket
  uint32_t* mb_stage_ = nullptr;     // v2-geometry reply staging for mailbox delivery with wire v3 (lazy)

  // One staging set serves every chunk: each chunk's enqueue, drain and pack run
  // in order on the compute stream.
  uint32_t* mb_stage(hipStream_t cs) {
    (void)cs;
    if (!mb_stage_) {
      PT_HIP_CHECK(hipMalloc(&mb_stage_, (size_t)R_ * (size_t)wire_rep_words(C_alloc_) * sizeof(uint32_t)));
    }
    return mb_stage_;
  }
  int64_t agree_words_ = kMetaWords;  // meta + count matrix [R][R][chunks]
  size_t xs_[kMaxCapCols] = {}, xr_[kMaxCapCols] = {};  // bytes to / from each peer for the a2av in flight
  bool exact_ = false;  // this Send
  bool packed_ = false;
  int prepped_ = 0;  // chunks whose route pass 1 ran ahead of the agreement wait (this Send)
  // world 1 without collectives: the fused local Send (batch.hip local_send_kernel);
  // tune local=0 keeps the epoch-slot pipeline there (A/B and tests)
  bool local_ = tune().local != 0;
  PackedLayout L_{};
  WireInfo wire_;
  HostProfile prof_;
};

}  // namespace ptype
