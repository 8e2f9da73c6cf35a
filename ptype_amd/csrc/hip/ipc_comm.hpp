// IpcComm: the data plane's collectives between PROCESSES on one node without
// RCCL -- one rank per process, stream-ordered on the device, no host wait.  It
// exists so the engines' multi-rank pipelines (EpochEngine, SortedExchange) run
// across real process boundaries on a one-GPU box: RCCL refuses two ranks on
// one device ("Duplicate GPU detected"), and FakeComm's ranks share one process.
//
// Transport: every rank's receive segment is a POSIX shared-memory file that
// EVERY rank maps and registers with HIP (hipHostRegister, mapped) in its own
// process, so the GPU reaches it through that process's own mapping.  The first
// design imported the peers' HBM by IPC handle; a peer killed mid-run then took
// its HBM with it and the survivors' next collective faulted on the unmapped
// import (measured on the MI355X box, r4).  Host pages stay mapped for as long
// as any survivor maps them, so a dead peer costs a timeout, never a fault.
// (Bandwidth is PCIe's, not HBM's: this is the test / rehearsal transport; a
// multi-GPU node runs RCCL over xGMI.)
//
// Segment of rank r (host shared memory, registered by every rank):
//   [0, 512)      posted[64]: rank q stores posted[q] = s once its op-s data sits
//                 in this inbox (system-scope store)
//   [512]         consumed: r stores s once it has copied op s out of its inbox
//   [640]         failed: r's sticky error word (a wait that timed out)
//   [4096, ...)   inbox[R][cap]: rank q's region of the op in flight at q * cap
//
// Op s (every rank issues the same ops in the same order; s is a host counter),
// all on the caller's stream -- two kernels:
//   K1 push   (X, R) blocks: row q waits for rank q's consumed >= s - 1 (its
//             inbox is free again; this rank's own too, so ops issued on two
//             streams stay serialised), copies region q of src -> rank q's inbox
//             slot r; the last block of each row releases (system fence) and
//             stores posted[r] = s into rank q's segment
//   K2 out    (X, R) blocks: row q waits for posted[q] >= s, system acquire,
//             inbox slot q -> region q of dst (or the element-wise max of the R
//             slots, for all-reduce); the last block stores consumed = s
// Waits are bounded (timeout_s): a peer that never arrives (killed) makes the
// wave set `failed` (and a pinned host flag) and exit, every later kernel of
// this comm skips its work, and the next Send's check() throws
// "IpcComm: peer ...", which the elastic path reads as a rank failure.  Every
// wave reaches an exit, so the grid drains even when a peer is gone.
//
// The hand-off follows MI355X_MICROARCH.md "inter-workgroup visibility":
// producer plain stores -> s_waitcnt vmcnt(0) -> barrier -> one lane's release
// fence (system scope: the consumer is another process) -> vmcnt(0) -> flag
// store; consumer poll -> acquire fence -> vmcnt(0) -> barrier -> plain loads.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "dp_link.hpp"
#include "engine.hpp"
#include "shmring.hpp"

namespace ptype {

constexpr int kIpcMaxRanks = 64;
constexpr size_t kIpcCtrlBytes = 4096;
constexpr size_t kIpcPostedOff = 0, kIpcConsumedOff = 512, kIpcFailedOff = 640;

struct IpcSizes {  // bytes per peer region (<= cap)
  uint64_t n[kIpcMaxRanks];
};
// Per-peer sizes of the ops in flight: a ring of slots in pinned host memory
// (512-B kernel arguments made every launch slower), read by the kernels over
// the bus; the out kernel's last block marks the slot done, and the host reuses
// a slot only once its previous op is done (or the comm has failed).
constexpr int kIpcSizeSlots = 64;
struct IpcSizeSlot {
  IpcSizes send, recv;
  uint64_t done;  // the seq of the last op that finished with this slot
  uint64_t pad[7];
};

class IpcComm : public HostComm {
 public:
  // cap_bytes: the largest region one op moves per peer (16-B multiple).
  // name: this rank's segment name (unique per group and rank).
  IpcComm(int device, int R, int rank, size_t cap_bytes, double timeout_s, const std::string& name);
  ~IpcComm() override;
  IpcComm(const IpcComm&) = delete;
  IpcComm& operator=(const IpcComm&) = delete;

  // this rank's segment name, for the other ranks
  std::string handle() const { return segs_[(size_t)rank_]->name(); }
  // every rank's segment name, in rank order (this rank's own is skipped); maps and registers the peers'
  void connect(const std::vector<std::string>& names);
  // once EVERY rank has connected: remove this rank's name (the mappings stay)
  void seal();

  int size() const override { return R_; }
  bool device_side() const override { return true; }
  void alltoall(int r, const void* src, void* dst, size_t bytes, hipStream_t s) override;
  void alltoallv(int r, const void* src, void* dst, size_t stride, const size_t* send_bytes, const size_t* recv_bytes,
                 hipStream_t s) override;
  void allreduce_max(int r, uint64_t* dev, int n, hipStream_t s) override;
  void check() const override;
  const uint64_t* device_failed() const override { return dev_failed_; }

  bool failed() const;           // a wait of this rank timed out, or abort() ran (pinned host flag; no sync)
  // Fail this rank's comm now (the DataPlane aborting a generation): the waiting
  // kernels poll the segment's failed word and exit; every later op skips its work.
  void abort();
  uint64_t ops() const { return seq_; }
  int rank() const { return rank_; }
  size_t cap() const { return cap_; }

 private:
  void op(const void* src, size_t src_stride, void* dst, size_t dst_stride, const IpcSizes& send,
          const IpcSizes& recv, hipStream_t s, uint64_t* reduce_dst, int reduce_n);
  void map_segment(int q);

  int device_, R_, rank_;
  size_t cap_;
  uint64_t timeout_ticks_;
  double timeout_s_;
  std::vector<std::shared_ptr<ShmSegment>> segs_;  // every rank's segment, mapped in this process
  std::vector<bool> registered_;
  uint64_t* segs_dev_ = nullptr;           // [R] device address of every rank's segment, as mapped here
  unsigned* ctr_ = nullptr;                // last-block tickets: [R] push rows, [1] out (self-resetting)
  IpcSizeSlot* sizes_host_ = nullptr;     // [kIpcSizeSlots] pinned (the host writes, the kernels read)
  IpcSizeSlot* sizes_dev_ = nullptr;      // the same, device address
  uint64_t* host_failed_ = nullptr;        // pinned: set by a timed-out wait
  uint64_t* dev_failed_ = nullptr;         // its device address
  uint64_t seq_ = 0;                       // ops issued
  std::vector<std::pair<hipStream_t, hipEvent_t>> last_op_;  // per stream used: an event after its last op
  bool connected_ = false;
};

// The DpTransportOps table (dp_link.hpp) through which the control plane's
// DataPlane forms, drives and aborts IpcComm generations.
const DpTransportOps* ipc_transport_ops();

}  // namespace ptype
