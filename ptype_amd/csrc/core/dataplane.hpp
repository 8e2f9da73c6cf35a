// The data plane's RCCL communicator lifecycle, compiled (VERDICT r4 Missing #3;
// SURVEY 3.1 step 5 and 5.3).
//
// The reference's Join is one compiled call that brings a member up, registers
// it and returns (cluster/cluster.go:28-84, :161-196); a dead member is noticed
// through its lapsed lease (cluster/registry.go:51-86) and the survivors carry
// on.  The GPU data plane of a service is an RCCL communicator over the
// service's nodes, and its whole life runs here, in the control-plane module:
//
//   form(gen, members)   rank 0 (members[0]) draws an ncclUniqueId and publishes
//                        it with the member list under
//                        store/_ptype/nccl/<service>/<gen>/uid; every member
//                        reads it from the replicated store and runs
//                        ncclCommInitRank on its device (no TCPStore, no torch
//                        process group);
//   async_error()        ncclCommGetAsyncError: a peer that died mid-collective;
//   abort()              ncclCommAbort: nothing of this generation blocks again;
//   settle(members)      the registry's live nodes (2 s leases): the members
//                        minus those whose lease lapsed (waited on for at most
//                        grace_s) -- the next generation's proposal;
//   recover()            abort + settle + form(gen + 1): the elastic step.
//
// RCCL and HIP are resolved at run time from the libraries the process already
// loaded (the device runtime's torch / HIP), so this host-only module links
// neither; without them every call throws.  Host-level agreements of the data
// plane (a few words, all-reduce MAX) and point-to-point state moves (buddy
// replicas) go through the same communicator.
#pragma once
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "api.hpp"

namespace ptype {

class DataPlane {
 public:
  // device: this member's HIP ordinal (-1: set_device before form); timeout_s bounds the rendezvous and waits
  DataPlane(std::shared_ptr<EtcdRegistry> registry, std::shared_ptr<KvClient> kv, std::string service, std::string me,
            int device, double timeout_s);
  ~DataPlane();
  DataPlane(const DataPlane&) = delete;
  DataPlane& operator=(const DataPlane&) = delete;

  // Generation `gen` over `proposal` (node ids "address:port"): rendezvous -- the
  // first published record still current wins, so differing views converge -- and
  // ncclCommInitRank.  Returns this member's rank; throws "excluded" if left out.
  int form(uint64_t gen, const std::vector<std::string>& proposal);
  void set_device(int device);  // before the first form() (no communicator yet)
  int device() const { return device_; }
  // The service's registered nodes with a live lease (sorted "address:port").
  std::vector<std::string> alive_nodes();
  // Wait until `world` nodes are registered; the first `world` of them (sorted).
  std::vector<std::string> wait_nodes(int world);
  // The next proposal: `current` minus the nodes whose lease lapsed, waiting at
  // most grace_s for one to lapse (survivors keep their order).
  std::vector<std::string> settle(const std::vector<std::string>& current, double grace_s);
  // abort + settle + form(gen + 1); returns the new member list
  std::vector<std::string> recover(double grace_s);

  int async_error() const;  // ncclResult_t of the communicator (0: fine)
  void abort();             // ncclCommAbort (idempotent)
  bool aborted() const { return comm_.load() == nullptr; }

  // element-wise MAX of `v` over the members (host values; a device round trip)
  std::vector<uint64_t> allreduce_max(const std::vector<uint64_t>& v);
  // the same on n device words in place, enqueued on `stream` (no host wait)
  void allreduce_max_dev(uintptr_t dev, size_t n, uintptr_t stream);
  // grouped send of `sbytes` at device address `send` to rank `dst` and receive of
  // `rbytes` into `recv` from rank `src` (dst / src < 0: that half skipped); synchronous.
  // Host waits are bounded by timeout_s: a peer that never answers aborts the
  // communicator and raises "ncclRemoteError" (a rank failure).
  void sendrecv(uintptr_t send, size_t sbytes, int dst, uintptr_t recv, size_t rbytes, int src);
  void barrier();

  uintptr_t comm() const { return (uintptr_t)comm_.load(); }
  int rank() const { return rank_; }
  int size() const { return (int)members_.size(); }
  uint64_t gen() const { return gen_; }
  const std::vector<std::string>& members() const { return members_; }
  const std::string& me() const { return me_; }
  static bool available();  // RCCL and HIP entry points found in this process

 private:
  void destroy_comm();
  void* live_comm() const;     // the communicator, or a peer-failure error once aborted
  void wait_stream(void* comm);  // bounded by timeout_s; a dead peer aborts and raises
  std::shared_ptr<EtcdRegistry> reg_;
  std::shared_ptr<KvClient> kv_;
  std::string service_, me_;
  int device_;
  double timeout_s_;
  std::atomic<void*> comm_{nullptr};  // ncclComm_t (a watchdog thread may abort it)
  void* stream_ = nullptr;  // hipStream_t of this object's collectives
  void* scratch_ = nullptr; // device words for allreduce_max
  size_t scratch_words_ = 0;
  int rank_ = -1;
  uint64_t gen_ = 0;
  std::vector<std::string> members_;
};

}  // namespace ptype
