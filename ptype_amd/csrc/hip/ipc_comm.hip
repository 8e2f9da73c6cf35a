// IpcComm (ipc_comm.hpp): process-to-process collectives through shared-memory
// segments every rank maps and registers, stream-ordered on the device.
#include "ipc_comm.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <atomic>

namespace ptype {

namespace {

// Flag words live in host memory mapped into every process: system-scope loads
// and stores (the dispatcher's polling idiom, server.hpp sys_ld / sys_st) -- no
// read-modify-write, which would need PCIe atomics.
__device__ __forceinline__ uint64_t ipc_ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ipc_st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t* word_at(uint64_t base, size_t off) {
  return reinterpret_cast<uint64_t*>(base + off);
}

// `bytes` (a multiple of 4) from s to d by the blocks of one grid row.
__device__ __forceinline__ void row_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint64_t bytes) {
  const uint64_t n16 = bytes / 16, stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* s16 = reinterpret_cast<const uint4*>(s);
  uint4* d16 = reinterpret_cast<uint4*>(d);
  for (uint64_t i = i0; i < n16; i += stride) d16[i] = s16[i];
  for (uint64_t i = n16 * 4 + i0; i < bytes / 4; i += stride)
    reinterpret_cast<uint32_t*>(d)[i] = reinterpret_cast<const uint32_t*>(s)[i];
}

// `bytes` (a multiple of 4) of zeros at d by the blocks of one grid row.
__device__ __forceinline__ void row_zero(uint8_t* __restrict__ d, uint64_t bytes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes / 4; i += stride)
    reinterpret_cast<uint32_t*>(d)[i] = 0u;
}

__device__ __forceinline__ bool rank_failed(const uint64_t* segs, int rank) {
  __shared__ bool f;
  if (threadIdx.x == 0) f = ipc_ld(word_at(segs[rank], kIpcFailedOff)) != 0;
  __syncthreads();
  return f;
}

// Bounded wait of one lane for *w >= want (another process's store, system
// scope); a timeout marks this rank failed (sticky, and the pinned host flag).
// Returns false when this rank's comm is (or just became) failed.
__device__ __forceinline__ bool wait_word(const uint64_t* w, uint64_t want, uint64_t* mine_failed,
                                          uint64_t timeout_ticks, uint64_t* host_failed) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t n = 0;
  while (ipc_ld(w) < want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
      ipc_st(mine_failed, 1);
      __hip_atomic_store(host_failed, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    if ((++n & 63) == 0 && ipc_ld(mine_failed)) return false;  // another wave of this rank gave up already
    __builtin_amdgcn_s_sleep(2);
  }
  return ipc_ld(mine_failed) == 0;
}

// K1: every block of row q waits until peer q's inbox is free for this op
// (consumed >= seq - 1; this rank's own too, so ops issued on two streams stay
// serialised), then copies region q of src into slot `rank` of peer q's inbox;
// the last block of row q publishes posted[rank] = seq in peer q's segment.
__global__ __launch_bounds__(256) void ipc_push_kernel(const uint8_t* __restrict__ src, uint64_t src_stride,
                                                       const IpcSizes* __restrict__ send, const uint64_t* __restrict__ segs,
                                                       int rank, uint64_t cap, uint64_t seq, unsigned* __restrict__ ctr,
                                                       uint64_t timeout_ticks, uint64_t* __restrict__ host_failed) {
  const int q = (int)blockIdx.y;
  uint64_t* mine_failed = word_at(segs[rank], kIpcFailedOff);
  __shared__ bool go;
  if (threadIdx.x == 0)
    go = wait_word(word_at(segs[q], kIpcConsumedOff), seq - 1, mine_failed, timeout_ticks, host_failed);
  __syncthreads();
  if (!go) return;  // this comm is dead: nobody waits for this op any more
  row_copy(src + (uint64_t)q * src_stride, reinterpret_cast<uint8_t*>(segs[q]) + kIpcCtrlBytes + (uint64_t)rank * cap,
           send->n[q]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();  // release this block's stores (the reader is another process)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (atomicAdd(&ctr[q], 1u) == gridDim.x - 1) {  // every block of the row has released its part
      atomicExch(&ctr[q], 0u);
      __threadfence_system();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ipc_st(word_at(segs[q], kIpcPostedOff) + rank, seq);
    }
  }
}

// K2: every block of row q waits for posted[q] >= seq (rank q's data is in this
// rank's inbox), then copies inbox slot q to region q of dst (or, reduce_n > 0,
// one block waits for every rank and takes the element-wise max of the R slots
// into reduce_dst); the last block marks the inbox consumed.
__global__ __launch_bounds__(256) void ipc_out_kernel(uint8_t* __restrict__ dst, uint64_t dst_stride,
                                                      const IpcSizes* __restrict__ recv,
                                                      const uint64_t* __restrict__ segs, int rank, int R, uint64_t cap,
                                                      uint64_t seq, unsigned* __restrict__ ctr,
                                                      uint64_t* __restrict__ reduce_dst, int reduce_n,
                                                      uint64_t timeout_ticks, uint64_t* __restrict__ host_failed,
                                                      uint64_t* __restrict__ slot_done) {
  uint64_t* mine_failed = word_at(segs[rank], kIpcFailedOff);
  const uint64_t* posted = word_at(segs[rank], kIpcPostedOff);
  __shared__ bool go;
  if (reduce_n > 0) {  // one block: lane q waits for rank q
    const int q = (int)threadIdx.x;
    bool ok = true;
    if (q < R) ok = wait_word(posted + q, seq, mine_failed, timeout_ticks, host_failed);
    go = __syncthreads_and(ok) != 0;
  } else {
    if (threadIdx.x == 0) go = wait_word(posted + blockIdx.y, seq, mine_failed, timeout_ticks, host_failed);
    __syncthreads();
  }
  if (!go) {
    // the op never completed: its destination is zeroed rather than left as the
    // buffer's old (or never written) contents -- a zero region header is an
    // empty region to every consumer; the completion kernels read the failure
    // word and answer kStatusNotDelivered; an all-reduce keeps this rank's input
    if (reduce_n == 0) row_zero(dst + (uint64_t)blockIdx.y * dst_stride, recv->n[blockIdx.y]);
    return;
  }
  if (threadIdx.x == 0) {  // acquire: the posted flag was read above
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const uint8_t* inbox = reinterpret_cast<const uint8_t*>(segs[rank]) + kIpcCtrlBytes;
  if (reduce_n > 0) {
    for (int k = (int)threadIdx.x; k < reduce_n; k += (int)blockDim.x) {
      uint64_t m = 0;
      for (int q = 0; q < R; ++q) m = max(m, reinterpret_cast<const uint64_t*>(inbox + (uint64_t)q * cap)[k]);
      reduce_dst[k] = m;
    }
  } else {
    const int q = (int)blockIdx.y;
    row_copy(inbox + (uint64_t)q * cap, dst + (uint64_t)q * dst_stride, recv->n[q]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every inbox load has returned (its data is stored)
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(ctr, 1u) == gridDim.x * gridDim.y - 1) {
    atomicExch(ctr, 0u);
    ipc_st(word_at(segs[rank], kIpcConsumedOff), seq);
    ipc_st(slot_done, seq);  // every block has read this op's sizes: the host may reuse the slot
  }
}

}  // namespace

IpcComm::IpcComm(int device, int R, int rank, size_t cap_bytes, double timeout_s, const std::string& name)
    : device_(device), R_(R), rank_(rank), cap_((cap_bytes + 15) / 16 * 16), timeout_s_(timeout_s) {
  if (R < 1 || R > kIpcMaxRanks || rank < 0 || rank >= R) throw std::invalid_argument("IpcComm: 0 <= rank < R <= 64");
  if (cap_ < 16) throw std::invalid_argument("IpcComm: capacity");
  timeout_ticks_ = (uint64_t)(std::max(0.01, timeout_s) * 1e8);  // s_memrealtime: 100 MHz
  PT_HIP_CHECK(hipSetDevice(device_));
  segs_.assign((size_t)R, nullptr);
  registered_.assign((size_t)R, false);
  segs_[(size_t)rank] = ShmSegment::create(name, kIpcCtrlBytes + (size_t)R * cap_);  // zero-filled
  map_segment(rank);
  PT_HIP_CHECK(hipMalloc((void**)&segs_dev_, kIpcMaxRanks * sizeof(uint64_t)));
  PT_HIP_CHECK(hipMalloc((void**)&ctr_, (kIpcMaxRanks + 1) * sizeof(unsigned)));
  PT_HIP_CHECK(hipHostMalloc((void**)&sizes_host_, kIpcSizeSlots * sizeof(IpcSizeSlot), hipHostMallocMapped));
  memset((void*)sizes_host_, 0, kIpcSizeSlots * sizeof(IpcSizeSlot));
  PT_HIP_CHECK(hipHostGetDevicePointer((void**)&sizes_dev_, sizes_host_, 0));
  PT_HIP_CHECK(hipMemset(ctr_, 0, (kIpcMaxRanks + 1) * sizeof(unsigned)));
  PT_HIP_CHECK(hipHostMalloc((void**)&host_failed_, 64, hipHostMallocMapped));
  *host_failed_ = 0;
  PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dev_failed_, host_failed_, 0));
  PT_HIP_CHECK(hipDeviceSynchronize());
}

IpcComm::~IpcComm() {
  (void)hipSetDevice(device_);
  // the last op on every stream this comm used: its kernels read the segments
  // unregistered below.  Bounded -- a wait on a dead peer ends at the timeout.
  for (auto& se : last_op_) {
    (void)hipEventSynchronize(se.second);
    (void)hipEventDestroy(se.second);
  }
  for (size_t q = 0; q < segs_.size(); ++q)
    if (registered_[q]) (void)hipHostUnregister(segs_[q]->base());
  (void)hipFree(segs_dev_);
  (void)hipFree(ctr_);
  (void)hipHostFree(sizes_host_);
  (void)hipHostFree(host_failed_);
}

void IpcComm::map_segment(int q) {
  PT_HIP_CHECK(hipHostRegister(segs_[(size_t)q]->base(), segs_[(size_t)q]->size(),
                               hipHostRegisterMapped | hipHostRegisterPortable));
  registered_[(size_t)q] = true;
}

void IpcComm::connect(const std::vector<std::string>& names) {
  if ((int)names.size() != R_) throw std::invalid_argument("IpcComm.connect: one segment name per rank");
  if (connected_) throw std::runtime_error("IpcComm.connect: already connected");
  PT_HIP_CHECK(hipSetDevice(device_));
  uint64_t segs[kIpcMaxRanks] = {};
  const size_t want = kIpcCtrlBytes + (size_t)R_ * cap_;
  for (int q = 0; q < R_; ++q) {
    if (q != rank_) {
      segs_[(size_t)q] = ShmSegment::attach(names[(size_t)q]);
      if (!segs_[(size_t)q] || segs_[(size_t)q]->size() < want)
        throw std::runtime_error("IpcComm.connect: no segment " + names[(size_t)q] + " of rank " + std::to_string(q));
      map_segment(q);
    }
    void* d = nullptr;
    PT_HIP_CHECK(hipHostGetDevicePointer(&d, segs_[(size_t)q]->base(), 0));
    segs[q] = (uint64_t)(uintptr_t)d;
  }
  PT_HIP_CHECK(hipMemcpy(segs_dev_, segs, sizeof segs, hipMemcpyHostToDevice));
  connected_ = true;
}

void IpcComm::seal() { segs_[(size_t)rank_]->unlink_now(); }

bool IpcComm::failed() const { return __atomic_load_n(host_failed_, __ATOMIC_ACQUIRE) != 0; }

void IpcComm::abort() {
  auto* mine = reinterpret_cast<uint64_t*>(static_cast<char*>(segs_[(size_t)rank_]->base()) + kIpcFailedOff);
  __atomic_store_n(mine, 1ull, __ATOMIC_RELEASE);
  __atomic_store_n(host_failed_, 1ull, __ATOMIC_RELEASE);
}

void IpcComm::check() const {
  if (failed())
    throw std::runtime_error("IpcComm: peer did not reach a collective within " + std::to_string(timeout_s_) +
                             " s (rank " + std::to_string(rank_) + " of " + std::to_string(R_) + ", op " +
                             std::to_string(seq_) + ")");
}

void IpcComm::op(const void* src, size_t src_stride, void* dst, size_t dst_stride, const IpcSizes& send,
                 const IpcSizes& recv, hipStream_t s, uint64_t* reduce_dst, int reduce_n) {
  if (!connected_) throw std::runtime_error("IpcComm: connect() first");
  uint64_t smax = 0, rmax = 0;
  for (int q = 0; q < R_; ++q) {
    if (send.n[q] > cap_ || recv.n[q] > cap_ || send.n[q] % 4 || recv.n[q] % 4)
      throw std::invalid_argument("IpcComm: a region exceeds the capacity or is not a 4-B multiple");
    smax = std::max(smax, send.n[q]);
    rmax = std::max(rmax, recv.n[q]);
  }
  PT_HIP_CHECK(hipSetDevice(device_));
  const uint64_t seq = ++seq_;
  auto blocks = [](uint64_t bytes) {  // ~16 KB per block, at most 64 per peer
    return (unsigned)std::min<uint64_t>(64, std::max<uint64_t>(1, (bytes + 16383) / 16384));
  };
  // the per-peer sizes go through a small device ring of IpcSizes (kernel
  // arguments of 512 B each made every launch slower); slot reuse is safe once
  // the ring has wrapped, because ops on a comm complete in order
  const int k = (int)(seq % kIpcSizeSlots);
  IpcSizeSlot* hs = sizes_host_ + k;
  const uint64_t prev = seq > (uint64_t)kIpcSizeSlots ? seq - kIpcSizeSlots : 0;
  while (__atomic_load_n(&hs->done, __ATOMIC_ACQUIRE) < prev) {  // (the host is kIpcSizeSlots ops ahead: rare)
    if (failed()) break;  // a failed comm's kernels return early and mark nothing: the slot is free
    std::this_thread::yield();
  }
  hs->send = send;
  hs->recv = recv;
  std::atomic_thread_fence(std::memory_order_release);
  IpcSizeSlot* ds = sizes_dev_ + k;
  hipLaunchKernelGGL(ipc_push_kernel, dim3(blocks(smax), R_), dim3(256), 0, s, (const uint8_t*)src,
                     (uint64_t)src_stride, (const IpcSizes*)&ds->send, segs_dev_, rank_, (uint64_t)cap_, seq, ctr_,
                     timeout_ticks_, dev_failed_);
  hipLaunchKernelGGL(ipc_out_kernel, dim3(reduce_n > 0 ? 1 : blocks(rmax), reduce_n > 0 ? 1 : R_), dim3(256), 0, s,
                     (uint8_t*)dst, (uint64_t)dst_stride, (const IpcSizes*)&ds->recv, segs_dev_, rank_, R_,
                     (uint64_t)cap_, seq, ctr_ + kIpcMaxRanks, reduce_dst, reduce_n, timeout_ticks_, dev_failed_,
                     &ds->done);
  PT_HIP_CHECK(hipGetLastError());
  hipEvent_t* ev = nullptr;
  for (auto& se : last_op_)
    if (se.first == s) ev = &se.second;
  if (!ev) {
    last_op_.emplace_back(s, nullptr);
    ev = &last_op_.back().second;
    PT_HIP_CHECK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  }
  PT_HIP_CHECK(hipEventRecord(*ev, s));
}

void IpcComm::alltoall(int r, const void* src, void* dst, size_t bytes, hipStream_t s) {
  alltoallv(r, src, dst, bytes, nullptr, nullptr, s);
}

void IpcComm::alltoallv(int r, const void* src, void* dst, size_t stride, const size_t* send_bytes,
                        const size_t* recv_bytes, hipStream_t s) {
  if (r != rank_) throw std::invalid_argument("IpcComm: one rank per process");
  IpcSizes sn{}, rn{};
  for (int q = 0; q < R_; ++q) {
    sn.n[q] = send_bytes ? send_bytes[q] : stride;
    rn.n[q] = recv_bytes ? recv_bytes[q] : stride;
  }
  op(src, stride, dst, stride, sn, rn, s, nullptr, 0);
}

void IpcComm::allreduce_max(int r, uint64_t* dev, int n, hipStream_t s) {
  if (r != rank_) throw std::invalid_argument("IpcComm: one rank per process");
  if (n < 1 || (size_t)n * 8 > cap_) throw std::invalid_argument("IpcComm: all-reduce larger than the capacity");
  IpcSizes sn{}, rn{};
  for (int q = 0; q < R_; ++q) sn.n[q] = (uint64_t)n * 8;
  op(dev, 0, nullptr, 0, sn, rn, s, dev, n);
}

// ---------------------------------------------------------------- DataPlane transport (dp_link.hpp)
namespace {
using IpcRef = std::shared_ptr<IpcComm>;
IpcComm& ipc_of(void* h) { return **static_cast<IpcRef*>(h); }
void put_err(char* err, size_t n, const char* m) {
  if (err && n) {
    strncpy(err, m, n - 1);
    err[n - 1] = 0;
  }
}
void* t_open(int device, int world, int rank, uint64_t cap, double timeout_s, const char* name, char* err, size_t n) {
  try {
    return new IpcRef(std::make_shared<IpcComm>(device, world, rank, (size_t)cap, timeout_s, std::string(name)));
  } catch (const std::exception& e) {
    put_err(err, n, e.what());
    return nullptr;
  }
}
int t_connect(void* h, const char* const* names, int count, char* err, size_t n) {
  try {
    ipc_of(h).connect(std::vector<std::string>(names, names + count));
    return 0;
  } catch (const std::exception& e) {
    put_err(err, n, e.what());
    return 1;
  }
}
void t_seal(void* h) {
  try {
    ipc_of(h).seal();
  } catch (const std::exception&) {
  }
}
int t_allreduce(void* h, uint64_t* dev, int cnt, void* stream, char* err, size_t n) {
  try {
    IpcComm& c = ipc_of(h);
    c.check();
    c.allreduce_max(c.rank(), dev, cnt, (hipStream_t)stream);
    return 0;
  } catch (const std::exception& e) {
    put_err(err, n, e.what());
    return 1;
  }
}
int t_alltoallv(void* h, const void* src, void* dst, size_t stride, const size_t* sb, const size_t* rb, void* stream,
                char* err, size_t n) {
  try {
    IpcComm& c = ipc_of(h);
    c.check();
    c.alltoallv(c.rank(), src, dst, stride, sb, rb, (hipStream_t)stream);
    return 0;
  } catch (const std::exception& e) {
    put_err(err, n, e.what());
    return 1;
  }
}
int t_failed(void* h) { return ipc_of(h).failed() ? 1 : 0; }
void t_abort(void* h) { ipc_of(h).abort(); }
uint64_t t_cap(void* h) { return (uint64_t)ipc_of(h).cap(); }
void* t_engine_ref(void* h) { return new std::shared_ptr<HostComm>(*static_cast<IpcRef*>(h)); }
void t_release(void* h) { delete static_cast<IpcRef*>(h); }
}  // namespace

const DpTransportOps* ipc_transport_ops() {
  static const DpTransportOps ops{kDpTransportAbi, t_open,   t_connect, t_seal, t_allreduce, t_alltoallv,
                                  t_failed,        t_abort,  t_cap,     t_engine_ref, t_release};
  return &ops;
}

}  // namespace ptype
