// K4 on the net/rpc serving path: batched gob requests decoded
// on the GPU straight into HBM mailbox columns.
//
// A Go-protocol client pipelines calls on one connection; the net/rpc server
// (csrc/core/netrpc.cpp, RpcServer::register_device_batch) keeps each request's
// header on the host but captures the argument VALUE messages raw, and when the
// connection's input runs dry hands the buffered batch here:
//
//   bytes, offsets --H2D--> gob_decode_kernel (one message per lane: int64
//   columns in wire-field order + a status per message) --> actor column -->
//   Mailboxes::send_sorted (count / scatter into the shard rings, drain) -->
//   replies --D2H--> the server, which encodes every Response with the same
//   host encoder as the single-call path (identical bytes on the wire).
//
// Reference: the reference's server runs net/rpc's gob codec per call in a
// goroutine (example/calculator/server/server.go:16-20, cluster/rpc.go:65,88);
// here a connection's pipelined calls cost one GPU decode pass and one mailbox Send.
#pragma once
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.hpp"
#include "mailbox.hpp"

namespace ptype {

void launch_gob_decode(uintptr_t buf, uintptr_t offsets, int64_t M, uint32_t type_id, const std::vector<uintptr_t>& cols,
                       uintptr_t status, uintptr_t stream);

// actor[i] = the actor field's column (or the fixed actor); a message that failed
// to decode (gob status != 0) gets no actor (0xffffffff): it is answered
// no-actor by the enqueue and never runs a handler -- the client is told
// "decoding error", so a stateful method must not have changed state for it
__global__ __launch_bounds__(256) void gob_bridge_actor_kernel(const int64_t* __restrict__ col, uint32_t fixed,
                                                               const int32_t* __restrict__ gst, int64_t n,
                                                               uint32_t* __restrict__ actor) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    actor[i] = gst[i] != 0 ? 0xffffffffu : col ? (uint32_t)col[i] : fixed;
}

class GobBridge {
 public:
  static constexpr int kMaxFields = 8;  // gob.hip kGobMaxFields

  // mb: this process's HBM mailboxes; table: the registry mirror used for ids
  // past the directory (mailbox index = actor id below n_state: computed routes)
  // order_stream: the runtime's stream (0: the null stream).  Each batch starts
  // after the work queued there and that stream's later work waits for the
  // batch, so a bridge batch and the runtime's Sends never update actor state
  // concurrently.
  GobBridge(int device, Mailboxes* mb, uint32_t method, uint32_t fixed_actor, uintptr_t table, uint64_t cap,
            uintptr_t state, uint32_t n_state, uint64_t delay_ticks, uintptr_t order_stream = 0)
      : device_(device), mb_(mb), method_(method), fixed_actor_(fixed_actor), table_(table), cap_(cap),
        state_(state), n_state_(n_state), delay_ticks_(delay_ticks), order_(as_stream(order_stream)) {
    if (!mb_) throw std::invalid_argument("GobBridge: mailboxes required");
    PT_HIP_CHECK(hipSetDevice(device_));
    PT_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    PT_HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    PT_HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  }
  // After a data-plane recovery re-homed the actors (runtime._rehome): the new
  // registry mirror and state tensor, taken at the next batch.  The handle the
  // net/rpc server holds stays valid.
  void retarget(uintptr_t table, uint64_t cap, uintptr_t state, uint32_t n_state) {
    std::lock_guard<std::mutex> g(mu_);
    if (stream_) PT_HIP_CHECK(hipStreamSynchronize(stream_));
    table_ = table, cap_ = cap, state_ = state, n_state_ = n_state;
  }
  ~GobBridge() {
    (void)hipSetDevice(device_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    release();
    (void)hipEventDestroy(ev_in_);
    (void)hipEventDestroy(ev_out_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  GobBridge(const GobBridge&) = delete;
  GobBridge& operator=(const GobBridge&) = delete;

  // DeviceBatchFn (netrpc.hpp)
  static int batch_c(void* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n, int64_t type_id, int nf,
                     const int32_t* field_col, int32_t* gob_status, ReplyRecord* out) {
    try {
      static_cast<GobBridge*>(ctx)->run(bytes, offsets, n, type_id, nf, field_col, gob_status, out);
      return 0;
    } catch (const std::exception& e) {
      if (getenv("PTYPE_DEBUG")) fprintf(stderr, "ptype: gob bridge: %s\n", e.what());
      return -1;
    }
  }

  uint64_t batches() const { return batches_; }
  uint64_t calls() const { return calls_; }

 private:
  void run(const uint8_t* bytes, const int64_t* offsets, int64_t n, int64_t type_id, int nf, const int32_t* col,
           int32_t* gob_status, ReplyRecord* out) {
    if (n <= 0) return;
    if (nf < 1 || nf > kMaxFields) throw std::invalid_argument("GobBridge: 1..8 integer fields");
    std::lock_guard<std::mutex> g(mu_);  // connections flush concurrently
    PT_HIP_CHECK(hipSetDevice(device_));
    const size_t nbytes = (size_t)offsets[n];
    grow(n, nbytes);
    PT_HIP_CHECK(hipEventRecord(ev_in_, order_));  // after the runtime's queued Sends
    PT_HIP_CHECK(hipStreamWaitEvent(stream_, ev_in_, 0));
    memcpy(h_bytes_, bytes, nbytes);
    memcpy(h_off_, offsets, (size_t)(n + 1) * sizeof(int64_t));
    PT_HIP_CHECK(hipMemcpyAsync(d_bytes_, h_bytes_, nbytes, hipMemcpyHostToDevice, stream_));
    PT_HIP_CHECK(hipMemcpyAsync(d_off_, h_off_, (size_t)(n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, stream_));
    std::vector<uintptr_t> cols((size_t)nf);
    for (int f = 0; f < nf; ++f) cols[(size_t)f] = (uintptr_t)(d_cols_ + (size_t)f * cap_n_);
    launch_gob_decode((uintptr_t)d_bytes_, (uintptr_t)d_off_, n, (uint32_t)type_id, cols, (uintptr_t)d_gst_,
                      (uintptr_t)stream_);
    auto column = [&](int k) -> uintptr_t { return col[k] >= 0 && col[k] < nf ? cols[(size_t)col[k]] : 0; };
    const unsigned gx = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(gob_bridge_actor_kernel, dim3(gx), dim3(256), 0, stream_, (const int64_t*)column(3),
                       fixed_actor_, (const int32_t*)d_gst_, n, d_actor_);
    PT_HIP_CHECK(hipGetLastError());
    MboxSend a;
    a.actor = (uintptr_t)d_actor_;
    a.a0 = column(0) ? column(0) : (uintptr_t)d_zero_;
    a.a1 = column(1);
    a.a2 = column(2);
    a.method_uniform = (int)method_;
    a.M = n;
    a.table = table_;
    a.cap = cap_;
    a.n_dir = n_state_;  // ids below n_state: mailbox = id (computed routes, no registry read)
    a.affine_w = 1;
    a.rank_self = 0;
    a.origin_base = 0;
    a.out_val = (uintptr_t)d_val_;
    a.out_st = (uintptr_t)d_st_;
    a.out_n = (uint64_t)cap_n_;
    a.state = state_;
    a.n_state = n_state_;
    a.delay_ticks = delay_ticks_;
    a.ordered = method_ordered(method_);
    a.fixed_method = (int)method_;
    a.stream = (uintptr_t)stream_;
    mb_->send_sorted(a);
    PT_HIP_CHECK(hipMemcpyAsync(h_val_, d_val_, (size_t)n * 8, hipMemcpyDeviceToHost, stream_));
    PT_HIP_CHECK(hipMemcpyAsync(h_st_, d_st_, (size_t)n * 4, hipMemcpyDeviceToHost, stream_));
    PT_HIP_CHECK(hipMemcpyAsync(h_gst_, d_gst_, (size_t)n * 4, hipMemcpyDeviceToHost, stream_));
    PT_HIP_CHECK(hipEventRecord(ev_out_, stream_));
    PT_HIP_CHECK(hipStreamWaitEvent(order_, ev_out_, 0));  // the runtime's later Sends run after this batch
    PT_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int64_t i = 0; i < n; ++i) {
      out[i].value = h_val_[i];
      out[i].status = h_st_[i];
      out[i].actor = 0;
      gob_status[i] = h_gst_[i];
    }
    ++batches_;
    calls_ += (uint64_t)n;
  }

  void grow(int64_t n, size_t nbytes) {
    if ((uint64_t)n > cap_n_) {
      PT_HIP_CHECK(hipStreamSynchronize(stream_));
      release_cols();
      cap_n_ = (uint64_t)std::max<int64_t>(n, 4096);
      PT_HIP_CHECK(hipMalloc((void**)&d_cols_, cap_n_ * kMaxFields * 8));
      PT_HIP_CHECK(hipMalloc((void**)&d_zero_, cap_n_ * 8));
      PT_HIP_CHECK(hipMemset(d_zero_, 0, cap_n_ * 8));
      PT_HIP_CHECK(hipMalloc((void**)&d_actor_, cap_n_ * 4));
      PT_HIP_CHECK(hipMalloc((void**)&d_off_, (cap_n_ + 1) * 8));
      PT_HIP_CHECK(hipMalloc((void**)&d_val_, cap_n_ * 8));
      PT_HIP_CHECK(hipMalloc((void**)&d_st_, cap_n_ * 4));
      PT_HIP_CHECK(hipMalloc((void**)&d_gst_, cap_n_ * 4));
      PT_HIP_CHECK(hipHostMalloc((void**)&h_off_, (cap_n_ + 1) * 8, hipHostMallocDefault));
      PT_HIP_CHECK(hipHostMalloc((void**)&h_val_, cap_n_ * 8, hipHostMallocDefault));
      PT_HIP_CHECK(hipHostMalloc((void**)&h_st_, cap_n_ * 4, hipHostMallocDefault));
      PT_HIP_CHECK(hipHostMalloc((void**)&h_gst_, cap_n_ * 4, hipHostMallocDefault));
    }
    if (nbytes > cap_bytes_) {
      PT_HIP_CHECK(hipStreamSynchronize(stream_));
      if (d_bytes_) (void)hipFree(d_bytes_);
      if (h_bytes_) (void)hipHostFree(h_bytes_);
      cap_bytes_ = std::max<size_t>(nbytes, 1 << 16);
      PT_HIP_CHECK(hipMalloc((void**)&d_bytes_, cap_bytes_));
      PT_HIP_CHECK(hipHostMalloc((void**)&h_bytes_, cap_bytes_, hipHostMallocDefault));
    }
  }
  void release_cols() {
    for (void* p : {(void*)d_cols_, (void*)d_zero_, (void*)d_actor_, (void*)d_off_, (void*)d_val_, (void*)d_st_,
                    (void*)d_gst_})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)h_off_, (void*)h_val_, (void*)h_st_, (void*)h_gst_})
      if (p) (void)hipHostFree(p);
    d_cols_ = d_zero_ = d_val_ = nullptr;
    d_off_ = nullptr;
    d_actor_ = nullptr;
    d_st_ = d_gst_ = nullptr;
    h_off_ = nullptr;
    h_val_ = nullptr;
    h_st_ = h_gst_ = nullptr;
    cap_n_ = 0;
  }
  void release() {
    release_cols();
    if (d_bytes_) (void)hipFree(d_bytes_);
    if (h_bytes_) (void)hipHostFree(h_bytes_);
    d_bytes_ = nullptr;
    h_bytes_ = nullptr;
    cap_bytes_ = 0;
  }

  int device_;
  Mailboxes* mb_;
  uint32_t method_, fixed_actor_;
  uintptr_t table_;
  uint64_t cap_;
  uintptr_t state_;
  uint32_t n_state_;
  uint64_t delay_ticks_;
  hipStream_t order_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  std::mutex mu_;
  uint64_t cap_n_ = 0;
  size_t cap_bytes_ = 0;
  int64_t *d_cols_ = nullptr, *d_zero_ = nullptr, *d_off_ = nullptr, *d_val_ = nullptr;
  uint32_t* d_actor_ = nullptr;
  int32_t *d_st_ = nullptr, *d_gst_ = nullptr;
  uint8_t *d_bytes_ = nullptr, *h_bytes_ = nullptr;
  int64_t *h_off_ = nullptr, *h_val_ = nullptr;
  int32_t *h_st_ = nullptr, *h_gst_ = nullptr;
  uint64_t batches_ = 0, calls_ = 0;
};

}  // namespace ptype
