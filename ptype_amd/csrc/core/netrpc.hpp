// Go net/rpc over HTTP CONNECT + gob, client and server (SURVEY C10/C11/C12,
// Appendix A.2).  The reference's data plane is exactly this protocol
// (rpc.DialHTTP at cluster/rpc.go:277; servers call rpc.Register +
// rpc.HandleHTTP, example/calculator/server/server.go:16-20), so a stock Go
// client can call ptype_amd services and ptype_amd clients can call Go servers.
//
// Server methods are C++ callables: host handlers (e.g. Python callbacks) or
// device-backed handlers that pack the gob args into a 32-B MsgRecord and run
// it on a GPU actor through the persistent dispatcher (records.hpp
// DeviceSubmitFn).  Each request runs on its own thread, as Go runs each
// request in its own goroutine; responses are serialised per connection.
#pragma once
#include <stdint.h>

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "gob.hpp"
#include "net.hpp"
#include "records.hpp"
#include "shmring.hpp"
#include "util.hpp"

namespace ptype {

// A completed call: reply value or error text (rpc.ServerError / transport error).
struct RpcOutcome {
  gob::Value reply;
  std::string error;
  Errc code = Errc::kGeneric;
  bool ok() const { return error.empty(); }
};
using RpcDone = std::function<void(RpcOutcome)>;

// What the balancer holds per selected node (the reference's *rpc.Client).
class RpcConn {
 public:
  virtual ~RpcConn() = default;
  virtual void go(const std::string& method, const gob::Value& args, RpcDone done) = 0;
  virtual RpcOutcome call(const std::string& method, const gob::Value& args, int64_t timeout_ms = -1);
  virtual void close() = 0;
  virtual std::string target() const = 0;
};

// net/rpc client over TCP (rpc.DialHTTP).
class NetRpcConn : public RpcConn, public std::enable_shared_from_this<NetRpcConn> {
 public:
  static std::shared_ptr<NetRpcConn> dial_http(const std::string& host, int port, int64_t timeout_ms);
  ~NetRpcConn() override;
  void go(const std::string& method, const gob::Value& args, RpcDone done) override;
  void close() override;
  std::string target() const override { return target_; }

 private:
  NetRpcConn() = default;
  void reader();
  void fail_all(const std::string& why, Errc code);
  std::shared_ptr<Conn> conn_;
  std::string target_;
  std::mutex wmu_;
  gob::Encoder enc_;
  std::mutex pmu_;
  std::map<uint64_t, RpcDone> pending_;
  uint64_t seq_ = 0;
  bool shutdown_ = false;
  std::thread th_;
};

using RpcHandler = std::function<gob::Value(const gob::Value& args)>;  // throw Error(kRpc, msg) to fail

// K4 on the serving path: a device-BATCHED method takes n raw gob VALUE messages
// of one integer-struct type (length prefixes included, message i at
// bytes[offsets[i], offsets[i+1])) and answers all n at once -- decoded on the
// GPU straight into mailbox columns.  field_col[k] is the wire-field index of the
// method's k-th argument field (k < 3) and field_col[3] the actor field's (-1:
// absent / fixed actor).  gob_status[i] != 0: message i did not decode.
typedef int (*DeviceBatchFn)(void* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n, int64_t type_id,
                             int nf, const int32_t* field_col, int32_t* gob_status, ReplyRecord* out);

class RpcServer {
 public:
  RpcServer() = default;
  ~RpcServer();
  // "Type.Method" (rpc.Register's naming)
  void register_method(const std::string& service_method, RpcHandler h);
  bool has_service(const std::string& service) const;
  // Serve HTTP CONNECT /_goRPC_ (and GET /debug/rpc) on host:port; returns the bound port.
  int listen(const std::string& host, int port);
  void close();
  int port() const { return port_; }
  // In-process dispatch (the LocalConn fast path and the device bridge use it).
  RpcOutcome dispatch(const std::string& service_method, const gob::Value& args);
  std::map<std::string, uint64_t> call_counts() const;
  std::string debug_page() const;
  // Extra GET endpoints answering JSON (e.g. /debug/ptype -> Cluster.Stats()).
  void set_debug_handler(const std::string& path, std::function<std::string()> fn);
  // The shared-memory segment of this server's GPU actors: published as the
  // port's locator while listening, so same-node clients call them directly.
  void set_shm_segment(const std::string& name) { shm_segment_ = name; }
  // Serve `service_method` (already registered for single calls) in batches:
  // the pipelined requests a connection has buffered go through `fn` together.
  void register_device_batch(const std::string& service_method, uintptr_t fn, uintptr_t ctx,
                             std::vector<std::string> fields, std::string actor_field, size_t max_batch = 1 << 16);
  uint64_t batches() const { return batches_.load(); }
  uint64_t batched_calls() const { return batched_calls_.load(); }

 private:
  struct BatchMethod {
    DeviceBatchFn fn = nullptr;
    void* ctx = nullptr;
    std::vector<std::string> fields;
    std::string actor_field;
    size_t max_batch = 1 << 16;
  };
  struct PendingCall {
    std::string sm;
    uint64_t seq = 0;
    int64_t type_id = 0;
    std::string raw;
    std::vector<std::string> names;  // the args type's wire fields
  };
  void flush_batch(std::vector<PendingCall>& pending, const BatchMethod& bm, gob::Encoder& enc, std::mutex& emu,
                   Conn& c);
  void serve_conn(std::shared_ptr<Conn> c);
  std::map<std::string, BatchMethod> batch_methods_;
  std::atomic<uint64_t> batches_{0}, batched_calls_{0};
  mutable std::mutex mu_;
  std::map<std::string, RpcHandler> methods_;
  std::map<std::string, std::function<std::string()>> debug_handlers_;
  std::map<std::string, uint64_t> counts_;
  std::unique_ptr<Listener> listener_;
  int port_ = 0;
  std::string shm_segment_;
  bool locator_ = false;
};

// The host twin of the GPU gob bridge, for GPU-less runs and the batching tests:
// decodes each integer-struct value message on the CPU (the same wire rules as
// gob_decode_kernel) and answers Calculator.Multiply (field 0 * field 1).
int host_batch_multiply(void* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n, int64_t type_id, int nf,
                        const int32_t* field_col, int32_t* gob_status, ReplyRecord* out);

// gob args -> device message, and a device reply -> net/rpc outcome: shared by
// the in-process device bridge and the cross-process shared-memory connection.
MsgRecord encode_device_call(const gob::Value& args, int method, uint32_t actor,
                             const std::vector<std::string>& fields, const std::string& actor_field);
RpcOutcome device_outcome(const ReplyRecord& r);

// Same-node connection to a server process whose GPU actors export their
// rings in shared memory (shmring.hpp): device methods are published straight
// into the dispatcher's ring; any other method goes over a lazily dialled TCP
// net/rpc connection to the same server.
class ShmRpcConn : public RpcConn, public std::enable_shared_from_this<ShmRpcConn> {
 public:
  ShmRpcConn(std::shared_ptr<ShmSegment> seg, std::string host, int port, int64_t dial_timeout_ms);
  void go(const std::string& method, const gob::Value& args, RpcDone done) override;
  RpcOutcome call(const std::string& method, const gob::Value& args, int64_t timeout_ms = -1) override;
  void close() override;
  std::string target() const override { return host_ + ":" + std::to_string(port_); }
  uint64_t shm_calls() const { return shm_calls_.load(); }
  // where the requests go: "device" (the server GPU's ring, mapped from its dma-buf) or "host" (the segment)
  const char* ring_placement() const { return view_.bar ? "device" : "host"; }

 private:
  struct DevMethod {
    uint32_t method = 0, actor = 0;
    std::vector<std::string> fields;
    std::string actor_field;
  };
  const DevMethod* device_method(const std::string& method);
  std::shared_ptr<RpcConn> tcp();
  std::shared_ptr<ShmSegment> seg_;
  std::shared_ptr<DevRingMap> devmap_;
  std::mutex methods_mu_;
  std::unordered_map<std::string, DevMethod> methods_;  // node-stable: pointers stay valid
  ShmView view_;
  std::string host_;
  int port_;
  int64_t dial_timeout_ms_;
  std::mutex mu_;
  std::shared_ptr<RpcConn> tcp_;
  std::atomic<bool> closed_{false};
  std::atomic<uint64_t> shm_calls_{0};
};

// In-process connection to a server living in this process: same semantics as
// a TCP connection, no sockets (used when the dialled port is served locally).
class LocalRpcConn : public RpcConn {
 public:
  LocalRpcConn(std::shared_ptr<RpcServer> s, std::string target) : srv_(std::move(s)), target_(std::move(target)) {}
  void go(const std::string& method, const gob::Value& args, RpcDone done) override;
  RpcOutcome call(const std::string& method, const gob::Value& args, int64_t timeout_ms = -1) override {
    (void)timeout_ms;  // inline dispatch on the caller's thread: no socket, no thread hop
    if (closed_.load()) {
      RpcOutcome o;
      o.error = "connection is shut down";
      o.code = Errc::kShutdown;
      return o;
    }
    return srv_->dispatch(method, args);
  }
  void close() override { closed_ = true; }
  std::string target() const override { return target_; }

 private:
  std::shared_ptr<RpcServer> srv_;
  std::string target_;
  std::atomic<bool> closed_{false};
};

// Process-wide table of servers by port, for the LocalRpcConn fast path.
void local_server_register(int port, std::shared_ptr<RpcServer> s);
void local_server_unregister(int port);
std::shared_ptr<RpcServer> local_server_lookup(const std::string& host, int port);
bool is_local_host(const std::string& host);

// Dial the way the reference does (rpc.DialHTTP("tcp", host:port)), taking the
// in-process fast path when the port is served by this process.
std::shared_ptr<RpcConn> dial_node(const std::string& host, int64_t port, int64_t timeout_ms, bool allow_local);

}  // namespace ptype
