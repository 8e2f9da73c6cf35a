#include "netrpc.hpp"

#include <condition_variable>
#include <set>

#include "config.hpp"

namespace ptype {

// ---------------------------------------------------------------- RpcConn
RpcOutcome RpcConn::call(const std::string& method, const gob::Value& args, int64_t timeout_ms) {
  struct Slot {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    RpcOutcome out;
  };
  auto s = std::make_shared<Slot>();
  go(method, args, [s](RpcOutcome o) {
    std::lock_guard<std::mutex> g(s->mu);
    s->out = std::move(o);
    s->done = true;
    s->cv.notify_all();
  });
  std::unique_lock<std::mutex> g(s->mu);
  if (timeout_ms < 0) {
    s->cv.wait(g, [&] { return s->done; });
  } else if (!s->cv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return s->done; })) {
    RpcOutcome o;
    o.error = "rpc: call timed out";
    o.code = Errc::kTimeout;
    return o;
  }
  return s->out;
}

// ---------------------------------------------------------------- NetRpcConn
static gob::Value make_request(const std::string& method, uint64_t seq) {
  gob::Value r = gob::Value::Struct("Request");
  r.fields.emplace_back("ServiceMethod", gob::Value::String(method));
  r.fields.emplace_back("Seq", gob::Value::Uint(seq));
  return r;
}

std::shared_ptr<NetRpcConn> NetRpcConn::dial_http(const std::string& host, int port, int64_t timeout_ms) {
  std::string err;
  auto c = tcp_connect(host, port, timeout_ms, &err);
  if (!c) fail(Errc::kUnavailable, err);
  if (!c->write_raw("CONNECT /_goRPC_ HTTP/1.0\n\n")) fail(Errc::kUnavailable, "rpc: handshake write failed");
  std::string status;
  if (!c->read_line(&status)) fail(Errc::kUnavailable, "unexpected EOF");
  for (std::string h; c->read_line(&h) && !h.empty();) {
  }
  if (status.find("200 Connected to Go RPC") == std::string::npos)
    fail(Errc::kUnavailable, "unexpected HTTP response: " + status);
  std::shared_ptr<NetRpcConn> r(new NetRpcConn());
  r->conn_ = c;
  r->target_ = host + ":" + std::to_string(port);
  NetRpcConn* raw = r.get();
  r->th_ = std::thread([raw] { raw->reader(); });
  return r;
}

NetRpcConn::~NetRpcConn() {
  close();
  if (th_.joinable()) th_.join();
}

void NetRpcConn::go(const std::string& method, const gob::Value& args, RpcDone done) {
  std::string buf;
  uint64_t seq;
  {
    std::lock_guard<std::mutex> g(pmu_);
    if (shutdown_) {
      RpcOutcome o;
      o.error = "connection is shut down";
      o.code = Errc::kShutdown;
      done(o);
      return;
    }
    seq = seq_++;
    pending_[seq] = std::move(done);
  }
  bool ok;
  {
    std::lock_guard<std::mutex> g(wmu_);
    try {
      enc_.encode(make_request(method, seq), &buf);
      enc_.encode(args, &buf);
      ok = conn_->write_raw(buf);
    } catch (const std::exception& e) {
      RpcDone d;
      {
        std::lock_guard<std::mutex> g2(pmu_);
        d = std::move(pending_[seq]);
        pending_.erase(seq);
      }
      RpcOutcome o;
      o.error = std::string("gob: ") + e.what();
      d(o);
      return;
    }
  }
  if (!ok) fail_all("connection is shut down", Errc::kShutdown);
}

void NetRpcConn::reader() {
  gob::Decoder dec([this](char* p, size_t n) { return conn_->read_exact(p, n); });
  std::string why = "connection is shut down";
  try {
    for (;;) {
      gob::Value hdr, body;
      if (!dec.decode(&hdr)) break;
      if (!dec.decode(&body)) {
        why = "unexpected EOF";
        break;
      }
      const gob::Value* seqv = hdr.field("Seq");
      const gob::Value* errv = hdr.field("Error");
      const uint64_t seq = seqv ? seqv->u : 0;
      RpcDone d;
      {
        std::lock_guard<std::mutex> g(pmu_);
        auto it = pending_.find(seq);
        if (it == pending_.end()) continue;
        d = std::move(it->second);
        pending_.erase(it);
      }
      RpcOutcome o;
      if (errv && !errv->s.empty()) {
        o.error = errv->s;
        o.code = Errc::kRpc;
      } else {
        o.reply = std::move(body);
      }
      d(std::move(o));
    }
  } catch (const std::exception& e) {
    why = e.what();
  }
  fail_all(why, Errc::kShutdown);
}

void NetRpcConn::fail_all(const std::string& why, Errc code) {
  std::map<uint64_t, RpcDone> ps;
  {
    std::lock_guard<std::mutex> g(pmu_);
    shutdown_ = true;
    ps.swap(pending_);
  }
  for (auto& kv : ps) {
    RpcOutcome o;
    o.error = why;
    o.code = code;
    kv.second(o);
  }
}

void NetRpcConn::close() {
  {
    std::lock_guard<std::mutex> g(pmu_);
    shutdown_ = true;
  }
  if (conn_) conn_->shutdown();
}

// ---------------------------------------------------------------- server
RpcServer::~RpcServer() { close(); }

void RpcServer::register_method(const std::string& sm, RpcHandler h) {
  if (sm.find('.') == std::string::npos) fail("rpc: method name must be Type.Method: " + sm);
  std::lock_guard<std::mutex> g(mu_);
  methods_[sm] = std::move(h);
}

bool RpcServer::has_service(const std::string& service) const {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : methods_)
    if (kv.first.compare(0, service.size() + 1, service + ".") == 0) return true;
  return false;
}

RpcOutcome RpcServer::dispatch(const std::string& sm, const gob::Value& args) {
  RpcOutcome o;
  o.code = Errc::kRpc;
  const size_t dot = sm.rfind('.');
  if (dot == std::string::npos || dot == 0 || dot + 1 == sm.size()) {
    o.error = "rpc: service/method request ill-formed: " + sm;
    return o;
  }
  RpcHandler h;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = methods_.find(sm);
    if (it == methods_.end()) {
      const std::string svc = sm.substr(0, dot);
      bool svc_found = false;
      for (const auto& kv : methods_)
        if (kv.first.compare(0, svc.size() + 1, svc + ".") == 0) svc_found = true;
      o.error = svc_found ? "rpc: can't find method " + sm : "rpc: can't find service " + sm;
      return o;
    }
    h = it->second;
    ++counts_[sm];
  }
  try {
    o.reply = h(args);
    o.code = Errc::kGeneric;
  } catch (const std::exception& e) {
    o.error = e.what();
  }
  return o;
}

int RpcServer::listen(const std::string& host, int port) {
  listener_.reset(new Listener(host.empty() ? "0.0.0.0" : host, port,
                               [this](std::shared_ptr<Conn> c) { serve_conn(c); }));
  port_ = listener_->port();
  if (!shm_segment_.empty()) {  // same-node clients may call the GPU actors through shared memory
    shm_locator_publish(port_, shm_segment_);
    locator_ = true;
  }
  return port_;
}

void RpcServer::close() {
  if (locator_) {
    shm_locator_remove(port_);
    locator_ = false;
  }
  if (listener_) listener_->close();
  listener_.reset();
}

std::map<std::string, uint64_t> RpcServer::call_counts() const {
  std::lock_guard<std::mutex> g(mu_);
  return counts_;
}

std::string RpcServer::debug_page() const {
  // the spirit of net/rpc's /debug/rpc: services, methods, call counts
  std::lock_guard<std::mutex> g(mu_);
  std::string o = "<html><body><title>Services</title>\n";
  std::string cur;
  for (const auto& kv : methods_) {
    const std::string svc = kv.first.substr(0, kv.first.rfind('.'));
    if (svc != cur) {
      o += "<hr>Service " + svc + "<hr>\n";
      cur = svc;
    }
    auto c = counts_.find(kv.first);
    o += "<tr><td>" + kv.first + "</td><td>" + std::to_string(c == counts_.end() ? 0 : c->second) + "</td></tr>\n";
  }
  return o + "</body></html>\n";
}

void RpcServer::set_debug_handler(const std::string& path, std::function<std::string()> fn) {
  std::lock_guard<std::mutex> g(mu_);
  if (fn)
    debug_handlers_[path] = std::move(fn);
  else
    debug_handlers_.erase(path);
}

void RpcServer::serve_conn(std::shared_ptr<Conn> c) {
  std::string line;
  if (!c->read_line(&line)) return;
  for (std::string h; c->read_line(&h) && !h.empty();) {
  }
  const auto parts = split(line, ' ');
  const std::string method = parts.size() > 0 ? parts[0] : "";
  const std::string path = parts.size() > 1 ? parts[1] : "";
  if (method == "GET" && path == "/debug/rpc") {
    const std::string body = debug_page();
    c->write_raw("HTTP/1.0 200 OK\r\nContent-Type: text/html; charset=utf-8\r\nContent-Length: " +
                 std::to_string(body.size()) + "\r\n\r\n" + body);
    return;
  }
  if (method == "GET") {
    std::function<std::string()> fn;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = debug_handlers_.find(path);
      if (it != debug_handlers_.end()) fn = it->second;
    }
    if (fn) {
      std::string body, status = "200 OK";
      try {
        body = fn();
      } catch (const std::exception& e) {
        status = "500 Internal Server Error";
        body = std::string("{\"error\": \"") + e.what() + "\"}";
      }
      c->write_raw("HTTP/1.0 " + status + "\r\nContent-Type: application/json\r\nContent-Length: " +
                   std::to_string(body.size()) + "\r\n\r\n" + body);
      return;
    }
  }
  if (method != "CONNECT") {
    c->write_raw("HTTP/1.0 405 Method Not Allowed\r\nContent-Type: text/plain; charset=utf-8\r\n\r\n405 must CONNECT\n");
    return;
  }
  if (path != "/_goRPC_") {
    c->write_raw("HTTP/1.0 404 Not Found\r\n\r\n404 page not found\n");
    return;
  }
  c->write_raw("HTTP/1.0 200 Connected to Go RPC\n\n");
  auto enc = std::make_shared<gob::Encoder>();
  auto emu = std::make_shared<std::mutex>();
  std::atomic<int> inflight{0};
  gob::Decoder dec([c](char* p, size_t n) { return c->read_exact(p, n); });
  std::vector<PendingCall> pending;  // K4: buffered requests of one batched method
  const BatchMethod* pending_bm = nullptr;
  auto flush = [&] {
    if (!pending.empty()) flush_batch(pending, *pending_bm, *enc, *emu, *c);
    pending.clear();
    pending_bm = nullptr;
  };
  try {
    for (;;) {
      gob::Value req, args;
      if (!dec.decode(&req)) break;
      const gob::Value* smv = req.field("ServiceMethod");
      const gob::Value* seqv = req.field("Seq");
      const std::string sm = smv ? smv->s : "";
      const uint64_t seq = seqv ? seqv->u : 0;
      const BatchMethod* bm = nullptr;
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = batch_methods_.find(sm);
        if (it != batch_methods_.end()) bm = &it->second;  // (entries are never erased)
      }
      if (bm) {
        PendingCall pc;
        pc.sm = sm;
        pc.seq = seq;
        if (!dec.next_raw(&pc.raw, &pc.type_id)) break;
        if (dec.int_struct_fields(pc.type_id, &pc.names) && pc.names.size() <= 8) {
          if (pending_bm && (pending_bm != bm || pending.back().type_id != pc.type_id)) flush();
          pending_bm = bm;
          pending.push_back(std::move(pc));
          // the connection's pipelined requests, until its input runs dry
          if (pending.size() >= bm->max_batch || !c->input_pending()) flush();
          continue;
        }
        dec.decode_raw(pc.raw, &args);  // not an integer struct: the single-call path
      } else if (!dec.decode(&args)) {
        break;
      }
      if (!c->input_pending()) flush();
      ++inflight;
      std::thread([this, c, enc, emu, sm, seq, args, &inflight] {  // a goroutine per request
        RpcOutcome o = dispatch(sm, args);
        gob::Value resp = gob::Value::Struct("Response");
        resp.fields.emplace_back("ServiceMethod", gob::Value::String(sm));
        resp.fields.emplace_back("Seq", gob::Value::Uint(seq));
        resp.fields.emplace_back("Error", gob::Value::String(o.error));
        std::string buf;
        {
          std::lock_guard<std::mutex> g(*emu);
          try {
            enc->encode(resp, &buf);
            enc->encode(o.ok() ? o.reply : gob::Value::Struct(""), &buf);  // invalidRequest = struct{}{}
          } catch (const std::exception& e) {
            buf.clear();
            resp.fields[2].second = gob::Value::String(std::string("gob: ") + e.what());
            enc->encode(resp, &buf);
            enc->encode(gob::Value::Struct(""), &buf);
          }
          c->write_raw(buf);
        }
        --inflight;
      }).detach();
    }
    flush();
  } catch (const std::exception&) {
  }
  c->shutdown();
  while (inflight.load() > 0) sleep_ms(1);
}

// ---------------------------------------------------------------- K4 batched device methods
void RpcServer::register_device_batch(const std::string& service_method, uintptr_t fn, uintptr_t ctx,
                                      std::vector<std::string> fields, std::string actor_field, size_t max_batch) {
  if (!fn) throw std::invalid_argument("register_device_batch: null batch function");
  if (fields.size() > 3) throw std::invalid_argument("register_device_batch: at most 3 argument fields");
  std::lock_guard<std::mutex> g(mu_);
  if (!methods_.count(service_method))
    fail(Errc::kRpc, "register_device_batch: register " + service_method + " for single calls first");
  BatchMethod& b = batch_methods_[service_method];
  b.fn = (DeviceBatchFn)fn;
  b.ctx = (void*)ctx;
  b.fields = std::move(fields);
  b.actor_field = std::move(actor_field);
  b.max_batch = std::max<size_t>(1, max_batch);
}

// One GPU pass for the buffered calls, then every Response + reply encoded in
// sequence (the same host encoder as the single-call path: identical bytes) and
// written with one syscall.
void RpcServer::flush_batch(std::vector<PendingCall>& pending, const BatchMethod& bm, gob::Encoder& enc,
                            std::mutex& emu, Conn& c) {
  const int64_t n = (int64_t)pending.size();
  const std::vector<std::string>& names = pending.front().names;
  int32_t col[4] = {-1, -1, -1, -1};
  auto index_of = [&](const std::string& f) {
    for (size_t j = 0; j < names.size(); ++j)
      if (names[j] == f) return (int32_t)j;
    return (int32_t)-1;
  };
  for (size_t k = 0; k < bm.fields.size(); ++k) col[k] = index_of(bm.fields[k]);
  if (!bm.actor_field.empty()) col[3] = index_of(bm.actor_field);
  std::string bytes;
  std::vector<int64_t> offsets((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    offsets[(size_t)i] = (int64_t)bytes.size();
    bytes += pending[(size_t)i].raw;
  }
  offsets[(size_t)n] = (int64_t)bytes.size();
  std::vector<int32_t> gst((size_t)n, 0);
  std::vector<ReplyRecord> rep((size_t)n);
  const int rc = bm.fn(bm.ctx, (const uint8_t*)bytes.data(), offsets.data(), n, pending.front().type_id,
                       (int)names.size(), col, gst.data(), rep.data());
  batches_.fetch_add(1);
  batched_calls_.fetch_add((uint64_t)n);
  {
    std::lock_guard<std::mutex> g(mu_);
    counts_[pending.front().sm] += (uint64_t)n;
  }
  std::string buf;
  std::lock_guard<std::mutex> g(emu);
  for (int64_t i = 0; i < n; ++i) {
    RpcOutcome o;
    if (rc != 0) {
      o.error = "device dispatcher unavailable";
    } else if (gst[(size_t)i] != 0) {
      o.error = "gob: decoding error (device status " + std::to_string(gst[(size_t)i]) + ")";
    } else {
      o = device_outcome(rep[(size_t)i]);
    }
    gob::Value resp = gob::Value::Struct("Response");
    resp.fields.emplace_back("ServiceMethod", gob::Value::String(pending[(size_t)i].sm));
    resp.fields.emplace_back("Seq", gob::Value::Uint(pending[(size_t)i].seq));
    resp.fields.emplace_back("Error", gob::Value::String(o.error));
    enc.encode(resp, &buf);
    enc.encode(o.ok() ? o.reply : gob::Value::Struct(""), &buf);
  }
  c.write_raw(buf);
}

namespace {
bool gob_get_uint(const uint8_t*& p, const uint8_t* end, uint64_t* x) {
  if (p >= end) return false;
  const uint8_t c = *p++;
  if (c < 128) {
    *x = c;
    return true;
  }
  const int n = 256 - c;
  if (n > 8 || end - p < n) return false;
  uint64_t v = 0;
  for (int i = 0; i < n; ++i) v = (v << 8) | *p++;
  *x = v;
  return true;
}
int64_t gob_unzz(uint64_t u) { return (u & 1) ? (int64_t)~(u >> 1) : (int64_t)(u >> 1); }
}  // namespace

int host_batch_multiply(void* ctx, const uint8_t* bytes, const int64_t* offsets, int64_t n, int64_t type_id, int nf,
                        const int32_t* field_col, int32_t* gob_status, ReplyRecord* out) {
  (void)ctx;
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* p = bytes + offsets[i];
    const uint8_t* end = bytes + offsets[i + 1];
    int64_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t st = 0;
    uint64_t len = 0, tid = 0;
    if (!gob_get_uint(p, end, &len) || (uint64_t)(end - p) != len) {
      st = 1;
    } else if (!gob_get_uint(p, end, &tid) || gob_unzz(tid) != type_id) {
      st = 2;
    } else {
      int field = -1;
      for (;;) {
        uint64_t delta, u;
        if (!gob_get_uint(p, end, &delta)) {
          st = 1;
          break;
        }
        if (delta == 0) break;
        field += (int)delta;
        if (field >= nf || field >= 8 || !gob_get_uint(p, end, &u)) {
          st = 3;
          break;
        }
        v[field] = gob_unzz(u);
      }
      if (st == 0 && p != end) st = 4;
    }
    gob_status[i] = st;
    const int64_t a = field_col[0] >= 0 ? v[field_col[0]] : 0, b = field_col[1] >= 0 ? v[field_col[1]] : 0;
    out[i].value = (int64_t)((uint64_t)a * (uint64_t)b);
    out[i].status = kStatusOk;
    out[i].actor = 0;
  }
  return 0;
}

// ---------------------------------------------------------------- local fast path
void LocalRpcConn::go(const std::string& method, const gob::Value& args, RpcDone done) {
  if (closed_.load()) {
    RpcOutcome o;
    o.error = "connection is shut down";
    o.code = Errc::kShutdown;
    done(o);
    return;
  }
  auto srv = srv_;
  std::thread([srv, method, args, done] { done(srv->dispatch(method, args)); }).detach();
}

static std::mutex g_local_mu;
static std::map<int, std::weak_ptr<RpcServer>> g_local;

void local_server_register(int port, std::shared_ptr<RpcServer> s) {
  std::lock_guard<std::mutex> g(g_local_mu);
  g_local[port] = s;
}

void local_server_unregister(int port) {
  std::lock_guard<std::mutex> g(g_local_mu);
  g_local.erase(port);
}

bool is_local_host(const std::string& host) {
  if (host == "127.0.0.1" || host == "localhost" || host == "0.0.0.0" || host == "::1") return true;
  static const std::string self = first_nonloopback_ipv4();
  return !self.empty() && host == self;
}

std::shared_ptr<RpcServer> local_server_lookup(const std::string& host, int port) {
  if (!is_local_host(host)) return nullptr;
  std::lock_guard<std::mutex> g(g_local_mu);
  auto it = g_local.find(port);
  return it == g_local.end() ? nullptr : it->second.lock();
}

MsgRecord encode_device_call(const gob::Value& args, int method, uint32_t actor,
                             const std::vector<std::string>& fields, const std::string& actor_field) {
  MsgRecord m{};
  m.actor = actor;
  m.method = (uint16_t)method;
  m.flags = kFlagValid;
  int64_t a[3] = {0, 0, 0};
  if (args.kind == gob::kStruct) {
    for (size_t k = 0; k < fields.size() && k < 3; ++k) {
      const gob::Value* f = args.field(fields[k]);
      if (f) a[k] = f->kind == gob::kUint ? (int64_t)f->u : f->i;
    }
    if (!actor_field.empty())
      if (const gob::Value* f = args.field(actor_field)) m.actor = (uint32_t)(f->kind == gob::kUint ? f->u : f->i);
  } else if (args.kind == gob::kInt) {
    a[0] = args.i;
  }
  m.a0 = a[0];
  m.a1 = a[1];
  m.a2 = a[2];
  return m;
}

RpcOutcome device_outcome(const ReplyRecord& r) {
  RpcOutcome o;
  switch (r.status) {
    case kStatusOk:
      o.reply = gob::Value::Int(r.value);
      return o;
    case kStatusFailed:
      o.error = "failed";
      break;
    case kStatusNoActor:
      o.error = "no such actor";
      break;
    default:
      o.error = "rpc: device method error status " + std::to_string(r.status);
  }
  o.code = Errc::kRpc;
  return o;
}

// ---- same-node shared-memory connection
ShmRpcConn::ShmRpcConn(std::shared_ptr<ShmSegment> seg, std::string host, int port, int64_t dial_timeout_ms)
    : seg_(std::move(seg)), host_(std::move(host)), port_(port), dial_timeout_ms_(dial_timeout_ms) {
  view_ = shm_attach_view(seg_, &devmap_);
}

// The segment's export of `method`, resolved once per name (exports are only
// ever appended, so a resolved entry stays valid; a miss re-scans the table).
const ShmRpcConn::DevMethod* ShmRpcConn::device_method(const std::string& method) {
  std::lock_guard<std::mutex> g(methods_mu_);
  auto it = methods_.find(method);
  if (it != methods_.end()) return &it->second;
  const ShmHeader* h = view_.hdr;
  const uint32_t n = std::min<uint32_t>(h->n_methods.load(std::memory_order_acquire), kShmMaxMethods);
  for (uint32_t k = 0; k < n; ++k) {
    const ShmMethod& mm = h->methods[k];
    if (method != mm.name) continue;
    DevMethod d;
    d.method = mm.method;
    d.actor = mm.actor;
    for (uint32_t f = 0; f < mm.n_fields && f < 3; ++f) d.fields.emplace_back(mm.fields[f]);
    d.actor_field = mm.actor_field;
    return &methods_.emplace(method, std::move(d)).first->second;
  }
  return nullptr;
}

std::shared_ptr<RpcConn> ShmRpcConn::tcp() {
  std::lock_guard<std::mutex> g(mu_);
  if (!tcp_) tcp_ = NetRpcConn::dial_http(host_, port_, dial_timeout_ms_);
  return tcp_;
}

RpcOutcome ShmRpcConn::call(const std::string& method, const gob::Value& args, int64_t timeout_ms) {
  if (closed_.load()) {
    RpcOutcome o;
    o.error = "connection is shut down";
    o.code = Errc::kShutdown;
    return o;
  }
  if (const DevMethod* dm = device_method(method)) {
    const MsgRecord m = encode_device_call(args, (int)dm->method, dm->actor, dm->fields, dm->actor_field);
    try {
      const ReplyRecord r = shm_call(view_, m, timeout_ms < 0 ? 30.0 : timeout_ms / 1e3);
      shm_calls_.fetch_add(1);
      return device_outcome(r);
    } catch (const Error& e) {
      RpcOutcome o;
      o.error = e.what();
      o.code = e.code();
      return o;
    }
  }
  try {  // not a device method: the server's regular net/rpc endpoint
    return tcp()->call(method, args, timeout_ms);
  } catch (const Error& e) {
    RpcOutcome o;
    o.error = e.what();
    o.code = e.code();
    return o;
  }
}

void ShmRpcConn::go(const std::string& method, const gob::Value& args, RpcDone done) {
  auto self = shared_from_this();
  std::thread([self, method, args, done] { done(self->call(method, args)); }).detach();
}

void ShmRpcConn::close() {
  closed_.store(true);
  std::lock_guard<std::mutex> g(mu_);
  if (tcp_) tcp_->close();
}

std::shared_ptr<RpcConn> dial_node(const std::string& host, int64_t port, int64_t timeout_ms, bool allow_local) {
  if (allow_local)
    if (auto s = local_server_lookup(host, (int)port)) return std::make_shared<LocalRpcConn>(s, host + ":" + std::to_string(port));
  if (allow_local && is_local_host(host)) {  // another process on this node with GPU actors in shared memory
    const std::string seg = shm_locator_lookup((int)port);
    if (!seg.empty())
      if (auto s = ShmSegment::attach(seg)) {
        try {
          return std::make_shared<ShmRpcConn>(s, host, (int)port, timeout_ms);
        } catch (const Error&) {
        }
      }
  }
  try {
    return NetRpcConn::dial_http(host, (int)port, timeout_ms);
  } catch (const Error& e) {
    fail(Errc::kUnavailable, "failed to dial service address " + host + ":" + std::to_string(port) + ": " + e.what());
  }
}

}  // namespace ptype
