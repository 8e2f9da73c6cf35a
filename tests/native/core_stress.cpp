// Host control-plane stress program, built with -fsanitize=thread and with
// -fsanitize=address,undefined (tests/test_sanitizers.py).
//
// The reference runs its whole suite under Go's race detector (`go test -race`,
// Makefile:2).  The C++ control plane is exercised here WITHOUT Python so the
// sanitizer runtime owns the process: concurrent channels, a 3-member Raft
// cluster with concurrent clients, watches, leases and a leader failover, the
// net/rpc server with a balancer-driven client under concurrent Call/Go, and
// the Cluster facade (Join -> register -> watch -> NewClient -> Call -> Close).
//
// usage: core_stress <workdir> [channel|raft|rpc|api|learner ...]   (default: all)
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "api.hpp"
#include "balancer.hpp"
#include "config.hpp"
#include "dp_link.hpp"
#include "kvclient.hpp"
#include "member.hpp"
#include "netrpc.hpp"
#include "shmring.hpp"
#include "util.hpp"

using namespace ptype;

namespace {

int g_failures = 0;
#define CHECK(cond)                                                                \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                                \
    }                                                                              \
  } while (0)

int free_port() {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  ::bind(fd, (sockaddr*)&a, sizeof a);
  socklen_t n = sizeof a;
  ::getsockname(fd, (sockaddr*)&a, &n);
  const int p = ntohs(a.sin_port);
  ::close(fd);
  return p;
}

std::string url(int port) { return "http://127.0.0.1:" + std::to_string(port); }

MemberConfig member_cfg(const std::string& dir, const std::string& name, int pp, int cp, const std::string& ic) {
  MemberConfig m;
  m.name = name;
  m.dir = dir + "/" + name;
  m.lpurls = m.apurls = {url(pp)};
  m.lcurls = m.acurls = {url(cp)};
  m.initial_cluster = ic;
  m.heartbeat_ms = 20;
  m.election_ms = 200;
  m.unsafe_no_fsync = true;
  return m;
}

// ---------------------------------------------------------------- scenarios
void scenario_channel() {
  auto ch = std::make_shared<Channel<int>>(16);
  std::atomic<long> sum{0};
  std::vector<std::thread> prod, cons;
  for (int p = 0; p < 4; ++p)
    prod.emplace_back([&, p] {
      for (int i = 1; i <= 5000; ++i) ch->send(i);
    });
  for (int c = 0; c < 3; ++c)
    cons.emplace_back([&] {
      for (;;) {
        bool closed = false;
        auto v = ch->recv(1000, &closed);
        if (v) sum += *v;
        if (closed) return;
      }
    });
  for (auto& t : prod) t.join();
  ch->close();
  for (auto& t : cons) t.join();
  CHECK(sum.load() == 4L * 5000 * 5001 / 2);
  // rendezvous channel: send returns once taken
  auto rv = std::make_shared<Channel<std::string>>(0);
  std::thread taker([&] {
    auto v = rv->recv(5000);
    CHECK(v && *v == "x");
  });
  CHECK(rv->send("x"));
  taker.join();
}

void scenario_raft(const std::string& dir) {
  const int n = 3;
  std::vector<int> pp(n), cp(n);
  std::string ic;
  for (int i = 0; i < n; ++i) {
    pp[i] = free_port();
    cp[i] = free_port();
    ic += (i ? "," : "") + std::string("m") + std::to_string(i) + "=" + url(pp[i]);
  }
  std::vector<std::unique_ptr<Member>> ms;
  for (int i = 0; i < n; ++i) ms.emplace_back(new Member(member_cfg(dir, "m" + std::to_string(i), pp[i], cp[i], ic)));
  {
    std::vector<std::thread> ts;
    for (auto& m : ms) ts.emplace_back([&m] { m->start(); });
    for (auto& t : ts) t.join();
  }
  for (auto& m : ms) CHECK(m->wait_ready(15000));

  std::vector<std::shared_ptr<KvClient>> cli;
  for (int i = 0; i < n; ++i) cli.push_back(std::make_shared<KvClient>(std::vector<std::string>{url(cp[i])}));

  // a prefix watch counting events while writers run
  auto ctx = Context::with_cancel(Context::background());
  auto wch = cli[0]->watch(ctx, "stress/", "stress0", 0);
  std::atomic<int> events{0};
  std::thread watcher([&] {
    for (;;) {
      bool closed = false;
      auto r = wch->recv(200, &closed);
      if (r) events += (int)r->events.size();
      if (closed) return;
    }
  });
  // leases: grant + keepalive stream while writes go on
  int64_t ttl = 0;
  const int64_t lease = cli[1]->grant(2, &ttl);
  CHECK(lease != 0);
  auto kctx = Context::with_cancel(Context::background());
  auto kch = cli[1]->keepalive(kctx, lease);

  std::atomic<int> ok{0};
  std::vector<std::thread> writers;
  for (int w = 0; w < 6; ++w)
    writers.emplace_back([&, w] {
      auto& c = cli[w % n];
      for (int i = 0; i < 40; ++i) {
        const std::string k = "stress/" + std::to_string(w) + "/" + std::to_string(i);
        try {
          c->put(k, "v" + std::to_string(i), (i % 5 == 0) ? lease : 0);
          RangeOpts o;
          auto r = c->get(k, o);
          if (!r.kvs.empty()) ++ok;
        } catch (const Error& e) {
          std::fprintf(stderr, "writer %d: %s\n", w, e.what());
        }
      }
    });
  for (auto& t : writers) t.join();
  CHECK(ok.load() == 6 * 40);
  RangeOpts all;
  all.end = "stress0";
  all.count_only = true;
  CHECK(cli[2]->get("stress/", all).count == 240);
  for (int i = 0; i < 50 && events.load() < 240; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  CHECK(events.load() >= 240);
  kctx->cancel();

  // leader failover: close the leader, the other two elect a new one and serve writes
  const uint64_t leader = ms[0]->leader();
  int li = -1;
  for (int i = 0; i < n; ++i)
    if (ms[i]->id() == leader) li = i;
  CHECK(li >= 0);
  if (li >= 0) {
    ms[li]->close();
    const int s = (li + 1) % n;
    bool wrote = false;
    for (int a = 0; a < 100 && !wrote; ++a) {
      try {
        cli[s]->put("after/failover", "ok", 0, 1000);
        wrote = true;
      } catch (const Error&) {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      }
    }
    CHECK(wrote);
    CHECK(ms[s]->leader() != leader);
  }
  ctx->cancel();
  watcher.join();
  for (auto& c : cli) c->close();
  for (auto& m : ms) m->close();
}

void scenario_rpc() {
  auto srv = std::make_shared<RpcServer>();
  srv->register_method("Calc.Multiply", [](const gob::Value& a) {
    const gob::Value* x = a.field("A");
    const gob::Value* y = a.field("B");
    if (!x || !y) fail(Errc::kRpc, "bad args");
    return gob::Value::Int(x->i * y->i);
  });
  std::atomic<int> flaky{0};
  srv->register_method("Calc.Flaky", [&flaky](const gob::Value&) {
    if (++flaky % 3) fail(Errc::kRpc, "failed");
    return gob::Value::Int(1);
  });
  const int port = srv->listen("127.0.0.1", 0);
  auto nodes = std::make_shared<NodesChan>(4);
  nodes->send({Node{"127.0.0.1", port}});
  ConnConfig cc;
  cc.retries = 2;
  cc.allow_local = false;  // force the socket path (HTTP CONNECT + gob)
  auto client = std::make_shared<RpcClient>("127.0.0.1", "calc", nodes, cc);
  std::atomic<int> good{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 100; ++i) {
        gob::Value args = gob::Value::Struct("Args");
        args.fields = {{"A", gob::Value::Int(t)}, {"B", gob::Value::Int(i)}};
        try {
          if (client->call("Calc.Multiply", args).i == (int64_t)t * i) ++good;
        } catch (const Error& e) {
          std::fprintf(stderr, "call: %s\n", e.what());
        }
      }
    });
  // async Go calls sharing one done channel
  auto done = std::make_shared<Channel<std::shared_ptr<RpcCall>>>(64);
  for (int i = 0; i < 50; ++i) {
    gob::Value args = gob::Value::Struct("Args");
    args.fields = {{"A", gob::Value::Int(i)}, {"B", gob::Value::Int(2)}};
    client->go("Calc.Multiply", args, done);
  }
  int async_ok = 0;
  for (int i = 0; i < 50; ++i) {
    auto c = done->recv(10000);
    if (c && (*c)->error.empty() && (*c)->reply.i == (*c)->args.field("A")->i * 2) ++async_ok;
  }
  for (auto& t : ts) t.join();
  CHECK(good.load() == 800);
  CHECK(async_ok == 50);
  // retry: fails twice, third attempt passes (bounded retries)
  gob::Value none = gob::Value::Struct("Args");
  bool passed = false;
  try {
    passed = client->call("Calc.Flaky", none).i == 1;
  } catch (const Error&) {
  }
  CHECK(passed);
  // re-balance while calls are in flight: same node list again, then a new server
  auto srv2 = std::make_shared<RpcServer>();
  srv2->register_method("Calc.Multiply", [](const gob::Value& a) { return gob::Value::Int(a.field("A")->i * 1000); });
  const int port2 = srv2->listen("127.0.0.1", 0);
  std::thread rebal([&] {
    nodes->send({Node{"127.0.0.1", port}, Node{"127.0.0.1", port2}});
    nodes->send({Node{"127.0.0.1", port2}});
  });
  for (int i = 0; i < 200; ++i) {
    gob::Value args = gob::Value::Struct("Args");
    args.fields = {{"A", gob::Value::Int(3)}, {"B", gob::Value::Int(5)}};
    try {
      const int64_t v = client->call("Calc.Multiply", args).i;
      CHECK(v == 15 || v == 3000);
    } catch (const Error&) {
    }
  }
  rebal.join();
  client->close();
  srv->close();
  srv2->close();
}

void scenario_cluster_api(const std::string& dir) {
  const int pp = free_port(), cp = free_port(), sp = free_port();
  Config cfg;
  cfg.service_name = "calculator";
  cfg.node_name = "node1";
  cfg.port = sp;
  cfg.member = std::make_shared<MemberConfig>(member_cfg(dir, "api0", pp, cp, "api0=" + url(pp)));
  setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1", 1);
  auto srv = std::make_shared<RpcServer>();
  srv->register_method("Calculator.Multiply",
                       [](const gob::Value& a) { return gob::Value::Int(a.field("A")->i * a.field("B")->i); });
  srv->listen("127.0.0.1", sp);
  auto c = Cluster::join(Context::background(), cfg);
  auto svcs = c->registry->services(Context::background());
  CHECK(svcs.count("calculator") == 1);
  ConnConfig cc;
  cc.allow_local = false;
  auto client = c->new_client("calculator", &cc);
  std::vector<std::thread> ts;
  std::atomic<int> good{0};
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 50; ++i) {
        gob::Value args = gob::Value::Struct("Args");
        args.fields = {{"A", gob::Value::Int(7)}, {"B", gob::Value::Int(t + i)}};
        try {
          if (client->call("Calculator.Multiply", args).i == 7 * (t + i)) ++good;
        } catch (const Error& e) {
          std::fprintf(stderr, "api call: %s\n", e.what());
        }
      }
    });
  // store traffic concurrently with the calls
  for (int i = 0; i < 50; ++i) c->store->put(Context::background(), "k" + std::to_string(i), "v");
  CHECK(c->store->get(Context::background(), "k7").size() == 1);
  for (auto& t : ts) t.join();
  CHECK(good.load() == 200);
  client->close();
  c->close();
  srv->close();
}

// Same-node shared-memory path (shmring.hpp): a CPU thread plays the GPU
// dispatcher (same protocol: in-order slots, tags, replies), client threads call
// through dial_node -> ShmRpcConn; a non-device method falls back to TCP.
void scenario_shm() {
  const uint32_t ring = 256;
  auto seg = ShmSegment::create("ptype-stress-" + std::to_string(getpid()), shm_bytes(ring));
  ShmView v = shm_view(seg->base(), ring);
  for (uint32_t i = 0; i < ring; ++i) v.owner[i].store(i);
  v.hdr->ring = ring;
  v.hdr->owner_pid = (int32_t)getpid();
  ShmMethod& mm = v.hdr->methods[0];
  std::strncpy(mm.name, "Calculator.Multiply", sizeof mm.name - 1);
  mm.method = kCalculatorMultiply;
  mm.n_fields = 2;
  std::strncpy(mm.fields[0], "A", 31);
  std::strncpy(mm.fields[1], "B", 31);
  v.hdr->n_methods.store(1);
  __atomic_store_n(&v.hdr->magic, kShmMagic, __ATOMIC_RELEASE);
  std::atomic<bool> stop{false};
  std::atomic<int> pokes{0};
  std::thread disp([&] {  // the "dispatcher": runs while RUNNING, parks after idling
    uint64_t head = 0;
    int idle = 0;
    __atomic_store_n(&v.ctrl->state, (uint64_t)kRunning, __ATOMIC_SEQ_CST);
    while (!stop.load()) {
      RingSlot* sl = &v.req[head & (ring - 1)];
      if (__atomic_load_n(&sl->tag, __ATOMIC_ACQUIRE) != head + 1) {
        if (++idle > 2000) {  // park as the GPU wave does: STOPPED, re-check, sleep until poked
          __atomic_store_n(&v.ctrl->state, (uint64_t)kStopped, __ATOMIC_SEQ_CST);
          while (!stop.load() && __atomic_load_n(&sl->tag, __ATOMIC_SEQ_CST) != head + 1) {
            shm_futex_wait(&v.hdr->wake, 0, 1000);
            if (v.hdr->wake.exchange(0)) ++pokes;
          }
          __atomic_store_n(&v.ctrl->state, (uint64_t)kRunning, __ATOMIC_SEQ_CST);
          idle = 0;
        }
        std::this_thread::yield();
        continue;
      }
      idle = 0;
      const MsgRecord m = sl->msg;
      ReplySlot* o = &v.rep[head & (ring - 1)];
      o->value = m.method == kCalculatorMultiply ? m.a0 * m.a1 : 0;
      const uint32_t st = m.method == kCalculatorMultiply ? kStatusOk : kStatusNoMethod;
      __atomic_store_n(&o->tag, reply_tag(head, st), __ATOMIC_RELEASE);  // the GPU writes value + tag as one 16-B store
      ++head;
    }
  });
  // the server process side: a net/rpc server on the same port for other methods
  auto srv = std::make_shared<RpcServer>();
  srv->register_method("Calculator.Echo", [](const gob::Value& a) { return gob::Value::Int(a.field("A")->i); });
  srv->set_shm_segment(seg->name());
  const int port = srv->listen("127.0.0.1", 0);
  auto conn = dial_node("127.0.0.1", port, 2000, true);
  CHECK(dynamic_cast<ShmRpcConn*>(conn.get()) != nullptr);
  std::atomic<int> good{0};
  std::mutex bad_mu;
  std::string first_bad;
  std::vector<std::thread> ts;
  for (int t = 0; t < 6; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 300; ++i) {
        gob::Value args = gob::Value::Struct("Args");
        args.fields = {{"A", gob::Value::Int(t + 1)}, {"B", gob::Value::Int(i)}};
        RpcOutcome o = conn->call("Calculator.Multiply", args, 5000);
        if (o.ok() && o.reply.i == (int64_t)(t + 1) * i) {
          ++good;
        } else {
          std::lock_guard<std::mutex> g(bad_mu);
          if (first_bad.empty())
            first_bad = "call " + std::to_string(t) + "/" + std::to_string(i) + ": ok=" + std::to_string(o.ok()) +
                        " err=" + o.error + " reply=" + std::to_string(o.reply.i);
        }
        if (i % 100 == 99) std::this_thread::sleep_for(std::chrono::milliseconds(30));  // let it park
      }
    });
  for (auto& th : ts) th.join();
  if (good.load() != 1800) fprintf(stderr, "shm: %d of 1800 good; first failure %s\n", good.load(), first_bad.c_str());
  CHECK(good.load() == 1800);
  CHECK(pokes.load() > 0);  // calls woke a parked dispatcher
  gob::Value e = gob::Value::Struct("Args");
  e.fields = {{"A", gob::Value::Int(42)}};
  RpcOutcome o = conn->call("Calculator.Echo", e, 5000);  // not exported: TCP fallback
  CHECK(o.ok() && o.reply.i == 42);
  CHECK(srv->call_counts()["Calculator.Echo"] == 1 && srv->call_counts().count("Calculator.Multiply") == 0);
  conn->close();
  srv->close();
  CHECK(shm_locator_lookup(port).empty());
  stop.store(true);
  shm_futex_wake(&v.hdr->wake);
  disp.join();
}

// The Send watchdog's abort against the engines' enqueues (csrc/core/dp_link.hpp;
// the watchdog must never free a communicator an engine is inside).
// Engine threads enter / "enqueue" / leave in a loop while the watchdog retires the
// cell mid-Send and then "aborts" the communicator: no enqueue may ever see it
// aborted, retire hands it out once, and every enqueue after the poison is refused.
void scenario_commcell() {
  struct Comm {
    std::atomic<int> alive{1};
    std::atomic<long> uses{0};
  };
  for (int round = 0; round < 24; ++round) {
    auto* comm = new Comm;
    CommCell cell;
    cell.install(comm);
    std::atomic<int> bad{0};
    std::atomic<long> refused{0};
    std::vector<std::thread> engines;
    for (int t = 0; t < 4; ++t)
      engines.emplace_back([&, t] {
        for (int i = 0; i < 4000; ++i) {
          void* c = cell.enter();
          if (!c) {
            refused.fetch_add(1);
            continue;
          }
          auto* cm = static_cast<Comm*>(c);
          if (!cm->alive.load()) bad.fetch_add(1);
          cm->uses.fetch_add(1);  // the RCCL enqueue
          if ((i + t) % 97 == 0) std::this_thread::sleep_for(std::chrono::microseconds(30));
          if (!cm->alive.load()) bad.fetch_add(1);
          cell.leave();
        }
      });
    std::this_thread::sleep_for(std::chrono::microseconds(200 + 150 * (round % 8)));
    void* c = cell.retire(5.0);  // the watchdog, mid-Send
    CHECK(c == comm);
    comm->alive.store(0);  // ncclCommAbort: from here any use would be a use after free
    CHECK(cell.retire(5.0) == nullptr);  // handed out once
    CHECK(cell.failed() && cell.enter() == nullptr);
    for (auto& th : engines) th.join();
    CHECK(bad.load() == 0);
    CHECK(cell.users.load() == 0);
    delete comm;
  }
}

// Elastic scale-out: a second member joins as a learner through the first one's
// client URL and is promoted once caught up (cluster/cluster.go:105-147, :183-195).
void scenario_learner(const std::string& dir) {
  setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1", 1);
  const int pp1 = free_port(), cp1 = free_port(), pp2 = free_port(), cp2 = free_port();
  Config a;
  a.service_name = "svc";
  a.node_name = "a";
  a.port = free_port();
  a.member = std::make_shared<MemberConfig>(member_cfg(dir, "la", pp1, cp1, "la=" + url(pp1)));
  auto ca = Cluster::join(Context::background(), a);
  for (int i = 0; i < 20; ++i) ca->store->put(Context::background(), "pre" + std::to_string(i), "x");
  Config b;
  b.service_name = "svc";
  b.node_name = "b";
  b.port = free_port();
  b.initial_cluster_client_urls = {url(cp1)};
  b.member = std::make_shared<MemberConfig>(member_cfg(dir, "lb", pp2, cp2, ""));
  b.member->cluster_state = "existing";
  auto cb = Cluster::join(Context::background(), b);
  auto ms = cb->member_list(Context::background());
  CHECK(ms.size() == 2);
  for (const auto& m : ms) CHECK(!m.is_learner);
  CHECK(cb->store->get(Context::background(), "pre19").size() == 1);  // caught up before promotion
  auto nodes = cb->registry->services(Context::background());
  CHECK(nodes["svc"].size() == 2);
  cb->close();
  ca->close();
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <workdir> [channel|raft|rpc|api]...\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  std::vector<std::string> want(argv + 2, argv + argc);
  if (want.empty()) want = {"channel", "raft", "rpc", "api", "learner", "shm", "commcell"};
  std::map<std::string, std::function<void()>> all = {
      {"channel", [] { scenario_channel(); }},
      {"raft", [&] { scenario_raft(dir); }},
      {"rpc", [] { scenario_rpc(); }},
      {"api", [&] { scenario_cluster_api(dir); }},
      {"learner", [&] { scenario_learner(dir); }},
      {"shm", [] { scenario_shm(); }},
      {"commcell", [] { scenario_commcell(); }},
  };
  for (const auto& w : want) {
    auto it = all.find(w);
    if (it == all.end()) {
      std::fprintf(stderr, "unknown scenario %s\n", w.c_str());
      return 2;
    }
    const int before = g_failures;
    try {
      it->second();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "scenario %s threw: %s\n", w.c_str(), e.what());
      ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "OK" : "FAIL", w.c_str());
    std::fflush(stdout);
  }
  return g_failures ? 1 : 0;
}
