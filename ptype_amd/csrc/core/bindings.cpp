// pybind11 bindings for the host control plane (_core).  Python is a thin
// layer over these: every behaviour lives in C++.
#include <pybind11/functional.h>
#include <condition_variable>
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <unordered_map>

#include "api.hpp"
#include "dataplane.hpp"
#include "follower.hpp"
#include "gob.hpp"
#include "json.hpp"
#include "records.hpp"
#include "yaml.hpp"

namespace py = pybind11;
using namespace ptype;

// ---------------------------------------------------------------- errors
static py::object g_err_base, g_err_nokey, g_err_noclient, g_err_learner, g_err_timeout, g_err_canceled, g_err_rpc,
    g_err_shutdown, g_err_config, g_err_unavail, g_err_member;

static void translate(const Error& e) {
  py::object cls = g_err_base;
  switch (e.code()) {
    case Errc::kNoKey: cls = g_err_nokey; break;
    case Errc::kNoClientAvailable: cls = g_err_noclient; break;
    case Errc::kLearnerNotReady: cls = g_err_learner; break;
    case Errc::kTimeout: cls = g_err_timeout; break;
    case Errc::kCanceled: cls = g_err_canceled; break;
    case Errc::kRpc: cls = g_err_rpc; break;
    case Errc::kShutdown: cls = g_err_shutdown; break;
    case Errc::kConfig: cls = g_err_config; break;
    case Errc::kUnavailable: cls = g_err_unavail; break;
    case Errc::kMemberExists:
    case Errc::kMemberNotFound: cls = g_err_member; break;
    default: break;
  }
  PyErr_SetString(cls.ptr(), e.what());
}

// ---------------------------------------------------------------- gob <-> python
static gob::Value to_gob(py::handle o);

static gob::Value struct_from(const std::string& name, py::iterable pairs) {
  gob::Value v = gob::Value::Struct(name);
  for (auto p : pairs) {
    auto t = p.cast<py::tuple>();
    v.fields.emplace_back(t[0].cast<std::string>(), to_gob(t[1]));
  }
  return v;
}

// Per-type facts to_gob needs for class instances (whether the type has a
// __gob_value__ helper, or its dataclass name and field names), computed once per
// type: `dataclasses.fields` and a failing hasattr cost microseconds per call on
// the single-call path (a same-node device call is ~3 us end to end).
namespace {  // internal linkage: pybind11 types are hidden-visibility
struct GobTypeInfo {
  py::object type;  // keeps the type alive, so its address is not reused
  bool helper = false, dataclass = false;
  std::string name;
  std::vector<std::pair<std::string, py::str>> fields;
};
}  // namespace

static const GobTypeInfo& gob_type_info(py::handle o) {
  static std::unordered_map<PyTypeObject*, std::unique_ptr<GobTypeInfo>> cache;  // under the GIL
  PyTypeObject* t = Py_TYPE(o.ptr());
  auto it = cache.find(t);
  if (it != cache.end()) return *it->second;
  auto info = std::make_unique<GobTypeInfo>();
  info->type = py::reinterpret_borrow<py::object>(reinterpret_cast<PyObject*>(t));
  info->helper = py::hasattr(info->type, "__gob_value__");
  info->dataclass = !info->helper && py::hasattr(info->type, "__dataclass_fields__");
  if (info->dataclass) {
    info->name = py::str(info->type.attr("__name__")).cast<std::string>();
    for (auto f : py::module_::import("dataclasses").attr("fields")(info->type)) {
      const std::string n = f.attr("name").cast<std::string>();
      info->fields.emplace_back(n, py::str(n));
    }
  }
  return *cache.emplace(t, std::move(info)).first->second;
}

static gob::Value to_gob(py::handle o) {
  if (o.is_none()) fail("gob: cannot encode None");
  if (py::isinstance<py::bool_>(o)) return gob::Value::Bool(o.cast<bool>());
  if (PyLong_CheckExact(o.ptr())) return gob::Value::Int(o.cast<int64_t>());  // hot: plain ints
  const GobTypeInfo& ti = gob_type_info(o);
  if (ti.dataclass) {
    gob::Value v = gob::Value::Struct(ti.name);
    v.fields.reserve(ti.fields.size());
    for (const auto& f : ti.fields) v.fields.emplace_back(f.first, to_gob(o.attr(f.second)));
    return v;
  }
  if (ti.helper) {  // GoUint / GoStruct helpers (ptype_amd.gobtypes)
    py::tuple t = o.attr("__gob_value__")();
    const std::string tag = t[0].cast<std::string>();
    if (tag == "uint") return gob::Value::Uint(t[1].cast<uint64_t>());
    if (tag == "struct") return struct_from(t[1].cast<std::string>(), t[2]);
    if (tag == "slice") {
      gob::Value v;
      v.kind = gob::kSlice;
      for (auto e : t[1]) v.elems.push_back(to_gob(e));
      v.elem_proto.push_back(to_gob(t[2]));
      return v;
    }
    fail("gob: unknown helper tag " + tag);
  }
  if (py::isinstance<py::int_>(o)) return gob::Value::Int(o.cast<int64_t>());
  if (py::isinstance<py::float_>(o)) return gob::Value::Float(o.cast<double>());
  if (py::isinstance<py::str>(o)) return gob::Value::String(o.cast<std::string>());
  if (py::isinstance<py::bytes>(o)) return gob::Value::Bytes(o.cast<std::string>());
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    gob::Value v;
    v.kind = gob::kSlice;
    for (auto e : o) v.elems.push_back(to_gob(e));
    if (v.elems.empty()) v.elem_proto.push_back(gob::Value::Int(0));
    return v;
  }
  if (py::isinstance<py::dict>(o)) {
    gob::Value v;
    v.kind = gob::kMap;
    for (auto kv : o.cast<py::dict>()) v.entries.emplace_back(to_gob(kv.first), to_gob(kv.second));
    if (v.entries.empty()) {
      v.key_proto.push_back(gob::Value::String(""));
      v.elem_proto.push_back(gob::Value::Int(0));
    }
    return v;
  }
  fail("gob: cannot encode Python type " + py::str(py::type::handle_of(o)).cast<std::string>());
}

static py::object from_gob(const gob::Value& v) {
  switch (v.kind) {
    case gob::kNil: return py::none();
    case gob::kBool: return py::bool_(v.b);
    case gob::kInt: return py::int_(v.i);
    case gob::kUint: return py::int_(v.u);
    case gob::kFloat: return py::float_(v.f);
    case gob::kString: return py::str(v.s);
    case gob::kBytes: return py::bytes(v.s);
    case gob::kSlice: {
      py::list l;
      for (const auto& e : v.elems) l.append(from_gob(e));
      return l;
    }
    case gob::kMap: {
      py::dict d;
      for (const auto& kv : v.entries) d[from_gob(kv.first)] = from_gob(kv.second);
      return d;
    }
    case gob::kStruct: {
      py::list pairs;
      for (const auto& f : v.fields) pairs.append(py::make_tuple(f.first, from_gob(f.second)));
      return py::module_::import("ptype_amd.gobtypes").attr("GoStruct")(v.type_name, pairs);
    }
  }
  return py::none();
}

// ---------------------------------------------------------------- helpers
template <class T>
static void bind_channel(py::module_& m, const char* name, std::function<py::object(const T&)> conv,
                         std::function<T(py::handle)> back) {
  py::class_<Channel<T>, std::shared_ptr<Channel<T>>>(m, name)
      .def(py::init<size_t>(), py::arg("cap") = 0)
      .def(
          "recv",
          [conv](Channel<T>& c, double timeout) -> py::object {
            std::optional<T> v;
            {
              py::gil_scoped_release nogil;
              v = c.recv(timeout < 0 ? -1 : (int64_t)(timeout * 1000));
            }
            if (!v) return py::none();
            return conv(*v);
          },
          py::arg("timeout") = -1.0)
      .def(
          "send",
          [back](Channel<T>& c, py::handle v, std::shared_ptr<Context> ctx) {
            T x = back(v);
            py::gil_scoped_release nogil;
            return c.send(std::move(x), ctx);
          },
          py::arg("value"), py::arg("ctx") = nullptr)
      .def("try_send", [back](Channel<T>& c, py::handle v) { return c.try_send(back(v)); })
      .def("close", &Channel<T>::close)
      .def_property_readonly("closed", &Channel<T>::closed)
      .def("__len__", &Channel<T>::size);
}

static std::vector<OpOption> opts_from(py::args a) {
  std::vector<OpOption> v;
  for (auto o : a) v.push_back(o.cast<OpOption>());
  return v;
}

// A device-backed net/rpc method: gob args -> 32-B MsgRecord -> GPU actor.
static RpcHandler device_handler(uintptr_t fn, uintptr_t ctx, int method, uint32_t actor,
                                 std::vector<std::string> fields, std::string actor_field) {
  auto submit = (DeviceSubmitFn)fn;
  return [submit, ctx, method, actor, fields, actor_field](const gob::Value& args) -> gob::Value {
    const MsgRecord m = encode_device_call(args, method, actor, fields, actor_field);
    ReplyRecord r{};
    if (submit((void*)ctx, &m, &r, 1) != 0) fail(Errc::kRpc, "device dispatcher unavailable");
    RpcOutcome o = device_outcome(r);
    if (!o.ok()) fail(o.code, o.error);
    return o.reply;
  };
}

PYBIND11_MODULE(_core, m) {
  m.doc() = "ptype_amd host control plane: config, Raft/MVCC member, registry, KV store, net/rpc, balancer";

  // errors (sentinels of the reference mapped to classes)
  g_err_base = py::reinterpret_borrow<py::object>(PyExc_RuntimeError);
  g_err_base = py::object(py::reinterpret_steal<py::object>(PyErr_NewException("ptype_amd._core.PtypeError", PyExc_RuntimeError, nullptr)));
  auto mk = [&](const char* n) {
    return py::reinterpret_steal<py::object>(
        PyErr_NewException((std::string("ptype_amd._core.") + n).c_str(), g_err_base.ptr(), nullptr));
  };
  g_err_nokey = mk("NoKeyError");
  g_err_noclient = mk("NoClientAvailableError");
  g_err_learner = mk("LearnerNotReadyError");
  g_err_timeout = mk("TimeoutError");
  g_err_canceled = mk("CanceledError");
  g_err_rpc = mk("RpcError");
  g_err_shutdown = mk("ShutdownError");
  g_err_config = mk("ConfigError");
  g_err_unavail = mk("UnavailableError");
  g_err_member = mk("MemberError");
  m.attr("PtypeError") = g_err_base;
  m.attr("NoKeyError") = g_err_nokey;
  m.attr("NoClientAvailableError") = g_err_noclient;
  m.attr("LearnerNotReadyError") = g_err_learner;
  m.attr("TimeoutError") = g_err_timeout;
  m.attr("CanceledError") = g_err_canceled;
  m.attr("RpcError") = g_err_rpc;
  m.attr("ShutdownError") = g_err_shutdown;
  m.attr("ConfigError") = g_err_config;
  m.attr("UnavailableError") = g_err_unavail;
  m.attr("MemberError") = g_err_member;
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const Error& e) {
      translate(e);
    }
  });

  // logging
  py::enum_<LogLevel>(m, "LogLevel")
      .value("DEBUG", LogLevel::kDebug)
      .value("INFO", LogLevel::kInfo)
      .value("WARN", LogLevel::kWarn)
      .value("ERROR", LogLevel::kError)
      .value("OFF", LogLevel::kOff);
  m.def("log_set_level", &log_set_level);
  m.def("log_level", &log_level);
  m.def("log_recent", &log_recent, py::arg("n") = 100);
  m.def("log", [](LogLevel lv, const std::string& msg) { log_write(lv, msg); });

  // context
  py::class_<Context, std::shared_ptr<Context>>(m, "Context")
      .def_static("background", &Context::background)
      .def_static("with_cancel", &Context::with_cancel, py::arg("parent") = nullptr)
      .def_static("with_timeout", &Context::with_timeout, py::arg("parent"), py::arg("ms"))
      .def("cancel", &Context::cancel)
      .def("done", &Context::done)
      .def("wait", &Context::wait, py::arg("ms") = -1, py::call_guard<py::gil_scoped_release>())
      .def("err", &Context::err);

  // util
  m.def("path_join", [](py::args a) {
    std::vector<std::string> v;
    for (auto x : a) v.push_back(x.cast<std::string>());
    return path_join(v);
  });
  m.def("fnv1a32", &fnv1a32);
  m.def("fnv1a64", &fnv1a64);
  m.def("first_nonloopback_ipv4", &first_nonloopback_ipv4);
  m.def("get_ip", &get_ip);
  m.def("yaml_to_json", [](const std::string& text) {
    std::function<std::string(const YNode&)> dump = [&](const YNode& n) -> std::string {
      switch (n.kind) {
        case YNode::kNull: return "null";
        case YNode::kScalar: {
          if (!n.quoted) {
            if (n.is_null()) return "null";
            bool b;
            if (n.is_bool(&b)) return b ? "true" : "false";
            if (n.is_float()) return n.scalar;
          }
          return json_quote(n.scalar);
        }
        case YNode::kSeq: {
          std::string o = "[";
          for (size_t i = 0; i < n.seq.size(); ++i) o += (i ? "," : "") + dump(n.seq[i]);
          return o + "]";
        }
        case YNode::kMap: {
          std::string o = "{";
          for (size_t i = 0; i < n.map.size(); ++i)
            o += (i ? "," : "") + json_quote(n.map[i].first) + ":" + dump(n.map[i].second);
          return o + "}";
        }
      }
      return "null";
    };
    return dump(yaml_parse(text));
  });

  // ---------------------------------------------------------------- config
  py::class_<GpuConfig>(m, "GpuConfig")
      .def(py::init<>())
      .def_readwrite("device", &GpuConfig::device)
      .def_readwrite("ring", &GpuConfig::ring)
      .def_readwrite("actors", &GpuConfig::actors)
      .def_readwrite("idle_ms", &GpuConfig::idle_ms)
      .def_readwrite("delay_us", &GpuConfig::delay_us)
      .def_readwrite("max_batch", &GpuConfig::max_batch)
      .def_readwrite("world", &GpuConfig::world)
      .def_readwrite("backend", &GpuConfig::backend)
      .def_readwrite("cpu", &GpuConfig::cpu)
      .def_readwrite("mailbox_shards", &GpuConfig::mailbox_shards)
      .def_readwrite("mailbox_slots", &GpuConfig::mailbox_slots)
      .def_readwrite("elastic", &GpuConfig::elastic)
      .def_readwrite("delivery", &GpuConfig::delivery)
      .def_readwrite("comm", &GpuConfig::comm)
      .def_readwrite("form_group", &GpuConfig::form_group)
      .def_readwrite("native_group", &GpuConfig::native_group)
      .def_readwrite("tune", &GpuConfig::tune)
      .def_readwrite("group_timeout_s", &GpuConfig::group_timeout_s)
      .def_readwrite("grace_s", &GpuConfig::grace_s)
      .def_readwrite("send_timeout_s", &GpuConfig::send_timeout_s)
      .def_readwrite("replicate_every", &GpuConfig::replicate_every)
      .def_readwrite("watch", &GpuConfig::watch);
  py::class_<MemberConfig, std::shared_ptr<MemberConfig>>(m, "MemberConfig")
      .def(py::init<>())
      .def_readwrite("name", &MemberConfig::name)
      .def_readwrite("dir", &MemberConfig::dir)
      .def_readwrite("lpurls", &MemberConfig::lpurls)
      .def_readwrite("lcurls", &MemberConfig::lcurls)
      .def_readwrite("apurls", &MemberConfig::apurls)
      .def_readwrite("acurls", &MemberConfig::acurls)
      .def_readwrite("initial_cluster", &MemberConfig::initial_cluster)
      .def_readwrite("initial_cluster_token", &MemberConfig::initial_cluster_token)
      .def_readwrite("cluster_state", &MemberConfig::cluster_state)
      .def_readwrite("strict_reconfig_check", &MemberConfig::strict_reconfig_check)
      .def_readwrite("logger", &MemberConfig::logger)
      .def_readwrite("heartbeat_ms", &MemberConfig::heartbeat_ms)
      .def_readwrite("election_ms", &MemberConfig::election_ms)
      .def_readwrite("snapshot_count", &MemberConfig::snapshot_count)
      .def_readwrite("unsafe_no_fsync", &MemberConfig::unsafe_no_fsync)
      .def("validate", &MemberConfig::validate)
      .def("effective_initial_cluster", &MemberConfig::effective_initial_cluster)
      .def_static("from_file", &MemberConfig::from_file);
  py::class_<Config>(m, "Config")
      .def(py::init<>())
      .def_readwrite("service_name", &Config::service_name)
      .def_readwrite("node_name", &Config::node_name)
      .def_readwrite("port", &Config::port)
      .def_readwrite("etcd_config_file", &Config::etcd_config_file)
      .def_readwrite("initial_cluster_client_urls", &Config::initial_cluster_client_urls)
      .def_readwrite("debug", &Config::debug)
      .def_readwrite("has_gpu", &Config::has_gpu)
      .def_readwrite("gpu", &Config::gpu)
      .def_readwrite("member", &Config::member);
  m.def("config_from_file", &config_from_file);
  m.def("config_from_yaml", &config_from_yaml);

  // ---------------------------------------------------------------- kv types
  py::class_<KeyValue>(m, "KeyValue")
      .def_readonly("key", &KeyValue::key)
      .def_property_readonly("value", [](const KeyValue& k) { return py::bytes(k.value); })
      .def_readonly("create_revision", &KeyValue::create_revision)
      .def_readonly("mod_revision", &KeyValue::mod_revision)
      .def_readonly("version", &KeyValue::version)
      .def_readonly("lease", &KeyValue::lease);
  py::class_<RangeOpts>(m, "RangeOpts")
      .def(py::init<>())
      .def_readwrite("end", &RangeOpts::end)
      .def_readwrite("limit", &RangeOpts::limit)
      .def_readwrite("rev", &RangeOpts::rev)
      .def_readwrite("sort_target", &RangeOpts::sort_target)
      .def_readwrite("sort_order", &RangeOpts::sort_order)
      .def_readwrite("serializable", &RangeOpts::serializable)
      .def_readwrite("keys_only", &RangeOpts::keys_only)
      .def_readwrite("count_only", &RangeOpts::count_only);
  py::class_<RangeResult>(m, "RangeResult")
      .def_readonly("kvs", &RangeResult::kvs)
      .def_readonly("count", &RangeResult::count)
      .def_readonly("more", &RangeResult::more)
      .def_readonly("rev", &RangeResult::rev);
  py::class_<Event>(m, "Event")
      .def_property_readonly("type", [](const Event& e) { return e.type == Event::kPut ? "PUT" : "DELETE"; })
      .def_readonly("kv", &Event::kv);
  py::class_<WatchResponse>(m, "WatchResponse")
      .def_readonly("events", &WatchResponse::events)
      .def_readonly("revision", &WatchResponse::revision)
      .def_readonly("canceled", &WatchResponse::canceled)
      .def_readonly("err", &WatchResponse::err);
  py::class_<MemberInfo>(m, "MemberInfo")
      .def_readonly("id", &MemberInfo::id)
      .def_readonly("name", &MemberInfo::name)
      .def_readonly("peer_urls", &MemberInfo::peer_urls)
      .def_readonly("client_urls", &MemberInfo::client_urls)
      .def_readonly("is_learner", &MemberInfo::is_learner)
      .def("__repr__", [](const MemberInfo& mi) {
        return "Member(id=" + std::to_string(mi.id) + ", name=" + mi.name + ", learner=" + (mi.is_learner ? "1" : "0") + ")";
      });
  py::class_<StatusInfo>(m, "StatusInfo")
      .def_readonly("id", &StatusInfo::id)
      .def_readonly("leader", &StatusInfo::leader)
      .def_readonly("term", &StatusInfo::term)
      .def_readonly("commit", &StatusInfo::commit)
      .def_readonly("applied", &StatusInfo::applied)
      .def_readonly("revision", &StatusInfo::revision)
      .def_readonly("is_learner", &StatusInfo::is_learner);
  py::class_<LeaseInfo>(m, "LeaseInfo").def_readonly("id", &LeaseInfo::id).def_readonly("ttl", &LeaseInfo::ttl);
  m.def("prefix_range_end", &prefix_range_end);

  // channels
  py::class_<Node>(m, "Node")
      .def(py::init<>())
      .def(py::init([](std::string a, int64_t p) { return Node{std::move(a), p}; }), py::arg("address"), py::arg("port"))
      .def_readwrite("address", &Node::address)
      .def_readwrite("port", &Node::port)
      .def("__eq__", [](const Node& a, const Node& b) { return a == b; })
      .def("__hash__", [](const Node& a) { return std::hash<std::string>()(a.address + ":" + std::to_string(a.port)); })
      .def("__repr__", [](const Node& n) { return "Node(address='" + n.address + "', port=" + std::to_string(n.port) + ")"; });
  bind_channel<std::vector<Node>>(
      m, "NodesChannel", [](const std::vector<Node>& v) { return py::cast(v); },
      [](py::handle h) { return h.cast<std::vector<Node>>(); });
  bind_channel<std::string>(
      m, "ErrChannel", [](const std::string& v) { return py::cast(v); }, [](py::handle h) { return h.cast<std::string>(); });
  bind_channel<int>(
      m, "IntChannel", [](const int& v) { return py::cast(v); }, [](py::handle h) { return h.cast<int>(); });
  bind_channel<int64_t>(
      m, "TTLChannel", [](const int64_t& v) { return py::cast(v); }, [](py::handle h) { return h.cast<int64_t>(); });
  bind_channel<WatchResponse>(
      m, "WatchChannel", [](const WatchResponse& v) { return py::cast(v); },
      [](py::handle h) { return h.cast<WatchResponse>(); });

  // ---------------------------------------------------------------- member + client
  py::class_<Member, std::shared_ptr<Member>>(m, "Member")
      .def(py::init<const MemberConfig&>())
      .def("start", &Member::start, py::call_guard<py::gil_scoped_release>())
      .def("wait_ready", &Member::wait_ready, py::arg("timeout_ms") = -1, py::call_guard<py::gil_scoped_release>())
      .def("close", &Member::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("id", &Member::id)
      .def_property_readonly("name", &Member::name)
      .def_property_readonly("closed", &Member::closed)
      .def("is_learner", &Member::is_learner)
      .def("leader", &Member::leader)
      .def("status", &Member::status)
      .def("client_ports", &Member::client_ports)
      .def("member_list", &Member::member_list)
      .def("lease_list", &Member::lease_list)
      .def_property_readonly("reads_served", &Member::reads_served);

  py::class_<KvClient, std::shared_ptr<KvClient>>(m, "KvClient")
      .def(py::init<std::vector<std::string>, int64_t>(), py::arg("endpoints"), py::arg("dial_timeout_ms") = 5000)
      .def("close", &KvClient::close, py::call_guard<py::gil_scoped_release>())
      .def("get", &KvClient::get, py::arg("key"), py::arg("opts") = RangeOpts(), py::arg("timeout_ms") = 5000,
           py::call_guard<py::gil_scoped_release>())
      .def(
          "put",
          [](KvClient& c, const std::string& k, py::bytes v, int64_t lease) {
            std::string s = v;
            py::gil_scoped_release nogil;
            return c.put(k, s, lease);
          },
          py::arg("key"), py::arg("value"), py::arg("lease") = 0)
      .def(
          "delete",
          [](KvClient& c, const std::string& k, const std::string& end) {
            py::gil_scoped_release nogil;
            int64_t d = 0;
            c.del(k, end, &d);
            return d;
          },
          py::arg("key"), py::arg("end") = "")
      .def(
          "grant",
          [](KvClient& c, int64_t ttl) {
            py::gil_scoped_release nogil;
            int64_t t = 0;
            int64_t id = c.grant(ttl, &t);
            return std::make_pair(id, t);
          },
          py::arg("ttl"))
      .def("revoke", &KvClient::revoke, py::arg("id"), py::arg("timeout_ms") = 5000,
           py::call_guard<py::gil_scoped_release>())
      .def("keepalive_once", &KvClient::keepalive_once, py::arg("id"), py::arg("timeout_ms") = 5000,
           py::call_guard<py::gil_scoped_release>())
      .def("keepalive", &KvClient::keepalive, py::arg("ctx"), py::arg("id"), py::call_guard<py::gil_scoped_release>())
      .def("time_to_live_ms", &KvClient::time_to_live_ms, py::arg("id"), py::arg("timeout_ms") = 5000,
           py::call_guard<py::gil_scoped_release>())
      .def("compact", &KvClient::compact, py::arg("rev"), py::arg("timeout_ms") = 5000,
           py::call_guard<py::gil_scoped_release>())
      .def("member_list", &KvClient::member_list, py::arg("timeout_ms") = 5000, py::call_guard<py::gil_scoped_release>())
      .def(
          "member_add",
          [](KvClient& c, std::vector<std::string> urls, bool learner) {
            py::gil_scoped_release nogil;
            std::vector<MemberInfo> ms;
            MemberInfo mi = c.member_add(urls, learner, &ms);
            return std::make_pair(mi, ms);
          },
          py::arg("peer_urls"), py::arg("learner") = true)
      .def("member_promote", &KvClient::member_promote, py::arg("id"), py::arg("timeout_ms") = 10000,
           py::call_guard<py::gil_scoped_release>())
      .def("member_remove", &KvClient::member_remove, py::arg("id"), py::arg("timeout_ms") = 10000,
           py::call_guard<py::gil_scoped_release>())
      .def("status", &KvClient::status, py::arg("timeout_ms") = 5000, py::call_guard<py::gil_scoped_release>())
      .def("watch", &KvClient::watch, py::arg("ctx"), py::arg("key"), py::arg("end") = "", py::arg("start_rev") = 0,
           py::call_guard<py::gil_scoped_release>());

  // the GPU registry mirror's compiled control side (follower.hpp)
  py::class_<RegistryFollower, std::shared_ptr<RegistryFollower>>(m, "RegistryFollower")
      .def(py::init([](std::shared_ptr<KvClient> kv, const std::string& prefix, int64_t ttl_ms, int64_t grace_ms,
                       double relist_s, bool watch) {
             py::gil_scoped_release nogil;
             return std::make_shared<RegistryFollower>(std::move(kv), prefix, ttl_ms, grace_ms, relist_s, watch);
           }),
           py::arg("kv"), py::arg("prefix"), py::arg("ttl_ms"), py::arg("grace_ms"), py::arg("relist_s"),
           py::arg("watch") = true)
      .def("quiet", &RegistryFollower::quiet, py::arg("now_ms"))
      .def(
          "take",
          [](RegistryFollower& f, int64_t now_ms) {
            bool sweep = false;
            int64_t changed = 0;
            std::vector<MirrorOp> ops;
            {
              py::gil_scoped_release nogil;
              ops = f.take(now_ms, &sweep, &changed);
            }
            py::list out;
            for (auto& op : ops) {  // (kind, key, rank, deadline, ids int64[n], mbox int32[n] or None)
              py::array_t<int64_t> ids((py::ssize_t)op.ids.size());
              std::copy(op.ids.begin(), op.ids.end(), ids.mutable_data());
              py::object mb = py::none();
              if (op.kind == MirrorOp::kUpsert) {
                py::array_t<int32_t> a((py::ssize_t)op.mbox.size());
                std::copy(op.mbox.begin(), op.mbox.end(), a.mutable_data());
                mb = a;
              }
              out.append(py::make_tuple((int)op.kind, op.key, op.rank, op.deadline_ms, ids, mb));
            }
            return py::make_tuple(out, sweep, changed);
          },
          py::arg("now_ms"), "apply what is queued: ([(kind, key, rank, deadline, ids, mbox)], sweep, changed)")
      .def("set_generation", &RegistryFollower::set_generation, py::arg("gen"))
      .def("shards", &RegistryFollower::shards, "applied shards: [(key, record JSON, deadline ms)]")
      .def_property_readonly("actors", &RegistryFollower::actors)
      .def_property_readonly("version", &RegistryFollower::version)
      .def_property_readonly("applies", &RegistryFollower::applies)
      .def_property_readonly("relists", &RegistryFollower::relists)
      .def_property_readonly("events", &RegistryFollower::events)
      .def("close", &RegistryFollower::close, py::call_guard<py::gil_scoped_release>());
  py::class_<ShardLease, std::shared_ptr<ShardLease>>(m, "ShardLease")
      .def(py::init([](std::shared_ptr<KvClient> kv, const std::string& key, const std::string& record, int64_t ttl_s) {
             py::gil_scoped_release nogil;
             return std::make_shared<ShardLease>(std::move(kv), key, record, ttl_s);
           }),
           py::arg("kv"), py::arg("key"), py::arg("record"), py::arg("ttl_s"))
      .def("update", &ShardLease::update, py::arg("record"), py::call_guard<py::gil_scoped_release>())
      .def("stop_keepalive", &ShardLease::stop_keepalive)
      .def("close", &ShardLease::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("record", &ShardLease::record)
      .def_property_readonly("lease", &ShardLease::lease);

  // ---------------------------------------------------------------- registry / store
  py::class_<Registry, std::shared_ptr<Registry>>(m, "Registry");
  py::class_<EtcdRegistry, Registry, std::shared_ptr<EtcdRegistry>>(m, "EtcdRegistry")
      .def(py::init([](std::vector<std::string> eps) {
             return std::make_shared<EtcdRegistry>(std::make_shared<KvClient>(eps, 5000));
           }),
           py::arg("endpoints"))
      .def("register", &EtcdRegistry::register_node, py::arg("ctx"), py::arg("service"), py::arg("node"),
           py::arg("host"), py::arg("port"), py::call_guard<py::gil_scoped_release>())
      .def("services", &EtcdRegistry::services, py::arg("ctx"), py::call_guard<py::gil_scoped_release>())
      .def("watch_service", &EtcdRegistry::watch_service, py::arg("ctx"), py::arg("service"),
           py::call_guard<py::gil_scoped_release>())
      .def("nodes", &EtcdRegistry::nodes, py::arg("ctx"), py::arg("service"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("kv", &EtcdRegistry::kv_ptr)
      .def("close", &EtcdRegistry::close, py::call_guard<py::gil_scoped_release>());
  m.def("etcd_key", [](py::args a) {
    std::vector<std::string> v;
    for (auto x : a) v.push_back(x.cast<std::string>());
    return etcd_key(v);
  });
  m.def("node_json", &node_json);
  m.def("node_from_json", &node_from_json);

  py::class_<OpOption>(m, "OpOption")
      .def_property_readonly("kind", [](const OpOption& o) { return (int)o.kind; })
      .def_readonly("n", &OpOption::n)
      .def_readonly("s", &OpOption::s);
  m.def("with_prefix", [] { return OpOption{OpOption::kPrefix}; });
  m.def("with_limit", [](int64_t n) { OpOption o{OpOption::kLimit}; o.n = n; return o; });
  m.def("with_rev", [](int64_t n) { OpOption o{OpOption::kRev}; o.n = n; return o; });
  m.def("with_range", [](std::string e) { OpOption o{OpOption::kRange}; o.s = e; return o; });
  m.def("with_from_key", [] { return OpOption{OpOption::kFromKey}; });
  m.def("with_serializable", [] { return OpOption{OpOption::kSerializable}; });
  m.def("with_keys_only", [] { return OpOption{OpOption::kKeysOnly}; });
  m.def("with_count_only", [] { return OpOption{OpOption::kCountOnly}; });
  m.def("with_lease", [](int64_t id) { OpOption o{OpOption::kLease}; o.n = id; return o; });
  m.def("with_sort", [](int target, int order) {
    OpOption o{OpOption::kSort};
    o.target = target;
    o.order = order;
    return o;
  });
  m.def("resolve_opts", [](std::string key, py::args a) {
    RangeOpts o = resolve_opts(&key, opts_from(a));
    return std::make_pair(key, o);
  });

  py::class_<KVStore, std::shared_ptr<KVStore>>(m, "KVStore")
      .def(py::init([](std::vector<std::string> eps) { return std::make_shared<KVStore>(std::make_shared<KvClient>(eps, 5000)); }),
           py::arg("endpoints"))
      .def("get", [](KVStore& s, Ctx ctx, const std::string& key, py::args a) {
        auto o = opts_from(a);
        py::gil_scoped_release nogil;
        return s.get(ctx, key, o);
      })
      .def("put", [](KVStore& s, Ctx ctx, const std::string& key, const std::string& val, py::args a) {
        auto o = opts_from(a);
        py::gil_scoped_release nogil;
        s.put(ctx, key, val, o);
      })
      .def("delete", [](KVStore& s, Ctx ctx, const std::string& key, py::args a) {
        auto o = opts_from(a);
        py::gil_scoped_release nogil;
        s.del(ctx, key, o);
      })
      .def("close", [](KVStore& s) { s.kv().close(); }, py::call_guard<py::gil_scoped_release>());

  // ---------------------------------------------------------------- rpc
  py::class_<ConnConfig>(m, "ConnConfig")
      .def(py::init([](int max_connections, double initial_node_timeout, double debounce_time, int retries,
                       bool allow_local) {
             ConnConfig c;
             c.max_connections = max_connections;
             c.initial_node_timeout_ms = (int64_t)(initial_node_timeout * 1000);
             c.debounce_ms = (int64_t)(debounce_time * 1000);
             c.retries = retries;
             c.allow_local = allow_local;
             return c;
           }),
           py::arg("max_connections") = 3, py::arg("initial_node_timeout") = 5.0, py::arg("debounce_time") = 3.0,
           py::arg("retries") = 2, py::arg("allow_local") = true)
      .def_readwrite("max_connections", &ConnConfig::max_connections)
      .def_property(
          "initial_node_timeout", [](const ConnConfig& c) { return c.initial_node_timeout_ms / 1000.0; },
          [](ConnConfig& c, double v) { c.initial_node_timeout_ms = (int64_t)(v * 1000); })
      .def_property(
          "debounce_time", [](const ConnConfig& c) { return c.debounce_ms / 1000.0; },
          [](ConnConfig& c, double v) { c.debounce_ms = (int64_t)(v * 1000); })
      .def_readwrite("retries", &ConnConfig::retries)
      .def_readwrite("allow_local", &ConnConfig::allow_local)
      .def("__eq__", [](const ConnConfig& a, const ConnConfig& b) {
        return a.max_connections == b.max_connections && a.initial_node_timeout_ms == b.initial_node_timeout_ms &&
               a.debounce_ms == b.debounce_ms && a.retries == b.retries;
      });
  m.def("default_conn_config", &default_conn_config);

  py::class_<RpcServer, std::shared_ptr<RpcServer>>(m, "RpcServer")
      .def(py::init<>())
      .def("register_method",
           [](std::shared_ptr<RpcServer> s, const std::string& name, py::function fn) {
             auto holder = std::shared_ptr<py::function>(new py::function(fn), [](py::function* p) {
               py::gil_scoped_acquire gil;  // a dispatch thread may drop the last reference
               delete p;
             });
             s->register_method(name, [holder](const gob::Value& args) -> gob::Value {
               py::gil_scoped_acquire gil;
               try {
                 return to_gob((*holder)(from_gob(args)));
               } catch (py::error_already_set& e) {
                 std::string msg = py::str(e.value()).cast<std::string>();
                 fail(Errc::kRpc, msg);
               }
             });
           })
      .def("register_device_method",
           [](std::shared_ptr<RpcServer> s, const std::string& name, uintptr_t fn, uintptr_t ctx, int method,
              uint32_t actor, std::vector<std::string> fields, std::string actor_field) {
             s->register_method(name, device_handler(fn, ctx, method, actor, fields, actor_field));
           },
           py::arg("name"), py::arg("submit_fn"), py::arg("submit_ctx"), py::arg("method"), py::arg("actor") = 0,
           py::arg("fields") = std::vector<std::string>{}, py::arg("actor_field") = "")
      .def("set_shm_segment", &RpcServer::set_shm_segment, py::arg("name"))
      .def("register_device_batch", &RpcServer::register_device_batch, py::arg("name"), py::arg("batch_fn"),
           py::arg("batch_ctx"), py::arg("fields") = std::vector<std::string>{}, py::arg("actor_field") = "",
           py::arg("max_batch") = (size_t)(1 << 16))
      .def_property_readonly("batches", &RpcServer::batches)
      .def_property_readonly("batched_calls", &RpcServer::batched_calls)
      .def("has_service", &RpcServer::has_service)
      .def(
          "listen",
          [](std::shared_ptr<RpcServer> s, const std::string& host, int port, bool local) {
            int p;
            {
              py::gil_scoped_release nogil;
              p = s->listen(host, port);
            }
            if (local) local_server_register(p, s);
            return p;
          },
          py::arg("host") = "0.0.0.0", py::arg("port") = 0, py::arg("local") = true)
      .def("close",
           [](std::shared_ptr<RpcServer> s) {
             local_server_unregister(s->port());
             py::gil_scoped_release nogil;
             s->close();
           })
      .def_property_readonly("port", &RpcServer::port)
      .def("call_counts", &RpcServer::call_counts)
      .def("debug_page", &RpcServer::debug_page)
      .def("set_debug_handler",
           [](std::shared_ptr<RpcServer> s, const std::string& path, py::object fn) {
             if (fn.is_none()) {
               s->set_debug_handler(path, nullptr);
               return;
             }
             auto holder = std::shared_ptr<py::object>(new py::object(fn), [](py::object* p) {
               py::gil_scoped_acquire gil;  // the last owner may be a server thread
               delete p;
             });
             s->set_debug_handler(path, [holder]() -> std::string {
               py::gil_scoped_acquire gil;
               try {
                 return (*holder)().cast<std::string>();
               } catch (py::error_already_set& e) {
                 throw std::runtime_error(py::str(e.value()).cast<std::string>());
               }
             });
           })
      .def("dispatch", [](RpcServer& s, const std::string& sm, py::object args) {
        gob::Value a = to_gob(args);
        RpcOutcome o;
        {
          py::gil_scoped_release nogil;
          o = s.dispatch(sm, a);
        }
        if (!o.ok()) fail(o.code, o.error);
        return from_gob(o.reply);
      });

  py::class_<RpcConn, std::shared_ptr<RpcConn>>(m, "RpcConn")
      .def_property_readonly("target", &RpcConn::target)
      .def_property_readonly("transport",
                             [](RpcConn& c) -> std::string {
                               if (dynamic_cast<ShmRpcConn*>(&c)) return "shm";
                               if (dynamic_cast<LocalRpcConn*>(&c)) return "local";
                               return "tcp";
                             })
      .def_property_readonly("ring_placement",
                             [](RpcConn& c) -> py::object {
                               if (auto* s = dynamic_cast<ShmRpcConn*>(&c)) return py::str(s->ring_placement());
                               return py::none();
                             })
      .def("call",
           [](RpcConn& c, const std::string& method, py::object args) {
             gob::Value a = to_gob(args);
             RpcOutcome o;
             {
               py::gil_scoped_release nogil;
               o = c.call(method, a);
             }
             if (!o.ok()) fail(o.code, o.error);
             return from_gob(o.reply);
           })
      .def(
          "call_many",
          [](RpcConn& c, const std::string& method, py::list args, double timeout) {
            // every call pipelined on the connection (Go's client.Go in a loop), then all replies
            std::vector<gob::Value> in;
            in.reserve(args.size());
            for (auto a : args) in.push_back(to_gob(py::reinterpret_borrow<py::object>(a)));
            std::vector<RpcOutcome> out(in.size());
            {
              py::gil_scoped_release nogil;
              std::mutex mu;
              std::condition_variable cv;
              size_t left = in.size();
              for (size_t i = 0; i < in.size(); ++i)
                c.go(method, in[i], [&, i](RpcOutcome o) {
                  std::lock_guard<std::mutex> g(mu);
                  out[i] = std::move(o);
                  if (--left == 0) cv.notify_all();
                });
              std::unique_lock<std::mutex> lk(mu);
              if (!cv.wait_for(lk, std::chrono::duration<double>(timeout), [&] { return left == 0; }))
                fail(Errc::kTimeout, "call_many: replies outstanding after the timeout");
            }
            py::list res;
            for (auto& o : out) res.append(o.ok() ? from_gob(o.reply) : py::object(py::str("error: " + o.error)));
            return res;
          },
          py::arg("method"), py::arg("args"), py::arg("timeout") = 60.0)
      .def("close", &RpcConn::close);
  // A raw handle on another process's dispatcher segment (by name): device calls
  // straight into the rings that process's GPU polls -- used to time remote calls
  // between the GPUs of a node (bench.py) without a net/rpc server in the way.
  struct ShmClient {
    std::shared_ptr<ShmSegment> seg;
    std::shared_ptr<DevRingMap> devmap;
    ShmView view;
  };
  py::class_<ShmClient, std::shared_ptr<ShmClient>>(m, "ShmClient")
      .def(py::init([](const std::string& name) {
             auto seg = ShmSegment::attach(name);
             if (!seg) fail(Errc::kUnavailable, "no dispatcher segment " + name);
             auto c = std::make_shared<ShmClient>();
             c->view = shm_attach_view(seg, &c->devmap);
             c->seg = std::move(seg);
             return c;
           }),
           py::arg("name"))
      .def_property_readonly("ring_placement",
                             [](const ShmClient& c) { return std::string(c.view.bar ? "device" : "host"); })
      .def(
          "call",
          [](ShmClient& c, int method, uint32_t actor, int64_t a0, int64_t a1, int64_t a2, double timeout) {
            MsgRecord m{actor, (uint16_t)method, (uint16_t)kFlagValid, a0, a1, a2};
            ReplyRecord r;
            {
              py::gil_scoped_release nogil;
              r = shm_call(c.view, m, timeout);
            }
            return py::make_tuple(r.value, r.status);
          },
          py::arg("method"), py::arg("actor"), py::arg("a0") = 0, py::arg("a1") = 0, py::arg("a2") = 0,
          py::arg("timeout") = 10.0);
  py::class_<HostDispatcher, std::shared_ptr<HostDispatcher>>(
      m, "HostDispatcher", "CPU stand-in for the GPU dispatcher on a shared-memory segment of its own")
      .def(py::init([](const std::string& name, uint32_t ring) { return std::make_shared<HostDispatcher>(name, ring); }),
           py::arg("name"), py::arg("ring") = 64)
      .def_property_readonly("name", &HostDispatcher::name)
      .def_property_readonly("processed", &HostDispatcher::processed)
      .def_property_readonly("noops", &HostDispatcher::noops);
  // the dma-buf fd hand-off of the cross-process device ring, bound for tests
  py::class_<FdHandoff, std::shared_ptr<FdHandoff>>(m, "FdHandoff")
      .def(py::init([](const std::string& name, int fd) { return std::make_shared<FdHandoff>(name, fd); }),
           py::arg("name"), py::arg("fd"))
      .def_property_readonly("handed", &FdHandoff::handed);
  m.def(
      "fd_receive",
      [](const std::string& name) {
        std::string why;
        int fd;
        {
          py::gil_scoped_release nogil;
          fd = shm_receive_fd(name, &why);
        }
        if (fd < 0) fail(Errc::kUnavailable, "fd hand-off " + name + ": " + why);
        return fd;
      },
      py::arg("name"));
  m.def("host_batch_multiply", []() { return py::make_tuple((uintptr_t)&host_batch_multiply, (uintptr_t)0); },
        "(fn, ctx) of the CPU batch handler twin of the GPU gob bridge (Calculator.Multiply)");
  m.def(
      "dial_http",
      [](const std::string& host, int port, double timeout, bool allow_local) {
        py::gil_scoped_release nogil;
        return dial_node(host, port, (int64_t)(timeout * 1000), allow_local);
      },
      py::arg("host"), py::arg("port"), py::arg("timeout") = 5.0, py::arg("allow_local") = false);

  py::class_<RpcCall, std::shared_ptr<RpcCall>>(m, "RpcCall")
      .def_readonly("service_method", &RpcCall::method)
      .def_property_readonly("reply", [](const RpcCall& c) { return from_gob(c.reply); })
      .def_property_readonly("error", [](const RpcCall& c) -> py::object {
        if (c.error.empty()) return py::none();
        return py::str(c.error);
      })
      .def_readonly("done", &RpcCall::done);
  bind_channel<std::shared_ptr<RpcCall>>(
      m, "CallChannel", [](const std::shared_ptr<RpcCall>& v) { return py::cast(v); },
      [](py::handle h) { return h.cast<std::shared_ptr<RpcCall>>(); });

  py::class_<ConnectionBalancer>(m, "ConnectionBalancer")
      .def(py::init([](std::string local, std::string svc, std::shared_ptr<NodesChan> nodes, ConnConfig cfg) {
             py::gil_scoped_release nogil;
             return new ConnectionBalancer(local, svc, nodes, cfg);
           }),
           py::arg("local_addr"), py::arg("service"), py::arg("nodes"), py::arg("cfg"))
      .def_static("select_nodes", &ConnectionBalancer::select_nodes)
      .def_static("hash_index", &ConnectionBalancer::hash_index)
      .def("selected_nodes", &ConnectionBalancer::selected_nodes)
      .def("client_count", &ConnectionBalancer::client_count)
      .def_property_readonly("errs", &ConnectionBalancer::errs)
      .def_property_readonly("conns_updated", &ConnectionBalancer::conns_updated)
      .def_property_readonly("cfg", &ConnectionBalancer::config)
      .def("get_target", [](ConnectionBalancer& b) -> py::object {
        auto c = b.get();
        if (!c) return py::none();
        return py::str(c->target());
      })
      .def("close", &ConnectionBalancer::close, py::call_guard<py::gil_scoped_release>());

  py::class_<RpcClient, std::shared_ptr<RpcClient>>(m, "RpcClient")
      .def(py::init([](std::string local, std::string svc, std::shared_ptr<NodesChan> nodes, ConnConfig cfg) {
             py::gil_scoped_release nogil;
             return std::make_shared<RpcClient>(local, svc, nodes, cfg);
           }),
           py::arg("local_addr"), py::arg("service"), py::arg("nodes"), py::arg("cfg"))
      .def("call",
           [](RpcClient& c, const std::string& method, py::object args) {
             gob::Value a = to_gob(args);
             gob::Value r;
             {
               py::gil_scoped_release nogil;
               r = c.call(method, a);
             }
             return from_gob(r);
           })
      .def(
          "go",
          [](RpcClient& c, const std::string& method, py::object args,
             std::shared_ptr<Channel<std::shared_ptr<RpcCall>>> done) {
            gob::Value a = to_gob(args);
            py::gil_scoped_release nogil;
            return c.go(method, a, done);
          },
          py::arg("method"), py::arg("args"), py::arg("done") = nullptr)
      .def("close", &RpcClient::close, py::call_guard<py::gil_scoped_release>())
      .def("connection_errs", &RpcClient::connection_errs)
      .def_property_readonly("cfg", &RpcClient::config)
      .def_property_readonly("calls", &RpcClient::calls)
      .def_property_readonly("attempts", &RpcClient::attempts)
      .def("selected_nodes", [](RpcClient& c) { return c.balancer().selected_nodes(); })
      .def_property_readonly("retired_conns", [](RpcClient& c) { return c.balancer().retired_count(); })
      .def_property_readonly("conns_updated", [](RpcClient& c) { return c.balancer().conns_updated(); });

  // ---------------------------------------------------------------- cluster
  py::class_<Cluster, std::shared_ptr<Cluster>>(m, "Cluster")
      .def_static("join", &Cluster::join, py::arg("ctx"), py::arg("cfg"), py::call_guard<py::gil_scoped_release>())
      .def_static("join_existing_cluster", &Cluster::join_existing_cluster, py::call_guard<py::gil_scoped_release>())
      .def_readonly("registry", &Cluster::registry)
      .def_readonly("store", &Cluster::store)
      .def("member_list", &Cluster::member_list, py::arg("ctx"), py::call_guard<py::gil_scoped_release>())
      .def(
          "new_client",
          [](Cluster& c, const std::string& svc, py::object cfg) {
            ConnConfig cc;
            const ConnConfig* p = nullptr;
            if (!cfg.is_none()) {
              cc = cfg.cast<ConnConfig>();
              p = &cc;
            }
            py::gil_scoped_release nogil;
            return c.new_client(svc, p);
          },
          py::arg("service"), py::arg("cfg") = py::none())
      .def("close", &Cluster::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("local_addr", &Cluster::local_addr)
      .def_property_readonly("member_id", [](Cluster& c) { return c.member().id(); })
      .def("member_status", [](Cluster& c) { return c.member().status(); });

  // ---------------------------------------------------------------- data-plane lifecycle (dataplane.hpp)
  py::class_<DataPlane, std::shared_ptr<DataPlane>>(m, "DataPlane",
                                                    "RCCL communicator lifecycle of a service's GPU data plane: "
                                                    "rendezvous through the replicated store, init, abort, "
                                                    "lease-driven membership, next generation")
      .def(py::init([](std::shared_ptr<Cluster> c, const std::string& service, const std::string& me, int device,
                       double timeout_s) {
             return std::make_shared<DataPlane>(c->registry, c->registry->kv_ptr(), service, me, device, timeout_s);
           }),
           py::arg("cluster"), py::arg("service"), py::arg("me"), py::arg("device"), py::arg("timeout_s") = 30.0)
      .def("form", &DataPlane::form, py::arg("gen"), py::arg("members"), py::call_guard<py::gil_scoped_release>())
      .def("set_device", &DataPlane::set_device, py::arg("device"))
      .def_property_readonly("device", &DataPlane::device)
      .def("alive_nodes", &DataPlane::alive_nodes, py::call_guard<py::gil_scoped_release>())
      .def("wait_nodes", &DataPlane::wait_nodes, py::arg("world"), py::call_guard<py::gil_scoped_release>())
      .def("settle", &DataPlane::settle, py::arg("current"), py::arg("grace_s"),
           py::call_guard<py::gil_scoped_release>())
      .def("use_transport", &DataPlane::use_transport, py::arg("ops"), py::arg("cap_bytes"),
           "a DpTransportOps table of the device runtime (IpcComm) instead of RCCL; before the first form()")
      .def_property_readonly("transport", &DataPlane::transport)
      .def(
          "recover",
          [](DataPlane& d, double grace_s) {
            DataPlane::Recovery r;
            {
              py::gil_scoped_release nogil;
              r = d.recover(grace_s);
            }
            py::dict out;
            out["lost"] = r.lost;
            out["members"] = r.members;
            out["blocks"] = r.blocks;
            out["kept_from"] = r.kept_from;
            out["from_replica"] = r.from_replica;
            return out;
          },
          py::arg("grace_s"),
          "abort + settle + form(gen + 1); the new placement: {lost, members, blocks, kept_from, from_replica}")
      .def("placement", &DataPlane::placement, py::arg("members"))
      .def_property_readonly("blocks", &DataPlane::blocks)
      .def("buddy", &DataPlane::buddy, py::arg("node"))
      .def("lost_blocks", &DataPlane::lost_blocks, py::arg("before"), py::arg("after"))
      .def_property_readonly("nodes0", &DataPlane::nodes0)
      .def("replica_blocks", &DataPlane::replica_blocks)
      .def("replicate", &DataPlane::replicate, py::arg("state"), py::arg("bytes"), py::arg("recv"),
           py::arg("recv_bytes"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("replicas", &DataPlane::replicas)
      .def("set_watchdog", &DataPlane::set_watchdog, py::arg("timeout_s"))
      .def("begin_send", &DataPlane::begin_send)
      .def("end_send", &DataPlane::end_send)
      .def("arm", &DataPlane::arm, py::arg("stream"))
      .def_property_readonly("watchdog_failed", &DataPlane::watchdog_failed)
      .def("reset_watchdog", &DataPlane::reset_watchdog)
      .def("fail_generation", &DataPlane::fail_generation, py::arg("why"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("comm_cell", &DataPlane::comm_cell)
      .def("engine_comm_ref", &DataPlane::engine_comm_ref)
      .def("async_error", &DataPlane::async_error)
      .def("abort", &DataPlane::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &DataPlane::aborted)
      .def("allreduce_max", &DataPlane::allreduce_max, py::arg("values"), py::call_guard<py::gil_scoped_release>())
      .def("allreduce_max_dev", &DataPlane::allreduce_max_dev, py::arg("dev"), py::arg("n"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("sendrecv", &DataPlane::sendrecv, py::arg("send"), py::arg("send_bytes"), py::arg("dst"), py::arg("recv"),
           py::arg("recv_bytes"), py::arg("src"), py::call_guard<py::gil_scoped_release>())
      .def("barrier", &DataPlane::barrier, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("comm", &DataPlane::comm)
      .def_property_readonly("rank", &DataPlane::rank)
      .def_property_readonly("size", &DataPlane::size)
      .def_property_readonly("gen", &DataPlane::gen)
      .def_property_readonly("members", &DataPlane::members)
      .def_property_readonly("me", &DataPlane::me)
      .def_static("available", &DataPlane::available);

  // ---------------------------------------------------------------- gob (golden tests)
  m.def("gob_encode", [](py::list values) {
    gob::Encoder enc;
    std::string out;
    for (auto v : values) enc.encode(to_gob(v), &out);
    return py::bytes(out);
  });
  m.def("gob_decode", [](py::bytes data) {
    std::string s = data;
    size_t pos = 0;
    gob::Decoder dec([&](char* p, size_t n) {
      if (pos + n > s.size()) return false;
      memcpy(p, s.data() + pos, n);
      pos += n;
      return true;
    });
    py::list out;
    gob::Value v;
    while (dec.decode(&v)) out.append(from_gob(v));
    return out;
  });

  // record layout constants shared with _hip
  m.attr("MSG_RECORD_BYTES") = (int)sizeof(MsgRecord);
  m.attr("REPLY_RECORD_BYTES") = (int)sizeof(ReplyRecord);
}
