#include "config.hpp"

#include <arpa/inet.h>

#include <fstream>
#include <sstream>

#include "util.hpp"

namespace ptype {

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) fail(Errc::kConfig, "open " + path + ": no such file or directory");
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

Url parse_url(const std::string& s) {
  Url u;
  u.raw = s;
  const size_t p = s.find("://");
  if (p == std::string::npos) fail(Errc::kConfig, "parse \"" + s + "\": missing protocol scheme");
  u.scheme = s.substr(0, p);
  if (u.scheme != "http" && u.scheme != "https" && u.scheme != "unix" && u.scheme != "unixs")
    fail(Errc::kConfig, "URL scheme must be http, https, unix, or unixs: " + s);
  std::string rest = s.substr(p + 3);
  const size_t slash = rest.find('/');
  if (slash != std::string::npos) rest = rest.substr(0, slash);
  const size_t colon = rest.rfind(':');
  if (colon == std::string::npos) {
    u.host = rest;
    u.port = u.scheme == "https" ? 443 : 80;
  } else {
    u.host = rest.substr(0, colon);
    const std::string ps = rest.substr(colon + 1);
    char* end = nullptr;
    long v = strtol(ps.c_str(), &end, 10);
    if (ps.empty() || *end || v < 0 || v > 65535) fail(Errc::kConfig, "invalid port in URL " + s);
    u.port = (int)v;
  }
  if (u.host.empty()) fail(Errc::kConfig, "URL address does not have the form \"host:port\": " + s);
  return u;
}

namespace {

[[noreturn]] void type_err(const std::string& strct, const std::string& field, const YNode& v,
                           const std::string& want) {
  fail(Errc::kConfig, "error unmarshaling JSON: json: cannot unmarshal " + v.type_name() +
                          " into Go struct field " + strct + "." + field + " of type " + want);
}

std::string want_string(const std::string& st, const std::string& f, const YNode& v) {
  if (v.is_null()) return "";
  if (v.kind != YNode::kScalar) type_err(st, f, v, "string");
  const std::string t = v.type_name();
  if (t != "string") type_err(st, f, v, "string");
  return v.scalar;
}

int64_t want_int(const std::string& st, const std::string& f, const YNode& v) {
  if (v.is_null()) return 0;
  long long x;
  if (!v.is_int(&x)) type_err(st, f, v, "int");
  return x;
}

double want_float(const std::string& st, const std::string& f, const YNode& v) {
  if (v.is_null()) return 0;
  double x;
  if (!v.is_float(&x)) type_err(st, f, v, "float64");
  return x;
}

bool want_bool(const std::string& st, const std::string& f, const YNode& v) {
  if (v.is_null()) return false;
  bool b;
  if (!v.is_bool(&b)) type_err(st, f, v, "bool");
  return b;
}

std::vector<std::string> want_strings(const std::string& st, const std::string& f, const YNode& v) {
  std::vector<std::string> out;
  if (v.is_null()) return out;
  if (v.kind != YNode::kSeq) type_err(st, f, v, "[]string");
  for (const auto& x : v.seq) out.push_back(want_string(st, f, x));
  return out;
}

std::vector<std::string> url_list(const std::string& s) {
  std::vector<std::string> out;
  for (auto& p : split(s, ','))
    if (!trim(p).empty()) out.push_back(trim(p));
  return out;
}

void decode_ptype(const YNode& root, Config& c) {
  if (root.kind == YNode::kNull) return;
  if (root.kind != YNode::kMap)
    fail(Errc::kConfig, "error unmarshaling JSON: json: cannot unmarshal " + root.type_name() +
                            " into Go value of type cluster.Config");
  const std::string S = "Config";
  for (const auto& kv : root.map) {
    const std::string& k = kv.first;
    const YNode& v = kv.second;
    if (k == "service_name") c.service_name = want_string(S, k, v);
    else if (k == "node_name") c.node_name = want_string(S, k, v);
    else if (k == "port") c.port = want_int(S, k, v);
    else if (k == "etcd_config_file") c.etcd_config_file = want_string(S, k, v);
    else if (k == "initial_cluster_client_urls") c.initial_cluster_client_urls = want_strings(S, k, v);
    else if (k == "debug") c.debug = want_bool(S, k, v);
    else if (k == "gpu") {
      if (v.is_null()) continue;
      if (v.kind != YNode::kMap) type_err(S, k, v, "cluster.GPUConfig");
      c.has_gpu = true;
      const std::string G = "GPUConfig";
      for (const auto& g : v.map) {
        if (g.first == "device") c.gpu.device = (int)want_int(G, g.first, g.second);
        else if (g.first == "ring") c.gpu.ring = (uint32_t)want_int(G, g.first, g.second);
        else if (g.first == "actors") c.gpu.actors = (uint32_t)want_int(G, g.first, g.second);
        else if (g.first == "idle_ms") c.gpu.idle_ms = want_float(G, g.first, g.second);
        else if (g.first == "delay_us") c.gpu.delay_us = (uint64_t)want_int(G, g.first, g.second);
        else if (g.first == "max_batch") c.gpu.max_batch = (uint64_t)want_int(G, g.first, g.second);
        else if (g.first == "world") c.gpu.world = (int)want_int(G, g.first, g.second);
        else if (g.first == "backend") c.gpu.backend = want_string(G, g.first, g.second);
        else if (g.first == "cpu") c.gpu.cpu = want_bool(G, g.first, g.second);
        else if (g.first == "mailbox_shards") c.gpu.mailbox_shards = (uint32_t)want_int(G, g.first, g.second);
        else if (g.first == "mailbox_slots") c.gpu.mailbox_slots = (uint32_t)want_int(G, g.first, g.second);
        else if (g.first == "watch") c.gpu.watch = want_bool(G, g.first, g.second);
        else if (g.first == "elastic") c.gpu.elastic = want_bool(G, g.first, g.second);
        else if (g.first == "delivery") c.gpu.delivery = want_string(G, g.first, g.second);
        else if (g.first == "comm") c.gpu.comm = want_string(G, g.first, g.second);
        else if (g.first == "form_group") c.gpu.form_group = want_bool(G, g.first, g.second);
        else if (g.first == "native_group") c.gpu.native_group = want_bool(G, g.first, g.second);
        else if (g.first == "group_timeout_s") c.gpu.group_timeout_s = want_float(G, g.first, g.second);
        else if (g.first == "grace_s") c.gpu.grace_s = want_float(G, g.first, g.second);
        else if (g.first == "send_timeout_s") c.gpu.send_timeout_s = want_float(G, g.first, g.second);
        else if (g.first == "replicate_every") c.gpu.replicate_every = (uint32_t)want_int(G, g.first, g.second);
        else if (g.first == "tune") {  // the data plane's path switches: {key: value} -> "key=value,..."
          if (g.second.is_null()) continue;
          if (g.second.kind != YNode::kMap) type_err(G, g.first, g.second, "map[string]string");
          for (const auto& t : g.second.map)
          {
            if (t.second.kind != YNode::kScalar) type_err(G, t.first, t.second, "scalar");
            c.gpu.tune += (c.gpu.tune.empty() ? "" : ",") + t.first + "=" + t.second.scalar;
          }
        }
      }
      if (c.gpu.mailbox_shards == 0 || (c.gpu.mailbox_shards & (c.gpu.mailbox_shards - 1)))
        fail(Errc::kConfig, "gpu.mailbox_shards must be a power of two");
      if (c.gpu.world < 0) fail(Errc::kConfig, "gpu.world must be >= 0");
      if (c.gpu.delivery != "auto" && c.gpu.delivery != "mailbox" && c.gpu.delivery != "direct")
        fail(Errc::kConfig, "gpu.delivery must be auto, mailbox or direct");
      if (c.gpu.comm != "rccl" && c.gpu.comm != "ipc") fail(Errc::kConfig, "gpu.comm must be rccl or ipc");
      if (c.gpu.ring == 0 || (c.gpu.ring & (c.gpu.ring - 1)))
        fail(Errc::kConfig, "gpu.ring must be a power of two");
    }
    // unknown keys are ignored, as encoding/json does
  }
}

bool is_ip_or_localhost(const std::string& h) {
  if (h == "localhost") return true;
  unsigned char buf[16];
  return inet_pton(AF_INET, h.c_str(), buf) == 1 || inet_pton(AF_INET6, h.c_str(), buf) == 1;
}

}  // namespace

MemberConfig MemberConfig::from_yaml(const YNode& root) {
  MemberConfig m;
  if (root.kind == YNode::kNull) return m;
  if (root.kind != YNode::kMap) fail(Errc::kConfig, "member config: expected a mapping");
  const std::string S = "configYAML";
  bool apset = false, acset = false;
  for (const auto& kv : root.map) {
    const std::string& k = kv.first;
    const YNode& v = kv.second;
    if (k == "name") m.name = want_string(S, k, v);
    else if (k == "data-dir") m.dir = want_string(S, k, v);
    else if (k == "listen-peer-urls") m.lpurls = url_list(want_string(S, k, v));
    else if (k == "listen-client-urls") m.lcurls = url_list(want_string(S, k, v));
    else if (k == "initial-advertise-peer-urls") {
      m.apurls = url_list(want_string(S, k, v));
      apset = true;
    } else if (k == "advertise-client-urls") {
      m.acurls = url_list(want_string(S, k, v));
      acset = true;
    } else if (k == "initial-cluster") m.initial_cluster = want_string(S, k, v);
    else if (k == "initial-cluster-token") m.initial_cluster_token = want_string(S, k, v);
    else if (k == "initial-cluster-state") m.cluster_state = want_string(S, k, v);
    else if (k == "strict-reconfig-check") m.strict_reconfig_check = want_bool(S, k, v);
    else if (k == "logger") m.logger = want_string(S, k, v);
    else if (k == "heartbeat-interval") m.heartbeat_ms = want_int(S, k, v);
    else if (k == "election-timeout") m.election_ms = want_int(S, k, v);
    else if (k == "snapshot-count") m.snapshot_count = (uint64_t)want_int(S, k, v);
    else if (k == "unsafe-no-fsync") m.unsafe_no_fsync = want_bool(S, k, v);
  }
  if (!apset && m.lpurls.size() && m.apurls == std::vector<std::string>{"http://localhost:2380"}) m.apurls = m.lpurls;
  if (!acset && m.lcurls.size() && m.acurls == std::vector<std::string>{"http://localhost:2379"}) m.acurls = m.lcurls;
  return m;
}

MemberConfig MemberConfig::from_file(const std::string& path) { return from_yaml(yaml_parse(read_file(path))); }

std::string MemberConfig::effective_initial_cluster() const {
  if (!initial_cluster.empty()) return initial_cluster;
  std::vector<std::string> parts;
  for (const auto& u : apurls) parts.push_back(name + "=" + u);
  return join(parts, ",");
}

void MemberConfig::validate() const {
  for (const auto& list : {lpurls, lcurls}) {
    if (list.empty()) fail(Errc::kConfig, "listen URLs must not be empty");
    for (const auto& s : list) {
      Url u = parse_url(s);
      if (!is_ip_or_localhost(u.host))
        fail(Errc::kConfig, "expected IP in URL for binding (" + s + ")");
    }
  }
  for (const auto& list : {apurls, acurls})
    for (const auto& s : list) parse_url(s);
  if (5 * heartbeat_ms > election_ms)
    fail(Errc::kConfig, "--election-timeout[" + std::to_string(election_ms) +
                            "ms] should be at least as 5 times as --heartbeat-interval[" +
                            std::to_string(heartbeat_ms) + "ms]");
  if (election_ms > 50000)
    fail(Errc::kConfig, "--election-timeout[" + std::to_string(election_ms) + "ms] is too long, and should be set less than 50 seconds");
  if (cluster_state != "new" && cluster_state != "existing")
    fail(Errc::kConfig, "unexpected clusterState \"" + cluster_state + "\"");
  for (const auto& ent : split(effective_initial_cluster(), ',')) {
    if (trim(ent).empty()) continue;
    const size_t eq = ent.find('=');
    if (eq == std::string::npos) fail(Errc::kConfig, "initial-cluster entry \"" + ent + "\" is not name=url");
    parse_url(trim(ent.substr(eq + 1)));
  }
}

Config config_from_yaml(const std::string& text) {
  Config c;
  try {
    decode_ptype(yaml_parse(text), c);
  } catch (const Error& e) {
    fail(Errc::kConfig, std::string("failed to read yaml of cluster config: ") + e.what());
  }
  return c;
}

Config config_from_file(const std::string& path) {
  std::string text;
  try {
    text = read_file(path);
  } catch (const Error& e) {
    fail(Errc::kConfig, "failed to read cluster config at " + path + ": " + e.what());
  }
  Config c = config_from_yaml(text);
  const std::string member_path = path_join({path_dir(path), c.etcd_config_file});
  try {
    c.member = std::make_shared<MemberConfig>(MemberConfig::from_file(member_path));
  } catch (const Error& e) {
    fail(Errc::kConfig, "failed to read etcd config from " + c.etcd_config_file + ": " + e.what());
  }
  try {
    c.member->validate();
  } catch (const Error& e) {
    fail(Errc::kConfig, std::string("etcd config provided is not valid: ") + e.what());
  }
  return c;
}

}  // namespace ptype
