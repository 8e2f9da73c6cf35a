// The data plane's path switches, in ONE place.
//
// Every switch here selects between two implementations that are both kept on
// purpose (the default is the measured-faster one; the other is either a
// correctness reference a GPU test compares against, or a path for a situation
// the default does not cover).  Variants that only measured slower were deleted
// and their A/B rows live in profiles/.
//
// Source: the `gpu: tune:` map of the config (ptype_amd.cluster applies it with
// _hip.set_tune) or the environment, PTYPE_TUNE="key=value,key=value" (tests and
// the profiling tools).  The table is re-read when PTYPE_TUNE changes, and each
// engine reads it when it is built or per Send -- never per kernel.
//
//   key               default  meaning
//   mbox_fused        -1       stateless world-1 mailbox Sends: fused sort + drain kernel
//                              (-1: up to 512 tiles, 0 never, 1 always)
//   mbox_rec8         -1       8-B ring records (-1: batches past 512 tiles, 0 never, 1 always)
//   mbox_sort         0        mailbox sort: 0 auto, 1 one-pass, 2 count + scatter
//   mbox_drain_msg    0        stateless drain in message order instead of ring order
//   sx_sort           0        sorted exchange, rank-only batches: 0 reserving one pass,
//                              1 look-back one pass, 2 count + scan + scatter
//   sx_self_copy      0        world-1 sorted exchange: the all-to-alls as device copies
//                              (RCCL calls on a forked stream cannot be graph-captured)
//   sx_comm_cs        -1       sorted exchange collectives on the caller's stream (-1: Sends
//                              of up to 2 Mi messages, 0 never, 1 always)
//   stream_sync       0        epoch engine hand-offs: 0 events, 1 stream wait-value packets
//   local             1        world-1 epoch Sends: the fused local pass (0: the slot pipeline)
//   persistent_stream low      queue of persistent kernels: low / high / cumask / pooled
//   poll_lanes        -1       dispatcher polling lanes (-1: built-in default)
//   poll_full         -1       dispatcher reads whole slots per poll
//   poll_sleep        -1       dispatcher s_sleep between idle polls
#pragma once
#include <cstdlib>
#include <mutex>
#include <string>

namespace ptype {

struct Tune {
  int mbox_fused = -1;
  int mbox_rec8 = -1;
  int mbox_sort = 0;
  int mbox_drain_msg = 0;
  int sx_sort = 0;
  int sx_self_copy = 0;
  int sx_comm_cs = -1;
  int stream_sync = 0;
  int local = 1;
  std::string persistent_stream = "low";
  int poll_lanes = -1, poll_full = -1, poll_sleep = -1;

  // one "key=value" item; false for an unknown key
  bool set(const std::string& k, const std::string& v) {
    auto i = [&](int& f) {
      f = std::atoi(v.c_str());
      return true;
    };
    if (k == "mbox_fused") return i(mbox_fused);
    if (k == "mbox_rec8") return i(mbox_rec8);
    if (k == "mbox_sort") return i(mbox_sort);
    if (k == "mbox_drain_msg") return i(mbox_drain_msg);
    if (k == "sx_sort") return i(sx_sort);
    if (k == "sx_self_copy") return i(sx_self_copy);
    if (k == "sx_comm_cs") return i(sx_comm_cs);
    if (k == "stream_sync") return i(stream_sync);
    if (k == "local") return i(local);
    if (k == "poll_lanes") return i(poll_lanes);
    if (k == "poll_full") return i(poll_full);
    if (k == "poll_sleep") return i(poll_sleep);
    if (k == "persistent_stream") {
      persistent_stream = v;
      return true;
    }
    return false;
  }
  static Tune parse(const std::string& spec) {
    Tune t;
    size_t p = 0;
    while (p < spec.size()) {
      size_t e = spec.find(',', p);
      if (e == std::string::npos) e = spec.size();
      const std::string item = spec.substr(p, e - p);
      const size_t eq = item.find('=');
      if (eq != std::string::npos) (void)t.set(item.substr(0, eq), item.substr(eq + 1));
      p = e + 1;
    }
    return t;
  }
};

namespace tune_detail {
struct State {
  std::mutex mu;
  std::string env_seen;  // the PTYPE_TUNE string the table was parsed from
  std::string overrides;  // set_tune(): applied after the environment
  Tune t;
  bool init = false;
};
inline State& state() {
  static State s;
  return s;
}
}  // namespace tune_detail

// The table in force (a copy: cheap, read per Send at most).
inline Tune tune() {
  auto& s = tune_detail::state();
  std::lock_guard<std::mutex> lk(s.mu);
  const char* e = std::getenv("PTYPE_TUNE");
  const std::string env = e ? e : "";
  if (!s.init || env != s.env_seen) {
    s.t = Tune::parse(env + (s.overrides.empty() ? "" : "," + s.overrides));
    s.env_seen = env;
    s.init = true;
  }
  return s.t;
}

// Programmatic overrides ("key=value,..."), e.g. from the config's gpu.tune map;
// returns false if a key is unknown (nothing applied then).
inline bool set_tune(const std::string& spec) {
  Tune probe;
  size_t p = 0;
  while (p < spec.size()) {
    size_t e = spec.find(',', p);
    if (e == std::string::npos) e = spec.size();
    const std::string item = spec.substr(p, e - p);
    const size_t eq = item.find('=');
    if (!item.empty() && (eq == std::string::npos || !probe.set(item.substr(0, eq), item.substr(eq + 1)))) return false;
    p = e + 1;
  }
  auto& s = tune_detail::state();
  std::lock_guard<std::mutex> lk(s.mu);
  s.overrides = spec;
  s.init = false;
  return true;
}

}  // namespace ptype
