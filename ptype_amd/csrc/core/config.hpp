// Configuration: the ptype YAML (cluster/config.go:12-21) and the
// control-plane member YAML that the reference hands to etcd's
// embed.ConfigFromFile (cluster/config.go:35-43; keys as in
// cluster/testdata/node1.yml).  Both are parsed by the C++ YAML subset with the
// YAML->JSON typing rules of sigs.k8s.io/yaml.  A `gpu:` section adds the
// device-runtime keys (device ordinal, ring slots, actor shard size, ...).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "yaml.hpp"

namespace ptype {

struct Url {
  std::string scheme, host, raw;
  int port = 0;
};
Url parse_url(const std::string& s);  // throws kConfig

// Control-plane member settings (the reference's embed.Config subset).
struct MemberConfig {
  std::string name = "default";
  std::string dir;  // data-dir (WAL + snapshots)
  std::vector<std::string> lpurls{"http://localhost:2380"};  // listen-peer-urls
  std::vector<std::string> lcurls{"http://localhost:2379"};  // listen-client-urls
  std::vector<std::string> apurls{"http://localhost:2380"};  // initial-advertise-peer-urls
  std::vector<std::string> acurls{"http://localhost:2379"};  // advertise-client-urls
  std::string initial_cluster;                               // name=url,...
  std::string initial_cluster_token = "etcd-cluster";
  std::string cluster_state = "new";  // new | existing
  bool strict_reconfig_check = true;
  std::string logger = "capnslog";
  int64_t heartbeat_ms = 100;
  int64_t election_ms = 1000;
  uint64_t snapshot_count = 100000;
  bool unsafe_no_fsync = false;

  void validate() const;  // throws kConfig (etcd's Config.Validate checks)
  std::string effective_initial_cluster() const;
  static MemberConfig from_yaml(const YNode& root);
  static MemberConfig from_file(const std::string& path);
};

struct GpuConfig {
  int device = -1;            // -1: LOCAL_RANK (one process per GPU)
  uint32_t ring = 4096;       // latency-path ring slots (power of two)
  uint32_t actors = 1024;     // actor mailboxes hosted by this process
  double idle_ms = 200.0;     // persistent dispatcher idle exit
  uint64_t delay_us = 0;      // Prime.Check per-candidate delay (250000 in the reference)
  uint64_t max_batch = 1 << 20;
  int world = 0;              // data-plane ranks of the service: > 1 makes Join form the group
  std::string backend;        // "" = nccl (RCCL) on a GPU, gloo with cpu
  bool cpu = false;           // actor runtime on the host reference path (tests, GPU-less hosts)
  uint32_t mailbox_shards = 256;
  uint32_t mailbox_slots = 0;  // 0: sized from max_batch
  std::string delivery = "auto";  // "mailbox": every Send through the HBM mailboxes; "direct"; "auto"
  // data-plane collectives at world > 1: "rccl" (the group's communicator, one GPU per rank) or
  // "ipc" (IpcComm: shared-memory segments every rank maps, over a gloo group; ranks may share a GPU)
  std::string comm = "rccl";
  bool watch = true;          // follow the store (shard records, leases) into the GPU registry mirror
  // rank failures (runtime.py recover): Join's group re-forms through the store
  bool elastic = true;          // recover a failed Send (abort, re-form, re-home, re-send)
  bool form_group = false;      // form the group through the store even at world <= 1 (collectives forced)
  double group_timeout_s = 10;  // collective timeout of the group (gloo; RCCL's is the send watchdog's)
  double grace_s = 8;           // how long a recovery waits for the dead node's lease to lapse
  double send_timeout_s = 30;   // GPU: a Send's device work overdue this long aborts the communicator
  uint32_t replicate_every = 0; // buddy replicas of the actor state every N Sends (0: only on request)
  // RCCL groups: the communicator's lifecycle in the control plane (dataplane.hpp: store
  // rendezvous, ncclCommInitRank, ncclCommAbort, next generation) instead of a torch process group
  bool native_group = true;
  // path switches of the data plane ("key=value,..."; csrc/hip/tune.hpp, ops/tune.py),
  // from the `tune:` map -- applied by Join before the device runtime starts
  std::string tune;
};

struct Config {
  std::string service_name;
  std::string node_name;
  int64_t port = 0;
  std::string etcd_config_file;
  std::vector<std::string> initial_cluster_client_urls;
  bool debug = false;
  bool has_gpu = false;
  GpuConfig gpu;
  std::shared_ptr<MemberConfig> member;  // reference: unexported Config.etcdConfig
};

// ConfigFromFile (cluster/config.go:23-46): ptype YAML, then the member YAML
// resolved relative to the ptype file's directory, then validation.
Config config_from_file(const std::string& path);
Config config_from_yaml(const std::string& text);  // ptype keys only (no member file)

std::string read_file(const std::string& path);

}  // namespace ptype
