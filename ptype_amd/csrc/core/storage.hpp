// Durable Raft storage: an append-only WAL of entries and hard
// states with CRC32C-checked records, plus an atomically replaced snapshot file
// of the applied state machine.  Mirrors what etcd keeps in `data-dir`
// (cluster/testdata/node1.yml:4-5); restarting a member on the same directory
// resumes its log, membership and KV state.
#pragma once
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "raft.hpp"

namespace ptype {

class Storage {
 public:
  Storage(const std::string& dir, bool fsync);
  ~Storage();

  struct Loaded {
    bool any = false;
    raft::HardState hs;
    uint64_t snap_index = 0, snap_term = 0;
    std::string snap_data;
    std::vector<raft::Entry> entries;  // after the snapshot, conflicts resolved
    std::string meta;
  };
  Loaded load();

  void append(const std::vector<raft::Entry>& ents, const raft::HardState* hs);
  void save_meta(const std::string& meta);
  // Persist a snapshot and rewrite the WAL to hold only what follows it.
  void save_snapshot(uint64_t index, uint64_t term, const std::string& data, const raft::HardState& hs,
                     const std::vector<raft::Entry>& tail);
  const std::string& dir() const { return dir_; }
  uint64_t bytes_written() const { return bytes_; }

 private:
  void open_wal();
  void write_record(int fd, uint8_t type, const std::string& payload);
  std::string dir_;
  bool fsync_;
  int wal_fd_ = -1;
  uint64_t bytes_ = 0;
  std::mutex mu_;
};

void mkdir_p(const std::string& dir);

}  // namespace ptype
