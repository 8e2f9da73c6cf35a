#include "storage.hpp"

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "codec.hpp"
#include "util.hpp"

namespace ptype {

namespace {
enum RecType : uint8_t { kRecEntry = 1, kRecHardState = 2 };

std::string enc_entry(const raft::Entry& e) {
  Writer w;
  w.u64(e.term);
  w.u64(e.index);
  w.u8(e.type);
  w.str(e.data);
  return w.buf;
}

std::string enc_hs(const raft::HardState& hs) {
  Writer w;
  w.u64(hs.term);
  w.u64(hs.vote);
  w.u64(hs.commit);
  return w.buf;
}

void write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::write(fd, p, n);
    if (k < 0) {
      if (errno == EINTR) continue;
      fail(std::string("wal write: ") + strerror(errno));
    }
    p += k;
    n -= (size_t)k;
  }
}

bool read_file_bytes(const std::string& path, std::string* out) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  out->clear();
  char buf[65536];
  for (;;) {
    ssize_t k = ::read(fd, buf, sizeof buf);
    if (k <= 0) break;
    out->append(buf, (size_t)k);
  }
  ::close(fd);
  return true;
}

void write_file_atomic(const std::string& path, const std::string& data, bool fsync) {
  const std::string tmp = path + ".tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) fail("open " + tmp + ": " + strerror(errno));
  write_all(fd, data.data(), data.size());
  if (fsync) ::fsync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path.c_str()) != 0) fail("rename " + tmp + ": " + strerror(errno));
}
}  // namespace

void mkdir_p(const std::string& dir) {
  if (dir.empty()) return;
  std::string cur;
  for (const auto& part : split(dir, '/')) {
    cur += part;
    if (!cur.empty()) ::mkdir(cur.c_str(), 0755);
    cur += "/";
  }
  struct stat st;
  if (::stat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) fail("cannot create data dir " + dir);
}

Storage::Storage(const std::string& dir, bool fsync) : dir_(dir), fsync_(fsync) { mkdir_p(dir_ + "/member"); }

Storage::~Storage() {
  if (wal_fd_ >= 0) ::close(wal_fd_);
}

void Storage::open_wal() {
  if (wal_fd_ >= 0) return;
  const std::string p = dir_ + "/member/wal.log";
  wal_fd_ = ::open(p.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (wal_fd_ < 0) fail("open " + p + ": " + strerror(errno));
}

void Storage::write_record(int fd, uint8_t type, const std::string& payload) {
  Writer w;
  w.u32((uint32_t)payload.size() + 1);
  std::string body;
  body.push_back((char)type);
  body += payload;
  w.u32(crc32c(body.data(), body.size()));
  w.buf += body;
  write_all(fd, w.buf.data(), w.buf.size());
  bytes_ += w.buf.size();
}

Storage::Loaded Storage::load() {
  std::lock_guard<std::mutex> g(mu_);
  Loaded L;
  std::string snap;
  if (read_file_bytes(dir_ + "/member/snap.bin", &snap) && !snap.empty()) {
    Reader r(snap);
    L.snap_index = r.u64();
    L.snap_term = r.u64();
    L.snap_data = r.str();
    L.hs.term = r.u64();
    L.hs.vote = r.u64();
    L.hs.commit = r.u64();
    L.any = true;
  }
  read_file_bytes(dir_ + "/member/meta.bin", &L.meta);
  if (!L.meta.empty()) L.any = true;
  std::string wal;
  if (read_file_bytes(dir_ + "/member/wal.log", &wal)) {
    size_t i = 0;
    while (i + 8 <= wal.size()) {
      uint32_t len, crc;
      memcpy(&len, wal.data() + i, 4);
      memcpy(&crc, wal.data() + i + 4, 4);
      if (len == 0 || i + 8 + len > wal.size()) break;  // torn tail: stop at the last whole record
      const char* body = wal.data() + i + 8;
      if (crc32c(body, len) != crc) break;
      const uint8_t type = (uint8_t)body[0];
      Reader r(body + 1, len - 1);
      if (type == kRecEntry) {
        raft::Entry e;
        e.term = r.u64();
        e.index = r.u64();
        e.type = r.u8();
        e.data = r.str();
        if (e.index > L.snap_index) {
          // an entry index that re-appears replaces the old suffix (conflict truncation)
          while (!L.entries.empty() && L.entries.back().index >= e.index) L.entries.pop_back();
          const uint64_t want = L.entries.empty() ? L.snap_index + 1 : L.entries.back().index + 1;
          if (e.index == want) L.entries.push_back(e);
        }
      } else if (type == kRecHardState) {
        L.hs.term = r.u64();
        L.hs.vote = r.u64();
        L.hs.commit = r.u64();
      }
      L.any = true;
      i += 8 + len;
    }
  }
  return L;
}

void Storage::append(const std::vector<raft::Entry>& ents, const raft::HardState* hs) {
  if (ents.empty() && !hs) return;
  std::lock_guard<std::mutex> g(mu_);
  open_wal();
  for (const auto& e : ents) write_record(wal_fd_, kRecEntry, enc_entry(e));
  if (hs) write_record(wal_fd_, kRecHardState, enc_hs(*hs));
  if (fsync_) ::fdatasync(wal_fd_);
}

void Storage::save_meta(const std::string& meta) {
  std::lock_guard<std::mutex> g(mu_);
  write_file_atomic(dir_ + "/member/meta.bin", meta, fsync_);
}

void Storage::save_snapshot(uint64_t index, uint64_t term, const std::string& data, const raft::HardState& hs,
                            const std::vector<raft::Entry>& tail) {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  w.u64(index);
  w.u64(term);
  w.str(data);
  w.u64(hs.term);
  w.u64(hs.vote);
  w.u64(hs.commit);
  write_file_atomic(dir_ + "/member/snap.bin", w.buf, fsync_);
  // rewrite the WAL with only the entries after the snapshot
  const std::string p = dir_ + "/member/wal.log";
  const std::string tmp = p + ".tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) fail("open " + tmp + ": " + strerror(errno));
  for (const auto& e : tail) write_record(fd, kRecEntry, enc_entry(e));
  write_record(fd, kRecHardState, enc_hs(hs));
  if (fsync_) ::fsync(fd);
  ::close(fd);
  if (wal_fd_ >= 0) {
    ::close(wal_fd_);
    wal_fd_ = -1;
  }
  if (::rename(tmp.c_str(), p.c_str()) != 0) fail("rename wal: " + std::string(strerror(errno)));
}

}  // namespace ptype
