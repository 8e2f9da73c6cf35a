// Small host utilities: errors, time, strings, context/cancellation, channels,
// leveled logger (zap replacement with the reference's event names).
#pragma once
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ptype {

// ---------------------------------------------------------------- errors
// Sentinel-style error with a stable code so bindings can map it to the
// reference's sentinel errors (ErrNoKey cluster/store.go:15,
// ErrNoClientAvailable cluster/rpc.go:16, etcd's ErrLearnerNotReady, ...).
enum class Errc : int {
  kGeneric = 1,
  kNoKey = 2,
  kNoClientAvailable = 3,
  kLearnerNotReady = 4,
  kTimeout = 5,
  kCanceled = 6,
  kNotLeader = 7,
  kConfig = 8,
  kUnavailable = 9,
  kRpc = 10,          // remote handler returned an error string (rpc.ServerError)
  kShutdown = 11,     // connection closed (rpc.ErrShutdown)
  kMemberExists = 12,
  kMemberNotFound = 13,
  kCompacted = 14,
  kLeaseNotFound = 15,
};

class Error : public std::runtime_error {
 public:
  Error(Errc c, const std::string& msg) : std::runtime_error(msg), code_(c) {}
  Errc code() const { return code_; }

 private:
  Errc code_;
};

[[noreturn]] inline void fail(Errc c, const std::string& msg) { throw Error(c, msg); }
[[noreturn]] inline void fail(const std::string& msg) { throw Error(Errc::kGeneric, msg); }

// ---------------------------------------------------------------- time
using Clock = std::chrono::steady_clock;
inline int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now().time_since_epoch()).count();
}
inline int64_t mono_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(Clock::now().time_since_epoch()).count();
}
void sleep_ms(int64_t ms);

// ---------------------------------------------------------------- strings
std::vector<std::string> split(const std::string& s, char sep);
std::string join(const std::vector<std::string>& v, const std::string& sep);
std::string trim(const std::string& s);
bool starts_with(const std::string& s, const std::string& p);
// Go's filepath.Join semantics (join non-empty elements with '/', then Clean).
std::string path_join(const std::vector<std::string>& elems);
std::string path_clean(const std::string& p);
std::string path_dir(const std::string& p);  // filepath.Split's dir part
uint32_t fnv1a32(const std::string& s);
uint64_t fnv1a64(const std::string& s);

// ---------------------------------------------------------------- context
// Go context.Context analogue: cancellation + optional deadline + callbacks.
class Context {
 public:
  static std::shared_ptr<Context> background();
  static std::shared_ptr<Context> with_cancel(const std::shared_ptr<Context>& parent);
  static std::shared_ptr<Context> with_timeout(const std::shared_ptr<Context>& parent, int64_t ms);

  void cancel();
  bool done() const;
  // Returns true if canceled/expired within `ms` (ms < 0: wait forever).
  bool wait(int64_t ms) const;
  // Registers a callback run (once) on cancellation; runs immediately if done.
  void on_done(std::function<void()> fn);
  std::string err() const;

  struct State;

 private:
  std::shared_ptr<State> st_;
  Context();
  friend struct ContextAccess;
};
using Ctx = std::shared_ptr<Context>;

// ---------------------------------------------------------------- channel
// Go channel analogue (bounded FIFO, cap 0 = rendezvous-ish: send blocks until
// the value has been taken).
template <class T>
class Channel {
 public:
  explicit Channel(size_t cap = 0) : cap_(cap) {}

  // Returns false if the channel is closed (or ctx canceled).
  bool send(T v, const Ctx& ctx = nullptr) {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t my = ++sent_;
    q_.push_back(std::move(v));
    cv_.notify_all();
    for (;;) {
      if (closed_) return false;
      // delivered once `taken_ >= my` when unbuffered, or once there is room
      if (cap_ == 0 ? taken_ >= my : q_.size() <= cap_) return true;
      if (ctx && ctx->done()) return false;
      cv_.wait_for(lk, std::chrono::milliseconds(ctx ? 5 : 50));
    }
  }
  bool try_send(T v) {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_ || q_.size() >= std::max<size_t>(cap_, 1)) return false;
    ++sent_;
    q_.push_back(std::move(v));
    cv_.notify_all();
    return true;
  }
  // timeout_ms < 0: forever.  Returns nullopt on timeout or when closed+drained.
  std::optional<T> recv(int64_t timeout_ms = -1, bool* closed = nullptr) {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [&] { return !q_.empty() || closed_; };
    if (timeout_ms < 0)
      cv_.wait(lk, pred);
    else
      cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred);
    if (closed) *closed = q_.empty() && closed_;
    if (q_.empty()) return std::nullopt;
    T v = std::move(q_.front());
    q_.pop_front();
    ++taken_;
    cv_.notify_all();
    return v;
  }
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    cv_.notify_all();
  }
  bool closed() const {
    std::lock_guard<std::mutex> lk(mu_);
    return closed_;
  }
  size_t size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 private:
  size_t cap_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
  bool closed_ = false;
  uint64_t sent_ = 0, taken_ = 0;
};

// ---------------------------------------------------------------- logging
// Leveled logger with zap-like structured fields.  Off by default, as
// zap's global no-op logger is in the reference; `debug: true` in the config
// switches it to Debug (cluster/cluster.go:29-35).
enum class LogLevel : int { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3, kOff = 4 };
using Fields = std::vector<std::pair<std::string, std::string>>;

void log_set_level(LogLevel lv);
LogLevel log_level();
void log_write(LogLevel lv, const std::string& msg, const Fields& f = {});
// Recent log lines kept in memory (for tests / debug endpoint).
std::vector<std::string> log_recent(size_t n);
inline void log_debug(const std::string& m, const Fields& f = {}) { log_write(LogLevel::kDebug, m, f); }
inline void log_info(const std::string& m, const Fields& f = {}) { log_write(LogLevel::kInfo, m, f); }
inline void log_warn(const std::string& m, const Fields& f = {}) { log_write(LogLevel::kWarn, m, f); }
inline void log_error(const std::string& m, const Fields& f = {}) { log_write(LogLevel::kError, m, f); }

}  // namespace ptype
