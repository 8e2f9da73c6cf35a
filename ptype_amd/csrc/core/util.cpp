#include "util.hpp"

#include <stdio.h>

#include <thread>

namespace ptype {

void sleep_ms(int64_t ms) { std::this_thread::sleep_for(std::chrono::milliseconds(ms)); }

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\t' || s[b] == '\r' || s[b] == '\n')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r' || s[e - 1] == '\n')) --e;
  return s.substr(b, e - b);
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }

// Go path.Clean: collapse //, resolve . and .., no trailing slash (except "/").
std::string path_clean(const std::string& p) {
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> out;
  for (const auto& part : split(p, '/')) {
    if (part.empty() || part == ".") continue;
    if (part == "..") {
      if (!out.empty() && out.back() != "..")
        out.pop_back();
      else if (!rooted)
        out.push_back("..");
      continue;
    }
    out.push_back(part);
  }
  std::string r = (rooted ? "/" : "") + join(out, "/");
  if (r.empty()) return ".";
  return r;
}

std::string path_join(const std::vector<std::string>& elems) {
  std::vector<std::string> nz;
  for (const auto& e : elems)
    if (!e.empty()) nz.push_back(e);
  if (nz.empty()) return "";
  return path_clean(join(nz, "/"));
}

std::string path_dir(const std::string& p) {
  const size_t i = p.rfind('/');
  return i == std::string::npos ? std::string() : p.substr(0, i + 1);
}

uint32_t fnv1a32(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) {
    h ^= c;
    h *= 16777619u;
  }
  return h;
}

uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 14695981039346656037ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

// ---------------------------------------------------------------- context
struct Context::State {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::string err;
  int64_t deadline_ms = -1;
  std::vector<std::function<void()>> cbs;
  std::vector<std::weak_ptr<State>> children;
};

struct ContextAccess {
  static std::shared_ptr<Context::State>& st(Context& c) { return c.st_; }
};

Context::Context() : st_(std::make_shared<State>()) {}

static void cancel_state(const std::shared_ptr<Context::State>& s, const std::string& why) {
  std::vector<std::function<void()>> cbs;
  std::vector<std::weak_ptr<Context::State>> kids;
  {
    std::lock_guard<std::mutex> g(s->mu);
    if (s->done) return;
    s->done = true;
    s->err = why;
    cbs.swap(s->cbs);
    kids.swap(s->children);
    s->cv.notify_all();
  }
  for (auto& k : kids)
    if (auto ks = k.lock()) cancel_state(ks, why);
  for (auto& f : cbs) f();
}

Ctx Context::background() {
  static Ctx bg(new Context());
  return bg;
}

Ctx Context::with_cancel(const Ctx& parent) {
  Ctx c(new Context());
  if (parent) {
    auto& ps = ContextAccess::st(*parent);
    bool pdone;
    {
      std::lock_guard<std::mutex> g(ps->mu);
      pdone = ps->done;
      if (!pdone) ps->children.push_back(c->st_);
      c->st_->deadline_ms = ps->deadline_ms;
    }
    if (pdone) cancel_state(c->st_, ps->err);
  }
  return c;
}

Ctx Context::with_timeout(const Ctx& parent, int64_t ms) {
  Ctx c = with_cancel(parent);
  const int64_t dl = mono_ms() + ms;
  {
    std::lock_guard<std::mutex> g(c->st_->mu);
    if (c->st_->deadline_ms < 0 || dl < c->st_->deadline_ms) c->st_->deadline_ms = dl;
  }
  return c;
}

void Context::cancel() { cancel_state(st_, "context canceled"); }

bool Context::done() const {
  std::unique_lock<std::mutex> g(st_->mu);
  if (st_->done) return true;
  if (st_->deadline_ms >= 0 && mono_ms() >= st_->deadline_ms) {
    g.unlock();
    cancel_state(st_, "context deadline exceeded");
    return true;
  }
  return false;
}

bool Context::wait(int64_t ms) const {
  const int64_t until = ms < 0 ? -1 : mono_ms() + ms;
  for (;;) {
    if (done()) return true;
    int64_t step = 20;
    {
      std::unique_lock<std::mutex> g(st_->mu);
      if (st_->deadline_ms >= 0) step = std::min<int64_t>(step, std::max<int64_t>(1, st_->deadline_ms - mono_ms()));
      if (until >= 0) {
        const int64_t left = until - mono_ms();
        if (left <= 0) return false;
        step = std::min(step, left);
      }
      st_->cv.wait_for(g, std::chrono::milliseconds(step), [&] { return st_->done; });
      if (st_->done) return true;
    }
  }
}

void Context::on_done(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(st_->mu);
    if (!st_->done) {
      st_->cbs.push_back(std::move(fn));
      return;
    }
  }
  fn();
}

std::string Context::err() const {
  done();
  std::lock_guard<std::mutex> g(st_->mu);
  return st_->err;
}

// ---------------------------------------------------------------- logging
static std::atomic<int> g_level{(int)LogLevel::kOff};  // zap global default: no-op
static std::mutex g_log_mu;
static std::deque<std::string> g_recent;

void log_set_level(LogLevel lv) { g_level.store((int)lv); }
LogLevel log_level() { return (LogLevel)g_level.load(); }

void log_write(LogLevel lv, const std::string& msg, const Fields& f) {
  static const char* names[] = {"DEBUG", "INFO", "WARN", "ERROR"};
  std::string line = std::string(names[(int)lv]) + "\t" + msg;
  for (const auto& kv : f) line += "\t" + kv.first + "=" + kv.second;
  std::lock_guard<std::mutex> g(g_log_mu);
  g_recent.push_back(line);
  if (g_recent.size() > 512) g_recent.pop_front();
  if ((int)lv >= g_level.load() && lv != LogLevel::kOff) fprintf(stderr, "%s\n", line.c_str());
}

std::vector<std::string> log_recent(size_t n) {
  std::lock_guard<std::mutex> g(g_log_mu);
  std::vector<std::string> out;
  const size_t start = g_recent.size() > n ? g_recent.size() - n : 0;
  for (size_t i = start; i < g_recent.size(); ++i) out.push_back(g_recent[i]);
  return out;
}

}  // namespace ptype
