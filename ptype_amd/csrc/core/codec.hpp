// Little-endian binary writer/reader for the control-plane wire protocol, the
// WAL and snapshots.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "util.hpp"

namespace ptype {

struct Writer {
  std::string buf;
  void u8(uint8_t v) { buf.push_back((char)v); }
  void u16(uint16_t v) { raw(&v, 2); }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void i64(int64_t v) { raw(&v, 8); }
  void f64(double v) { raw(&v, 8); }
  void b(bool v) { u8(v ? 1 : 0); }
  void str(const std::string& s) {
    u32((uint32_t)s.size());
    buf.append(s);
  }
  void strs(const std::vector<std::string>& v) {
    u32((uint32_t)v.size());
    for (const auto& s : v) str(s);
  }
  void raw(const void* p, size_t n) { buf.append((const char*)p, n); }
};

struct Reader {
  const char* p;
  size_t n, i = 0;
  Reader(const std::string& s) : p(s.data()), n(s.size()) {}
  Reader(const char* d, size_t len) : p(d), n(len) {}
  void need(size_t k) {
    if (i + k > n) fail(Errc::kGeneric, "codec: truncated message");
  }
  uint8_t u8() {
    need(1);
    return (uint8_t)p[i++];
  }
  template <class T>
  T pod() {
    need(sizeof(T));
    T v;
    memcpy(&v, p + i, sizeof(T));
    i += sizeof(T);
    return v;
  }
  uint16_t u16() { return pod<uint16_t>(); }
  uint32_t u32() { return pod<uint32_t>(); }
  uint64_t u64() { return pod<uint64_t>(); }
  int64_t i64() { return pod<int64_t>(); }
  double f64() { return pod<double>(); }
  bool b() { return u8() != 0; }
  std::string str() {
    uint32_t k = u32();
    need(k);
    std::string s(p + i, k);
    i += k;
    return s;
  }
  std::vector<std::string> strs() {
    uint32_t k = u32();
    std::vector<std::string> v;
    v.reserve(k);
    for (uint32_t j = 0; j < k; ++j) v.push_back(str());
    return v;
  }
  bool done() const { return i >= n; }
};

uint32_t crc32c(const void* data, size_t n, uint32_t crc = 0);

}  // namespace ptype
