// Minimal JSON value (parse / dump) for registry Node values
// (`{"address":"<ip>","port":<int>}`, cluster/registry.go:23-26,52-53) and debug dumps.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <utility>
#include <vector>

namespace ptype {

struct JValue {
  enum Kind { kNull, kBool, kNumber, kString, kArray, kObject } kind = kNull;
  bool b = false;
  double num = 0;
  bool is_int = false;
  long long i = 0;
  std::string str;
  std::vector<JValue> arr;
  std::vector<std::pair<std::string, JValue>> obj;  // insertion order

  const JValue* get(const std::string& k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  static JValue string(const std::string& s) {
    JValue v;
    v.kind = kString;
    v.str = s;
    return v;
  }
  static JValue integer(long long x) {
    JValue v;
    v.kind = kNumber;
    v.is_int = true;
    v.i = x;
    v.num = (double)x;
    return v;
  }
};

JValue json_parse(const std::string& text);  // throws ptype::Error
std::string json_dump(const JValue& v);       // compact, Go encoding/json style
std::string json_quote(const std::string& s);

}  // namespace ptype
