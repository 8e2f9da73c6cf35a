#include "json.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "util.hpp"

namespace ptype {

namespace {

struct P {
  const std::string& s;
  size_t i = 0;
  [[noreturn]] void err(const std::string& m) { fail("json: " + m + " at offset " + std::to_string(i)); }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  JValue value() {
    ws();
    if (i >= s.size()) err("unexpected end of input");
    char c = s[i];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return JValue::string(string());
    if (s.compare(i, 4, "true") == 0) {
      i += 4;
      JValue v;
      v.kind = JValue::kBool;
      v.b = true;
      return v;
    }
    if (s.compare(i, 5, "false") == 0) {
      i += 5;
      JValue v;
      v.kind = JValue::kBool;
      return v;
    }
    if (s.compare(i, 4, "null") == 0) {
      i += 4;
      return JValue{};
    }
    return number();
  }
  JValue number() {
    size_t st = i;
    if (i < s.size() && s[i] == '-') ++i;
    bool frac = false;
    while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                            s[i] == '+' || s[i] == '-')) {
      if (s[i] == '.' || s[i] == 'e' || s[i] == 'E') frac = true;
      ++i;
    }
    if (st == i) err("invalid character");
    std::string t = s.substr(st, i - st);
    JValue v;
    v.kind = JValue::kNumber;
    v.num = strtod(t.c_str(), nullptr);
    if (!frac) {
      v.is_int = true;
      v.i = strtoll(t.c_str(), nullptr, 10);
    }
    return v;
  }
  std::string string() {
    if (s[i] != '"') err("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        if (i >= s.size()) err("bad escape");
        char e = s[i++];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'u': {
            if (i + 4 > s.size()) err("bad \\u escape");
            unsigned cp = (unsigned)strtoul(s.substr(i, 4).c_str(), nullptr, 16);
            i += 4;
            if (cp < 0x80) {
              out.push_back((char)cp);
            } else if (cp < 0x800) {
              out.push_back((char)(0xC0 | (cp >> 6)));
              out.push_back((char)(0x80 | (cp & 0x3F)));
            } else {
              out.push_back((char)(0xE0 | (cp >> 12)));
              out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
              out.push_back((char)(0x80 | (cp & 0x3F)));
            }
            break;
          }
          default: out.push_back(e);
        }
      } else {
        out.push_back(c);
      }
    }
    if (i >= s.size()) err("unterminated string");
    ++i;
    return out;
  }
  JValue array() {
    JValue v;
    v.kind = JValue::kArray;
    ++i;
    ws();
    if (i < s.size() && s[i] == ']') {
      ++i;
      return v;
    }
    for (;;) {
      v.arr.push_back(value());
      ws();
      if (i < s.size() && s[i] == ',') {
        ++i;
        continue;
      }
      if (i < s.size() && s[i] == ']') {
        ++i;
        return v;
      }
      err("expected ',' or ']'");
    }
  }
  JValue object() {
    JValue v;
    v.kind = JValue::kObject;
    ++i;
    ws();
    if (i < s.size() && s[i] == '}') {
      ++i;
      return v;
    }
    for (;;) {
      ws();
      std::string k = string();
      ws();
      if (i >= s.size() || s[i] != ':') err("expected ':'");
      ++i;
      v.obj.emplace_back(k, value());
      ws();
      if (i < s.size() && s[i] == ',') {
        ++i;
        continue;
      }
      if (i < s.size() && s[i] == '}') {
        ++i;
        return v;
      }
      err("expected ',' or '}'");
    }
  }
};

}  // namespace

JValue json_parse(const std::string& text) {
  P p{text};
  JValue v = p.value();
  p.ws();
  if (p.i != text.size()) p.err("invalid character after top-level value");
  return v;
}

std::string json_quote(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '<': o += "\\u003c"; break;  // Go escapes HTML-sensitive characters
      case '>': o += "\\u003e"; break;
      case '&': o += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o.push_back((char)c);
        }
    }
  }
  return o + "\"";
}

std::string json_dump(const JValue& v) {
  switch (v.kind) {
    case JValue::kNull:
      return "null";
    case JValue::kBool:
      return v.b ? "true" : "false";
    case JValue::kNumber: {
      if (v.is_int) return std::to_string(v.i);
      char b[64];
      snprintf(b, sizeof b, "%.17g", v.num);
      return b;
    }
    case JValue::kString:
      return json_quote(v.str);
    case JValue::kArray: {
      std::string o = "[";
      for (size_t k = 0; k < v.arr.size(); ++k) o += (k ? "," : "") + json_dump(v.arr[k]);
      return o + "]";
    }
    case JValue::kObject: {
      std::string o = "{";
      for (size_t k = 0; k < v.obj.size(); ++k)
        o += (k ? "," : "") + json_quote(v.obj[k].first) + ":" + json_dump(v.obj[k].second);
      return o + "}";
    }
  }
  return "null";
}

}  // namespace ptype
