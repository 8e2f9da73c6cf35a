#include "yaml.hpp"

#include <cctype>
#include <cstdlib>

#include "util.hpp"

namespace ptype {

bool YNode::is_null() const {
  if (kind == kNull) return true;
  if (kind != kScalar || quoted) return false;
  return scalar.empty() || scalar == "~" || scalar == "null" || scalar == "Null" || scalar == "NULL";
}

bool YNode::is_bool(bool* v) const {
  if (kind != kScalar || quoted) return false;
  static const char* t[] = {"true", "True", "TRUE", "yes", "Yes", "YES", "on", "On", "ON", "y", "Y"};
  static const char* f[] = {"false", "False", "FALSE", "no", "No", "NO", "off", "Off", "OFF", "n", "N"};
  for (auto s : t)
    if (scalar == s) {
      if (v) *v = true;
      return true;
    }
  for (auto s : f)
    if (scalar == s) {
      if (v) *v = false;
      return true;
    }
  return false;
}

bool YNode::is_int(long long* v) const {
  if (kind != kScalar || quoted || scalar.empty()) return false;
  const char* s = scalar.c_str();
  char* end = nullptr;
  int base = 10;
  if ((s[0] == '0' && (s[1] == 'x' || s[1] == 'X'))) base = 16;
  long long x = strtoll(s, &end, base);
  if (*end != 0) return false;
  if (v) *v = x;
  return true;
}

bool YNode::is_float(double* v) const {
  if (kind != kScalar || quoted || scalar.empty()) return false;
  if (is_int()) {
    if (v) *v = (double)strtoll(scalar.c_str(), nullptr, 0);
    return true;
  }
  char* end = nullptr;
  double x = strtod(scalar.c_str(), &end);
  if (*end != 0) return false;
  if (v) *v = x;
  return true;
}

std::string YNode::type_name() const {
  switch (kind) {
    case kNull:
      return "null";
    case kMap:
      return "object";
    case kSeq:
      return "array";
    case kScalar:
      if (quoted) return "string";
      if (is_null()) return "null";
      if (is_bool()) return "bool";
      if (is_float()) return "number";
      return "string";
  }
  return "string";
}

namespace {

struct Line {
  int indent;
  std::string text;  // without indentation / comments, trimmed right
  int no;
};

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
  }
  return s;
}

[[noreturn]] void syntax(int line, const std::string& what) {
  fail(Errc::kConfig, "yaml: line " + std::to_string(line) + ": " + what);
}

YNode parse_scalar_text(const std::string& raw, int line) {
  YNode n;
  std::string s = trim(raw);
  n.kind = YNode::kScalar;
  if (s.size() >= 2 && s[0] == '\'') {
    if (s.back() != '\'') syntax(line, "unterminated single-quoted scalar");
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
        out.push_back('\'');
        ++i;
      } else {
        out.push_back(s[i]);
      }
    }
    n.scalar = out;
    n.quoted = true;
  } else if (s.size() >= 2 && s[0] == '"') {
    if (s.back() != '"') syntax(line, "unterminated double-quoted scalar");
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\\' && i + 2 < s.size()) {
        char e = s[++i];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case '0': out.push_back('\0'); break;
          default: out.push_back(e);
        }
      } else {
        out.push_back(s[i]);
      }
    }
    n.scalar = out;
    n.quoted = true;
  } else if (!s.empty() && (s[0] == '\'' || s[0] == '"')) {
    syntax(line, "unterminated quoted scalar");
  } else {
    n.scalar = s;
  }
  return n;
}

// flow collections: [a, b] / {k: v}
YNode parse_flow(const std::string& s, size_t& i, int line);

void skip_ws(const std::string& s, size_t& i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
}

YNode parse_flow_item(const std::string& s, size_t& i, int line) {
  skip_ws(s, i);
  if (i < s.size() && (s[i] == '[' || s[i] == '{')) return parse_flow(s, i, line);
  size_t st = i;
  bool sq = false, dq = false;
  while (i < s.size()) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (!sq && !dq && (c == ',' || c == ']' || c == '}' || (c == ':' && i + 1 < s.size() && s[i + 1] == ' ')))
      break;
    ++i;
  }
  return parse_scalar_text(s.substr(st, i - st), line);
}

YNode parse_flow(const std::string& s, size_t& i, int line) {
  YNode n;
  const char open = s[i++];
  const char close = open == '[' ? ']' : '}';
  n.kind = open == '[' ? YNode::kSeq : YNode::kMap;
  for (;;) {
    skip_ws(s, i);
    if (i >= s.size()) syntax(line, "unterminated flow collection");
    if (s[i] == close) {
      ++i;
      return n;
    }
    if (n.kind == YNode::kSeq) {
      n.seq.push_back(parse_flow_item(s, i, line));
    } else {
      YNode k = parse_flow_item(s, i, line);
      skip_ws(s, i);
      if (i >= s.size() || s[i] != ':') syntax(line, "expected ':' in flow mapping");
      ++i;
      n.map.emplace_back(k.scalar, parse_flow_item(s, i, line));
    }
    skip_ws(s, i);
    if (i < s.size() && s[i] == ',') ++i;
  }
}

YNode parse_value_text(const std::string& v, int line) {
  std::string t = trim(v);
  if (!t.empty() && (t[0] == '[' || t[0] == '{')) {
    size_t i = 0;
    YNode n = parse_flow(t, i, line);
    skip_ws(t, i);
    if (i != t.size()) syntax(line, "trailing characters after flow collection");
    return n;
  }
  if (t.empty()) return YNode{};
  return parse_scalar_text(t, line);
}

// find "key: value" separator outside quotes; returns npos if not a mapping line
size_t find_colon(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == ':' && !sq && !dq && (i + 1 == s.size() || s[i + 1] == ' ' || s[i + 1] == '\t')) return i;
  }
  return std::string::npos;
}

class Parser {
 public:
  explicit Parser(std::vector<Line> lines) : L(std::move(lines)) {}

  YNode parse_block(int indent) {
    if (pos >= L.size()) return YNode{};
    if (starts_with(L[pos].text, "- ") || L[pos].text == "-") return parse_seq(L[pos].indent);
    return parse_map(L[pos].indent);
    (void)indent;
  }

 private:
  YNode parse_map(int indent) {
    YNode n;
    n.kind = YNode::kMap;
    while (pos < L.size() && L[pos].indent == indent) {
      const Line& ln = L[pos];
      if (starts_with(ln.text, "- ")) syntax(ln.no, "unexpected sequence item in mapping");
      size_t c = find_colon(ln.text);
      if (c == std::string::npos) syntax(ln.no, "could not find expected ':'");
      std::string key = parse_scalar_text(ln.text.substr(0, c), ln.no).scalar;
      std::string rest = trim(ln.text.substr(c + 1));
      ++pos;
      for (const auto& kv : n.map)
        if (kv.first == key) syntax(ln.no, "duplicate key \"" + key + "\"");
      if (rest.empty()) {
        if (pos < L.size() && (L[pos].indent > indent ||
                               (L[pos].indent == indent && (starts_with(L[pos].text, "- ") || L[pos].text == "-")))) {
          n.map.emplace_back(key, parse_block(L[pos].indent));
        } else {
          n.map.emplace_back(key, YNode{});
        }
      } else {
        n.map.emplace_back(key, parse_value_text(rest, ln.no));
      }
    }
    if (pos < L.size() && L[pos].indent > indent) syntax(L[pos].no, "bad indentation of a mapping entry");
    return n;
  }

  YNode parse_seq(int indent) {
    YNode n;
    n.kind = YNode::kSeq;
    while (pos < L.size() && L[pos].indent == indent && (starts_with(L[pos].text, "- ") || L[pos].text == "-")) {
      Line ln = L[pos];
      std::string rest = ln.text == "-" ? "" : trim(ln.text.substr(2));
      ++pos;
      if (rest.empty()) {
        if (pos < L.size() && L[pos].indent > indent)
          n.seq.push_back(parse_block(L[pos].indent));
        else
          n.seq.push_back(YNode{});
      } else if (find_colon(rest) != std::string::npos && rest[0] != '[' && rest[0] != '{' && rest[0] != '"' &&
                 rest[0] != '\'') {
        // "- key: value" starts an inline mapping whose further keys are indented
        const int item_indent = indent + 2;
        L.insert(L.begin() + pos, Line{item_indent, rest, ln.no});
        n.seq.push_back(parse_map(item_indent));
      } else {
        n.seq.push_back(parse_value_text(rest, ln.no));
      }
    }
    return n;
  }

  std::vector<Line> L;
  size_t pos = 0;
};

}  // namespace

YNode yaml_parse(const std::string& text) {
  std::vector<Line> lines;
  int no = 0;
  for (const auto& raw0 : split(text, '\n')) {
    ++no;
    std::string raw = raw0;
    if (!raw.empty() && raw.back() == '\r') raw.pop_back();
    if (raw == "---" || raw == "...") continue;
    std::string s = strip_comment(raw);
    std::string t = trim(s);
    if (t.empty()) continue;
    int ind = 0;
    while (ind < (int)s.size() && s[ind] == ' ') ++ind;
    if (ind < (int)s.size() && s[ind] == '\t') fail(Errc::kConfig, "yaml: line " + std::to_string(no) + ": found character that cannot start any token");
    lines.push_back(Line{ind, t, no});
  }
  if (lines.empty()) return YNode{};
  Parser p(lines);
  return p.parse_block(lines[0].indent);
}

}  // namespace ptype
