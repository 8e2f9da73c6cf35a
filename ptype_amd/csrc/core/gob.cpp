#include "gob.hpp"

#include <string.h>

#include "util.hpp"

namespace ptype {
namespace gob {

void put_uint(std::string* b, uint64_t x) {
  if (x < 128) {
    b->push_back((char)x);
    return;
  }
  unsigned char tmp[8];
  int n = 0;
  while (x) {
    tmp[n++] = (unsigned char)(x & 0xff);
    x >>= 8;
  }
  b->push_back((char)(unsigned char)(256 - n));  // -(byte count)
  for (int i = n - 1; i >= 0; --i) b->push_back((char)tmp[i]);
}

void put_int(std::string* b, int64_t i) {
  const uint64_t x = i < 0 ? ((uint64_t)(~i) << 1) | 1 : (uint64_t)i << 1;
  put_uint(b, x);
}

static void put_string(std::string* b, const std::string& s) {
  put_uint(b, s.size());
  b->append(s);
}

static uint64_t float_bits(double f) {
  uint64_t u;
  memcpy(&u, &f, 8);
  return __builtin_bswap64(u);
}

std::string Value::debug() const {
  switch (kind) {
    case kNil: return "nil";
    case kBool: return b ? "true" : "false";
    case kInt: return std::to_string(i);
    case kUint: return std::to_string(u);
    case kFloat: return std::to_string(f);
    case kBytes: return "bytes(" + std::to_string(s.size()) + ")";
    case kString: return "\"" + s + "\"";
    case kStruct: {
      std::string o = type_name + "{";
      for (size_t k = 0; k < fields.size(); ++k) o += (k ? " " : "") + fields[k].first + ":" + fields[k].second.debug();
      return o + "}";
    }
    case kSlice: {
      std::string o = "[";
      for (size_t k = 0; k < elems.size(); ++k) o += (k ? " " : "") + elems[k].debug();
      return o + "]";
    }
    case kMap: return "map(" + std::to_string(entries.size()) + ")";
  }
  return "?";
}

// ------------------------------------------------------------------ encoder
static std::string signature(const Value& v);

static std::string signature(const Value& v) {
  switch (v.kind) {
    case kBool: return "bool";
    case kInt: return "int";
    case kUint: return "uint";
    case kFloat: return "float64";
    case kBytes: return "[]byte";
    case kString: return "string";
    case kStruct: {
      std::string s = "struct " + v.type_name + "{";
      for (const auto& f : v.fields) s += f.first + " " + signature(f.second) + ";";
      return s + "}";
    }
    case kSlice: {
      const Value* e = !v.elems.empty() ? &v.elems[0] : (!v.elem_proto.empty() ? &v.elem_proto[0] : nullptr);
      if (!e) fail("gob: cannot encode a slice with unknown element type");
      return "[]" + signature(*e);
    }
    case kMap: {
      const Value* k = !v.entries.empty() ? &v.entries[0].first : (!v.key_proto.empty() ? &v.key_proto[0] : nullptr);
      const Value* e = !v.entries.empty() ? &v.entries[0].second : (!v.elem_proto.empty() ? &v.elem_proto[0] : nullptr);
      if (!k || !e) fail("gob: cannot encode a map with unknown key/element type");
      return "map[" + signature(*k) + "]" + signature(*e);
    }
    default: fail("gob: cannot encode nil");
  }
}

static std::string go_name(const Value& v) {
  switch (v.kind) {
    case kStruct: return v.type_name.empty() ? signature(v) : v.type_name;
    case kSlice: {
      const Value& e = !v.elems.empty() ? v.elems[0] : v.elem_proto[0];
      return "[]" + go_name(e);
    }
    case kMap: {
      const Value& k = !v.entries.empty() ? v.entries[0].first : v.key_proto[0];
      const Value& e = !v.entries.empty() ? v.entries[0].second : v.elem_proto[0];
      return "map[" + go_name(k) + "]" + go_name(e);
    }
    default: return signature(v);
  }
}

namespace {
struct Pending {
  std::vector<std::string> defs;  // in Go's send order: a type, then its inner types
};
}  // namespace

static int builtin_id(Kind k) {
  switch (k) {
    case kBool: return kTBool;
    case kInt: return kTInt;
    case kUint: return kTUint;
    case kFloat: return kTFloat;
    case kBytes: return kTBytes;
    case kString: return kTString;
    default: return 0;
  }
}

int Encoder::type_id(const Value& v, std::string* out) {
  if (int b = builtin_id(v.kind)) return b;
  const std::string sig = signature(v);
  auto it = ids_.find(sig);
  if (it != ids_.end()) return it->second;
  const int id = next_++;
  ids_[sig] = id;
  // build this type's definition after assigning ids to its inner types, but
  // emit it BEFORE their definitions (Go's sendType order)
  std::string inner;
  std::string def;  // wireType value
  if (v.kind == kStruct) {
    std::vector<std::pair<std::string, int>> fids;
    for (const auto& f : v.fields) fids.emplace_back(f.first, type_id(f.second, &inner));
    std::string st;  // structType
    st.push_back(1);  // field 0: CommonType
    {
      const std::string name = go_name(v);
      if (!name.empty()) {
        st.push_back(1);
        put_string(&st, name);
        st.push_back(1);
      } else {
        st.push_back(2);
      }
      put_int(&st, id);
      st.push_back(0);
    }
    if (!fids.empty()) {
      st.push_back(1);  // field 1: Field []*fieldType
      put_uint(&st, fids.size());
      for (const auto& f : fids) {
        st.push_back(1);
        put_string(&st, f.first);
        st.push_back(1);
        put_int(&st, f.second);
        st.push_back(0);
      }
    }
    st.push_back(0);
    def.push_back(3);  // wireType field 2: StructT
    def += st;
    def.push_back(0);
  } else if (v.kind == kSlice) {
    const Value& e = !v.elems.empty() ? v.elems[0] : v.elem_proto[0];
    const int eid = type_id(e, &inner);
    std::string st;
    st.push_back(1);
    st.push_back(1);
    put_string(&st, go_name(v));
    st.push_back(1);
    put_int(&st, id);
    st.push_back(0);
    st.push_back(1);
    put_int(&st, eid);
    st.push_back(0);
    def.push_back(2);  // wireType field 1: SliceT
    def += st;
    def.push_back(0);
  } else if (v.kind == kMap) {
    const Value& k = !v.entries.empty() ? v.entries[0].first : v.key_proto[0];
    const Value& e = !v.entries.empty() ? v.entries[0].second : v.elem_proto[0];
    const int kid = type_id(k, &inner);
    const int eid = type_id(e, &inner);
    std::string st;
    st.push_back(1);
    st.push_back(1);
    put_string(&st, go_name(v));
    st.push_back(1);
    put_int(&st, id);
    st.push_back(0);
    st.push_back(1);
    put_int(&st, kid);
    st.push_back(1);
    put_int(&st, eid);
    st.push_back(0);
    def.push_back(4);  // wireType field 3: MapT
    def += st;
    def.push_back(0);
  } else {
    fail("gob: unsupported type");
  }
  std::string msg;
  put_int(&msg, -id);
  msg += def;
  std::string framed;
  put_uint(&framed, msg.size());
  framed += msg;
  out->append(framed);
  out->append(inner);
  return id;
}

static bool is_zero(const Value& v) {
  switch (v.kind) {
    case kBool: return !v.b;
    case kInt: return v.i == 0;
    case kUint: return v.u == 0;
    case kFloat: return v.f == 0;
    case kBytes:
    case kString: return v.s.empty();
    case kSlice: return v.elems.empty();
    case kMap: return v.entries.empty();
    case kNil: return true;
    default: return false;  // structs are always sent
  }
}

void Encoder::encode_value(const Value& v, std::string* b) {
  switch (v.kind) {
    case kBool: put_uint(b, v.b ? 1 : 0); break;
    case kInt: put_int(b, v.i); break;
    case kUint: put_uint(b, v.u); break;
    case kFloat: put_uint(b, float_bits(v.f)); break;
    case kBytes:
    case kString: put_string(b, v.s); break;
    case kStruct: encode_struct(v, b); break;
    case kSlice:
      put_uint(b, v.elems.size());
      for (const auto& e : v.elems) encode_value(e, b);
      break;
    case kMap:
      put_uint(b, v.entries.size());
      for (const auto& kv : v.entries) {
        encode_value(kv.first, b);
        encode_value(kv.second, b);
      }
      break;
    default: fail("gob: cannot encode nil value");
  }
}

void Encoder::encode_struct(const Value& v, std::string* b) {
  int last = -1;
  for (size_t k = 0; k < v.fields.size(); ++k) {
    const Value& f = v.fields[k].second;
    if (is_zero(f)) continue;
    put_uint(b, (uint64_t)((int)k - last));
    last = (int)k;
    encode_value(f, b);
  }
  b->push_back(0);
}

void Encoder::encode(const Value& v, std::string* out) {
  const int id = type_id(v, out);
  std::string msg;
  put_int(&msg, id);
  if (v.kind == kStruct) {
    encode_struct(v, &msg);
  } else {
    msg.push_back(0);  // singleton: field delta 0
    encode_value(v, &msg);
  }
  put_uint(out, msg.size());
  out->append(msg);
}

// ------------------------------------------------------------------ decoder
uint64_t Decoder::get_uint() {
  unsigned char c;
  if (remaining_ < 1 || !read_((char*)&c, 1)) fail(Errc::kRpc, "gob: unexpected EOF");
  --remaining_;
  if (c < 128) return c;
  const int n = 256 - c;
  if (n > 8 || remaining_ < (size_t)n) fail(Errc::kRpc, "gob: bad uint");
  unsigned char buf[8];
  if (!read_((char*)buf, n)) fail(Errc::kRpc, "gob: unexpected EOF");
  remaining_ -= n;
  uint64_t x = 0;
  for (int i = 0; i < n; ++i) x = (x << 8) | buf[i];
  return x;
}

int64_t Decoder::get_int() {
  const uint64_t x = get_uint();
  if (x & 1) return ~(int64_t)(x >> 1);
  return (int64_t)(x >> 1);
}

std::string Decoder::get_bytes() {
  const uint64_t n = get_uint();
  if (n > remaining_) fail(Errc::kRpc, "gob: string length exceeds message");
  std::string s(n, '\0');
  if (n && !read_(&s[0], n)) fail(Errc::kRpc, "gob: unexpected EOF");
  remaining_ -= n;
  return s;
}

void Decoder::skip_remaining() {
  char buf[256];
  while (remaining_) {
    const size_t k = std::min(remaining_, sizeof buf);
    if (!read_(buf, k)) fail(Errc::kRpc, "gob: unexpected EOF");
    remaining_ -= k;
  }
}

Decoder::WireType Decoder::decode_wiretype() {
  WireType wt;
  auto common = [&]() {
    int f = -1;
    for (;;) {
      uint64_t d = get_uint();
      if (!d) break;
      f += (int)d;
      if (f == 0) wt.name = get_bytes();
      else if (f == 1) get_int();  // our own id; the message id is authoritative
      else fail(Errc::kRpc, "gob: bad CommonType");
    }
  };
  int field = -1;
  for (;;) {
    const uint64_t d = get_uint();
    if (!d) break;
    field += (int)d;
    int f = -1;
    switch (field) {
      case 0:  // ArrayT
        wt.kind = 4;
        for (;;) {
          uint64_t dd = get_uint();
          if (!dd) break;
          f += (int)dd;
          if (f == 0) common();
          else if (f == 1) wt.elem = (int)get_int();
          else if (f == 2) wt.len = get_int();
        }
        break;
      case 1:  // SliceT
        wt.kind = 2;
        for (;;) {
          uint64_t dd = get_uint();
          if (!dd) break;
          f += (int)dd;
          if (f == 0) common();
          else if (f == 1) wt.elem = (int)get_int();
        }
        break;
      case 2:  // StructT
        wt.kind = 1;
        for (;;) {
          uint64_t dd = get_uint();
          if (!dd) break;
          f += (int)dd;
          if (f == 0) {
            common();
          } else if (f == 1) {
            const uint64_t n = get_uint();
            for (uint64_t k = 0; k < n; ++k) {
              std::string name;
              int fid = 0, ff = -1;
              for (;;) {
                uint64_t d3 = get_uint();
                if (!d3) break;
                ff += (int)d3;
                if (ff == 0) name = get_bytes();
                else if (ff == 1) fid = (int)get_int();
              }
              wt.fields.emplace_back(name, fid);
            }
          }
        }
        break;
      case 3:  // MapT
        wt.kind = 3;
        for (;;) {
          uint64_t dd = get_uint();
          if (!dd) break;
          f += (int)dd;
          if (f == 0) common();
          else if (f == 1) wt.key = (int)get_int();
          else if (f == 2) wt.elem = (int)get_int();
        }
        break;
      default:
        fail(Errc::kRpc, "gob: GobEncoder/Marshaler types are not supported");
    }
  }
  return wt;
}

Value Decoder::zero_of(int id) {
  Value v;
  switch (id) {
    case kTBool: v.kind = kBool; return v;
    case kTInt: v.kind = kInt; return v;
    case kTUint: v.kind = kUint; return v;
    case kTFloat: v.kind = kFloat; return v;
    case kTBytes: v.kind = kBytes; return v;
    case kTString: v.kind = kString; return v;
  }
  auto it = types_.find(id);
  if (it == types_.end()) return v;
  const WireType& wt = it->second;
  if (wt.kind == 1) {
    v.kind = kStruct;
    v.type_name = wt.name;
    for (const auto& f : wt.fields) v.fields.emplace_back(f.first, f.second == id ? Value{} : zero_of(f.second));
  } else if (wt.kind == 2 || wt.kind == 4) {
    v.kind = kSlice;
  } else if (wt.kind == 3) {
    v.kind = kMap;
  }
  return v;
}

void Decoder::decode_struct(int id, Value* v) {
  *v = zero_of(id);
  const WireType& wt = types_.at(id);
  int field = -1;
  for (;;) {
    const uint64_t d = get_uint();
    if (!d) break;
    field += (int)d;
    if (field < 0 || field >= (int)wt.fields.size()) fail(Errc::kRpc, "gob: field number out of range");
    decode_typed(wt.fields[field].second, &v->fields[field].second);
  }
}

void Decoder::decode_typed(int id, Value* v) {
  switch (id) {
    case kTBool: v->kind = kBool; v->b = get_uint() != 0; return;
    case kTInt: v->kind = kInt; v->i = get_int(); return;
    case kTUint: v->kind = kUint; v->u = get_uint(); return;
    case kTFloat: {
      v->kind = kFloat;
      uint64_t u = __builtin_bswap64(get_uint());
      memcpy(&v->f, &u, 8);
      return;
    }
    case kTBytes: v->kind = kBytes; v->s = get_bytes(); return;
    case kTString: v->kind = kString; v->s = get_bytes(); return;
  }
  auto it = types_.find(id);
  if (it == types_.end()) fail(Errc::kRpc, "gob: unknown type id " + std::to_string(id));
  const WireType wt = it->second;
  if (wt.kind == 1) {
    decode_struct(id, v);
  } else if (wt.kind == 2 || wt.kind == 4) {
    v->kind = kSlice;
    const uint64_t n = get_uint();
    if (n > remaining_) fail(Errc::kRpc, "gob: slice length exceeds message");
    v->elems.resize(n);
    for (auto& e : v->elems) decode_typed(wt.elem, &e);
  } else if (wt.kind == 3) {
    v->kind = kMap;
    const uint64_t n = get_uint();
    if (n > remaining_) fail(Errc::kRpc, "gob: map length exceeds message");
    v->entries.resize(n);
    for (auto& kv : v->entries) {
      decode_typed(wt.key, &kv.first);
      decode_typed(wt.elem, &kv.second);
    }
  } else {
    fail(Errc::kRpc, "gob: unsupported wire type");
  }
}

bool Decoder::decode(Value* out) {
  for (;;) {
    // message length (a uint) -- EOF before it is a clean end of stream
    unsigned char c;
    if (!read_((char*)&c, 1)) return false;
    uint64_t len;
    if (c < 128) {
      len = c;
    } else {
      const int n = 256 - c;
      if (n > 8) fail(Errc::kRpc, "gob: bad message length");
      unsigned char buf[8];
      if (!read_((char*)buf, n)) fail(Errc::kRpc, "gob: unexpected EOF");
      len = 0;
      for (int i = 0; i < n; ++i) len = (len << 8) | buf[i];
    }
    if (len > (1u << 28)) fail(Errc::kRpc, "gob: message too large");
    remaining_ = len;
    const int64_t id = get_int();
    if (id < 0) {
      types_[(int)-id] = decode_wiretype();
      skip_remaining();
      continue;
    }
    auto it = types_.find((int)id);
    if (it != types_.end() && it->second.kind == 1) {
      decode_struct((int)id, out);
    } else {
      if (get_uint() != 0) fail(Errc::kRpc, "gob: non-struct value without singleton delta");
      decode_typed((int)id, out);
    }
    skip_remaining();
    return true;
  }
}

namespace {
// Reads from an in-memory message while a Decoder parses it, then restores its source.
struct ReadSwap {
  std::function<bool(char*, size_t)>& slot;
  std::function<bool(char*, size_t)> saved;
  ReadSwap(std::function<bool(char*, size_t)>& s, const std::string& buf, size_t* pos) : slot(s), saved(std::move(s)) {
    slot = [&buf, pos](char* p, size_t n) {
      if (*pos + n > buf.size()) return false;
      memcpy(p, buf.data() + *pos, n);
      *pos += n;
      return true;
    };
  }
  ~ReadSwap() { slot = std::move(saved); }
};
}  // namespace

bool Decoder::next_raw(std::string* raw, int64_t* type_id) {
  for (;;) {
    raw->clear();
    unsigned char c;
    if (!read_((char*)&c, 1)) return false;
    raw->push_back((char)c);
    uint64_t len;
    if (c < 128) {
      len = c;
    } else {
      const int n = 256 - c;
      if (n > 8) fail(Errc::kRpc, "gob: bad message length");
      unsigned char buf[8];
      if (!read_((char*)buf, n)) fail(Errc::kRpc, "gob: unexpected EOF");
      len = 0;
      for (int i = 0; i < n; ++i) {
        len = (len << 8) | buf[i];
        raw->push_back((char)buf[i]);
      }
    }
    if (len > (1u << 28)) fail(Errc::kRpc, "gob: message too large");
    const size_t hdr = raw->size();
    raw->resize(hdr + len);
    if (len && !read_(&(*raw)[hdr], len)) fail(Errc::kRpc, "gob: unexpected EOF");
    size_t pos = hdr;
    int64_t id;
    {
      ReadSwap swap(read_, *raw, &pos);
      remaining_ = len;
      id = get_int();
      if (id < 0) {
        types_[(int)-id] = decode_wiretype();
        skip_remaining();
      }
      remaining_ = 0;
    }
    if (id < 0) continue;
    *type_id = id;
    return true;
  }
}

void Decoder::decode_raw(const std::string& raw, Value* out) {
  size_t pos = 0;
  ReadSwap swap(read_, raw, &pos);
  if (!decode(out)) fail(Errc::kRpc, "gob: empty message");
}

bool Decoder::int_struct_fields(int64_t type_id, std::vector<std::string>* names) const {
  auto it = types_.find((int)type_id);
  if (it == types_.end() || it->second.kind != 1) return false;
  names->clear();
  for (const auto& f : it->second.fields) {
    // only gob's predefined int (kTInt = 2): the device decoders zigzag every
    // field, which is wrong for uint (3); 7 is complex (two uints), not uint
    if (f.second != kTInt) return false;
    names->push_back(f.first);
  }
  return !names->empty();
}

}  // namespace gob
}  // namespace ptype
