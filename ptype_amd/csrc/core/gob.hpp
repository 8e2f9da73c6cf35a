// Go encoding/gob subset codec: enough of gob to
// speak stdlib net/rpc with a real Go peer -- the reference's data-plane wire
// format (cluster/rpc.go:65,88,277; example/calculator/calculator.go:3-12).
//
// Supported: bool, int, uint, float64, string, []byte, named/unnamed structs,
// slices, maps of those; type definitions are sent once per stream before the
// first value of a type (ids from 65), zero-valued struct fields are omitted,
// non-struct top-level values use the singleton form (delta 0).  Interfaces,
// complex numbers, arrays and GobEncoder types are rejected.
#pragma once
#include <stdint.h>

#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace ptype {
namespace gob {

enum Kind : uint8_t { kNil = 0, kBool, kInt, kUint, kFloat, kBytes, kString, kStruct, kSlice, kMap };

struct Value {
  Kind kind = kNil;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double f = 0;
  std::string s;                                      // string / bytes
  std::string type_name;                              // struct: Go type name ("" = anonymous)
  std::vector<std::pair<std::string, Value>> fields;  // struct fields, declaration order
  std::vector<Value> elems;                           // slice elements
  std::vector<std::pair<Value, Value>> entries;       // map
  // element / key types, needed for empty slices and maps
  std::vector<Value> elem_proto;                      // [0] = prototype of the element (slice/map value)
  std::vector<Value> key_proto;                       // [0] = prototype of the map key

  static Value Int(int64_t v) { Value x; x.kind = kInt; x.i = v; return x; }
  static Value Uint(uint64_t v) { Value x; x.kind = kUint; x.u = v; return x; }
  static Value Bool(bool v) { Value x; x.kind = kBool; x.b = v; return x; }
  static Value Float(double v) { Value x; x.kind = kFloat; x.f = v; return x; }
  static Value String(const std::string& v) { Value x; x.kind = kString; x.s = v; return x; }
  static Value Bytes(const std::string& v) { Value x; x.kind = kBytes; x.s = v; return x; }
  static Value Struct(const std::string& name) { Value x; x.kind = kStruct; x.type_name = name; return x; }
  const Value* field(const std::string& n) const {
    for (const auto& f : fields)
      if (f.first == n) return &f.second;
    return nullptr;
  }
  std::string debug() const;
};

// Builtin type ids.
enum : int { kTBool = 1, kTInt = 2, kTUint = 3, kTFloat = 4, kTBytes = 5, kTString = 6, kFirstUserId = 65 };

// Low-level primitives (exposed for golden-byte tests).
void put_uint(std::string* b, uint64_t x);
void put_int(std::string* b, int64_t x);

class Encoder {
 public:
  // Appends every message needed for `v` (type definitions first) to *out.
  void encode(const Value& v, std::string* out);

 private:
  int type_id(const Value& v, std::string* out);
  void encode_value(const Value& v, std::string* b);
  void encode_struct(const Value& v, std::string* b);
  std::map<std::string, int> ids_;
  int next_ = kFirstUserId;
};

class Decoder {
 public:
  // `read(p, n)` must fill exactly n bytes or return false (EOF).
  explicit Decoder(std::function<bool(char*, size_t)> read) : read_(std::move(read)) {}
  // Reads messages until one value is complete; consumes type definitions on the way.
  bool decode(Value* out);
  // The next VALUE message undecoded (its length prefix included) and its type
  // id; type definitions on the way are consumed (K4: a batch of such messages
  // is decoded on the GPU).  False at a clean end of stream.
  bool next_raw(std::string* raw, int64_t* type_id);
  // Decode a message captured by next_raw (host fallback for one message).
  void decode_raw(const std::string& raw, Value* out);
  // Field names of a received struct type in wire order, when every field is a
  // (signed / unsigned) integer; false otherwise.
  bool int_struct_fields(int64_t type_id, std::vector<std::string>* names) const;

 private:
  struct WireType {
    int kind = 0;  // 1 struct, 2 slice, 3 map, 4 array
    std::string name;
    std::vector<std::pair<std::string, int>> fields;
    int elem = 0, key = 0;
    int64_t len = 0;
  };
  uint64_t get_uint();
  int64_t get_int();
  std::string get_bytes();
  void decode_typed(int id, Value* v);
  void decode_struct(int id, Value* v);
  WireType decode_wiretype();
  void skip_remaining();
  Value zero_of(int id);
  std::function<bool(char*, size_t)> read_;
  std::map<int, WireType> types_;
  size_t remaining_ = 0;  // bytes left in the current message
};

}  // namespace gob
}  // namespace ptype
