// YAML-subset parser for the two configuration layers.
//
// Covers what the reference's configs use and what sigs.k8s.io/yaml / etcd's
// configYAML accept in practice: block mappings and sequences by indentation,
// flow sequences/maps, plain / single- / double-quoted scalars, comments.
// Scalars keep their source form (`quoted`) so the typed decoders can apply the
// YAML->JSON typing that Go's sigs.k8s.io/yaml performs (an unquoted `5` is a
// number and cannot decode into a string field -- cluster/testdata/bad_config.yml).
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace ptype {

struct YNode {
  enum Kind { kNull, kScalar, kMap, kSeq } kind = kNull;
  std::string scalar;
  bool quoted = false;
  std::vector<std::pair<std::string, YNode>> map;
  std::vector<YNode> seq;

  const YNode* get(const std::string& k) const {
    for (const auto& kv : map)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  // YAML 1.1 core typing of an unquoted scalar
  bool is_null() const;
  bool is_bool(bool* v = nullptr) const;
  bool is_int(long long* v = nullptr) const;
  bool is_float(double* v = nullptr) const;
  std::string type_name() const;  // "string" / "number" / "bool" / "null" / "object" / "array"
};

// Throws ptype::Error(kConfig) with a line number on syntax errors.
YNode yaml_parse(const std::string& text);

}  // namespace ptype
