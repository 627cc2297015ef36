// Minimal protobuf text-format reader for Caffe .prototxt files.
//
// No protoc / libprotobuf is assumed on the target (SURVEY.md §7 "hard
// parts"), so nets and solvers are parsed into a schema-less tree and the
// layers read the fields of caffe.proto they need (caffe.proto:102-297 for
// SolverParameter / FailurePatternParameter / FailureStrategyParameter, and
// the LayerParameter sub-messages).  Unknown fields are kept, not rejected,
// so every reference prototxt parses.
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace caffe {

class Msg;

struct Value {
  bool is_msg = false;
  bool quoted = false;      // scalar came from a "string literal"
  std::string scalar;       // raw token (number, enum identifier, string body)
  std::shared_ptr<Msg> msg;
};

class Msg {
 public:
  // ordered list of (field, value); repeated fields appear several times
  std::vector<std::pair<std::string, Value>> fields;

  bool has(const std::string& k) const;
  int count(const std::string& k) const;
  const Value* first(const std::string& k) const;
  std::vector<const Value*> all(const std::string& k) const;

  std::string str(const std::string& k, const std::string& def = "") const;
  double num(const std::string& k, double def = 0.0) const;
  long long integer(const std::string& k, long long def = 0) const;
  bool boolean(const std::string& k, bool def = false) const;
  std::vector<double> nums(const std::string& k) const;
  std::vector<std::string> strs(const std::string& k) const;
  const Msg* sub(const std::string& k) const;           // nullptr if absent
  std::vector<const Msg*> subs(const std::string& k) const;
  // helper: a sub-message or an empty message
  const Msg& sub_or_empty(const std::string& k) const;

  // mutation helpers (used for programmatic nets / overrides)
  void set(const std::string& k, const std::string& v, bool quoted = false);
  void add(const std::string& k, const std::string& v, bool quoted = false);  // repeated
  Msg& add_sub(const std::string& k);

  std::string debug_string(int indent = 0) const;
};

// Parse text-format; throws std::runtime_error with line/column on error.
Msg parse_prototxt(const std::string& text);
Msg parse_prototxt_file(const std::string& path);

}  // namespace caffe
