// Minimal JSON DOM for the gpupool control plane (no third-party deps).
//
// Objects keep insertion order (k8s objects round-trip stably, diffs stay readable).
// The parser is recursive-descent with a depth limit, so hostile input (watch streams, agent
// replies) cannot blow the stack; it is fuzzed under ASan/UBSan in native/tests.
#pragma once

#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace gpupool {

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using Members = std::vector<std::pair<std::string, Json>>;
  using Elements = std::vector<Json>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : t_(Type::Bool), b_(b) {}
  Json(int v) : t_(Type::Int), i_(v) {}
  Json(long v) : t_(Type::Int), i_(v) {}
  Json(long long v) : t_(Type::Int), i_(v) {}
  Json(unsigned v) : t_(Type::Int), i_(v) {}
  Json(unsigned long v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(unsigned long long v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(double v) : t_(Type::Double), d_(v) {}
  Json(const char* s) : t_(Type::String), s_(s) {}
  Json(std::string s) : t_(Type::String), s_(std::move(s)) {}
  Json(std::string_view s) : t_(Type::String), s_(s) {}

  Json(const Json& o);
  Json(Json&& o) noexcept = default;
  Json& operator=(const Json& o);
  Json& operator=(Json&& o) noexcept = default;
  ~Json() = default;

  static Json array();
  static Json object();
  static Json array(std::initializer_list<Json> xs);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_int() const { return t_ == Type::Int; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::Double; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  bool as_bool(bool def = false) const { return t_ == Type::Bool ? b_ : def; }
  int64_t as_int(int64_t def = 0) const;
  double as_double(double def = 0) const;
  const std::string& as_string() const;  // "" if not a string
  std::string str_or(const std::string& def) const { return t_ == Type::String ? s_ : def; }

  // ---- object access
  bool contains(std::string_view key) const;
  const Json& operator[](std::string_view key) const;  // null Json if missing / not object
  Json& operator[](std::string_view key);              // inserts; null -> object
  const Json& operator[](const char* key) const { return (*this)[std::string_view(key)]; }
  Json& operator[](const char* key) { return (*this)[std::string_view(key)]; }
  const Json& operator[](const std::string& key) const { return (*this)[std::string_view(key)]; }
  Json& operator[](const std::string& key) { return (*this)[std::string_view(key)]; }
  Json& set(std::string_view key, Json v) {
    (*this)[key] = std::move(v);
    return *this;
  }
  bool erase(std::string_view key);
  const Members& members() const;
  Members& members();

  // ---- array access
  size_t size() const;
  const Json& operator[](size_t i) const;
  const Json& operator[](int i) const { return (*this)[static_cast<size_t>(i)]; }
  // Non-const int index: read-only (use at() to mutate); avoids 0 -> const char* ambiguity.
  const Json& operator[](int i) { return static_cast<const Json&>(*this)[static_cast<size_t>(i)]; }
  Json& at(size_t i);
  void push_back(Json v);
  const Elements& elements() const;
  Elements& elements();

  // Dotted-path lookup: path("metadata.name"); missing -> null.
  const Json& path(std::string_view dotted) const;

  std::string dump(int indent = -1) const;
  static Json parse(std::string_view text);
  static std::optional<Json> try_parse(std::string_view text, std::string* err = nullptr);

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

  static const Json& null_ref();

 private:
  void dump_to(std::string& out, int indent, int depth) const;
  Type t_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::unique_ptr<Elements> arr_;
  std::unique_ptr<Members> obj_;
};

// JSON-escape a string (with surrounding quotes).
std::string json_quote(std::string_view s);

}  // namespace gpupool
