#include "gpupool/json.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace gpupool {

namespace {
constexpr int kMaxDepth = 256;
const std::string kEmpty;
}  // namespace

const Json& Json::null_ref() {
  static const Json n;
  return n;
}

Json::Json(const Json& o) : t_(o.t_), b_(o.b_), i_(o.i_), d_(o.d_), s_(o.s_) {
  if (o.arr_) arr_ = std::make_unique<Elements>(*o.arr_);
  if (o.obj_) obj_ = std::make_unique<Members>(*o.obj_);
}

Json& Json::operator=(const Json& o) {
  if (this == &o) return *this;
  Json tmp(o);
  *this = std::move(tmp);
  return *this;
}

Json Json::array() {
  Json j;
  j.t_ = Type::Array;
  j.arr_ = std::make_unique<Elements>();
  return j;
}

Json Json::object() {
  Json j;
  j.t_ = Type::Object;
  j.obj_ = std::make_unique<Members>();
  return j;
}

Json Json::array(std::initializer_list<Json> xs) {
  Json j = array();
  for (const auto& x : xs) j.arr_->push_back(x);
  return j;
}

int64_t Json::as_int(int64_t def) const {
  if (t_ == Type::Int) return i_;
  if (t_ == Type::Double && std::isfinite(d_)) return static_cast<int64_t>(d_);
  return def;
}

double Json::as_double(double def) const {
  if (t_ == Type::Double) return d_;
  if (t_ == Type::Int) return static_cast<double>(i_);
  return def;
}

const std::string& Json::as_string() const { return t_ == Type::String ? s_ : kEmpty; }

bool Json::contains(std::string_view key) const {
  if (t_ != Type::Object) return false;
  for (const auto& kv : *obj_)
    if (kv.first == key) return true;
  return false;
}

const Json& Json::operator[](std::string_view key) const {
  if (t_ != Type::Object) return null_ref();
  for (const auto& kv : *obj_)
    if (kv.first == key) return kv.second;
  return null_ref();
}

Json& Json::operator[](std::string_view key) {
  if (t_ == Type::Null) *this = object();
  if (t_ != Type::Object) throw JsonError("operator[](key) on non-object");
  for (auto& kv : *obj_)
    if (kv.first == key) return kv.second;
  obj_->emplace_back(std::string(key), Json());
  return obj_->back().second;
}

bool Json::erase(std::string_view key) {
  if (t_ != Type::Object) return false;
  for (auto it = obj_->begin(); it != obj_->end(); ++it) {
    if (it->first == key) {
      obj_->erase(it);
      return true;
    }
  }
  return false;
}

const Json::Members& Json::members() const {
  static const Members empty;
  return t_ == Type::Object ? *obj_ : empty;
}

Json::Members& Json::members() {
  if (t_ == Type::Null) *this = object();
  if (t_ != Type::Object) throw JsonError("members() on non-object");
  return *obj_;
}

size_t Json::size() const {
  if (t_ == Type::Array) return arr_->size();
  if (t_ == Type::Object) return obj_->size();
  return 0;
}

const Json& Json::operator[](size_t i) const {
  if (t_ != Type::Array || i >= arr_->size()) return null_ref();
  return (*arr_)[i];
}

Json& Json::at(size_t i) {
  if (t_ != Type::Array || i >= arr_->size()) throw JsonError("array index out of range");
  return (*arr_)[i];
}

void Json::push_back(Json v) {
  if (t_ == Type::Null) *this = array();
  if (t_ != Type::Array) throw JsonError("push_back on non-array");
  arr_->push_back(std::move(v));
}

const Json::Elements& Json::elements() const {
  static const Elements empty;
  return t_ == Type::Array ? *arr_ : empty;
}

Json::Elements& Json::elements() {
  if (t_ == Type::Null) *this = array();
  if (t_ != Type::Array) throw JsonError("elements() on non-array");
  return *arr_;
}

const Json& Json::path(std::string_view dotted) const {
  const Json* cur = this;
  size_t pos = 0;
  while (pos <= dotted.size()) {
    size_t dot = dotted.find('.', pos);
    std::string_view part = dotted.substr(pos, dot == std::string_view::npos ? dotted.npos : dot - pos);
    if (!part.empty()) {
      cur = &(*cur)[part];
      if (cur->is_null()) return null_ref();
    }
    if (dot == std::string_view::npos) break;
    pos = dot + 1;
  }
  return *cur;
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (t_ == Type::Int && o.t_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (t_ != o.t_) return false;
  switch (t_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *arr_ == *o.arr_;
    case Type::Object: {
      if (obj_->size() != o.obj_->size()) return false;
      for (const auto& kv : *obj_) {
        if (!o.contains(kv.first) || o[kv.first] != kv.second) return false;
      }
      return true;
    }
    default: return false;
  }
}

// ------------------------------------------------------------------ serialisation
std::string json_quote(std::string_view s) {
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
  return out;
}

static void newline(std::string& out, int indent, int depth) {
  if (indent < 0) return;
  out.push_back('\n');
  out.append(static_cast<size_t>(indent * depth), ' ');
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  switch (t_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: {
      if (!std::isfinite(d_)) {
        out += "null";
        break;
      }
      char buf[64];
      auto r = std::to_chars(buf, buf + sizeof buf, d_);
      std::string_view sv(buf, static_cast<size_t>(r.ptr - buf));
      out += sv;
      if (sv.find_first_of(".eE") == std::string_view::npos) out += ".0";
      break;
    }
    case Type::String: out += json_quote(s_); break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (const auto& e : *arr_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, depth + 1);
        e.dump_to(out, indent, depth + 1);
      }
      if (!arr_->empty()) newline(out, indent, depth);
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (const auto& kv : *obj_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, depth + 1);
        out += json_quote(kv.first);
        out += indent >= 0 ? ": " : ":";
        kv.second.dump_to(out, indent, depth + 1);
      }
      if (!obj_->empty()) newline(out, indent, depth);
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

// ------------------------------------------------------------------ parser
namespace {

class Parser {
 public:
  explicit Parser(std::string_view s) : s_(s) {}

  Json parse_document() {
    Json v = value(0);
    ws();
    if (p_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* what) {
    throw JsonError(std::string("json parse error at offset ") + std::to_string(p_) + ": " + what);
  }
  void ws() {
    while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\n' || s_[p_] == '\r' || s_[p_] == '\t')) ++p_;
  }
  bool eat(char c) {
    ws();
    if (p_ < s_.size() && s_[p_] == c) {
      ++p_;
      return true;
    }
    return false;
  }
  void expect_lit(const char* lit) {
    size_t n = std::strlen(lit);
    if (s_.substr(p_, n) != lit) fail("invalid literal");
    p_ += n;
  }

  Json value(int depth) {
    if (depth > kMaxDepth) fail("nesting too deep");
    ws();
    if (p_ >= s_.size()) fail("unexpected end");
    char c = s_[p_];
    if (c == '{') return object(depth);
    if (c == '[') return array(depth);
    if (c == '"') return Json(string());
    if (c == 't') {
      expect_lit("true");
      return Json(true);
    }
    if (c == 'f') {
      expect_lit("false");
      return Json(false);
    }
    if (c == 'n') {
      expect_lit("null");
      return Json();
    }
    if (c == '-' || (c >= '0' && c <= '9')) return number();
    fail("unexpected character");
  }

  Json object(int depth) {
    ++p_;
    Json o = Json::object();
    if (eat('}')) return o;
    for (;;) {
      ws();
      if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
      std::string k = string();
      if (!eat(':')) fail("expected ':'");
      Json v = value(depth + 1);
      o.members().emplace_back(std::move(k), std::move(v));
      if (eat(',')) continue;
      if (eat('}')) return o;
      fail("expected ',' or '}'");
    }
  }

  Json array(int depth) {
    ++p_;
    Json a = Json::array();
    if (eat(']')) return a;
    for (;;) {
      a.push_back(value(depth + 1));
      if (eat(',')) continue;
      if (eat(']')) return a;
      fail("expected ',' or ']'");
    }
  }

  unsigned hex4() {
    if (p_ + 4 > s_.size()) fail("short \\u escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = s_[p_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= static_cast<unsigned>(c - '0');
      else if (c >= 'a' && c <= 'f') v |= static_cast<unsigned>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= static_cast<unsigned>(c - 'A' + 10);
      else fail("bad hex digit");
    }
    return v;
  }

  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  std::string string() {
    ++p_;  // opening quote
    std::string out;
    for (;;) {
      if (p_ >= s_.size()) fail("unterminated string");
      char c = s_[p_++];
      if (c == '"') return out;
      if (static_cast<unsigned char>(c) < 0x20) fail("control character in string");
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (p_ >= s_.size()) fail("bad escape");
      char e = s_[p_++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (p_ + 2 <= s_.size() && s_[p_] == '\\' && s_[p_ + 1] == 'u') {
              p_ += 2;
              unsigned lo = hex4();
              if (lo < 0xDC00 || lo > 0xDFFF) fail("bad surrogate pair");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              fail("lone high surrogate");
            }
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            fail("lone low surrogate");
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }

  Json number() {
    size_t start = p_;
    bool is_float = false;
    if (s_[p_] == '-') ++p_;
    if (p_ >= s_.size()) fail("bad number");
    if (s_[p_] == '0') {
      ++p_;
    } else if (s_[p_] >= '1' && s_[p_] <= '9') {
      while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    } else {
      fail("bad number");
    }
    if (p_ < s_.size() && s_[p_] == '.') {
      is_float = true;
      ++p_;
      if (p_ >= s_.size() || s_[p_] < '0' || s_[p_] > '9') fail("bad fraction");
      while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    }
    if (p_ < s_.size() && (s_[p_] == 'e' || s_[p_] == 'E')) {
      is_float = true;
      ++p_;
      if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) ++p_;
      if (p_ >= s_.size() || s_[p_] < '0' || s_[p_] > '9') fail("bad exponent");
      while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    }
    const char* b = s_.data() + start;
    const char* e = s_.data() + p_;
    if (!is_float) {
      int64_t v = 0;
      auto r = std::from_chars(b, e, v);
      if (r.ec == std::errc() && r.ptr == e) return Json(static_cast<long long>(v));
    }
    std::string tmp(b, e);
    char* endp = nullptr;
    double d = std::strtod(tmp.c_str(), &endp);
    return Json(d);
  }

  std::string_view s_;
  size_t p_ = 0;
};

}  // namespace

Json Json::parse(std::string_view text) { return Parser(text).parse_document(); }

std::optional<Json> Json::try_parse(std::string_view text, std::string* err) {
  try {
    return Parser(text).parse_document();
  } catch (const JsonError& e) {
    if (err) *err = e.what();
    return std::nullopt;
  }
}

}  // namespace gpupool
