#include "gpupool/yaml.h"

#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <vector>

namespace gpupool {

namespace {

struct Line {
  int indent;
  std::string text;  // without indentation, comments or trailing blanks
  int no;            // 1-based source line
  std::string raw;   // original line (block scalars keep their inner indentation)
};

[[noreturn]] void fail(int no, const std::string& what) {
  throw YamlError("yaml line " + std::to_string(no) + ": " + what);
}

// Cuts a " #" comment that is not inside quotes.
std::string strip_comment(const std::string& s) {
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (q) {
      if (c == q) {
        if (q == '\'' && i + 1 < s.size() && s[i + 1] == '\'') ++i;  // '' escape
        else q = 0;
      } else if (q == '"' && c == '\\') {
        ++i;
      }
    } else if (c == '\'' || c == '"') {
      if (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t' || s[i - 1] == ':' || s[i - 1] == '[' ||
          s[i - 1] == '{' || s[i - 1] == ',' || s[i - 1] == '-')
        q = c;
    } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
      return s.substr(0, i);
    }
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t");
  if (a == std::string::npos) return "";
  return rtrim(s.substr(a));
}

void append_utf8(std::string& out, unsigned cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

// Parses a quoted scalar starting at s[i] (the quote); advances i past the closing quote.
std::string quoted(const std::string& s, size_t& i, int no) {
  char q = s[i++];
  std::string out;
  while (i < s.size()) {
    char c = s[i++];
    if (c == q) {
      if (q == '\'' && i < s.size() && s[i] == '\'') {
        out.push_back('\'');
        ++i;
        continue;
      }
      return out;
    }
    if (q == '"' && c == '\\') {
      if (i >= s.size()) break;
      char e = s[i++];
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case '0': out.push_back('\0'); break;
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'u': {
          if (i + 4 > s.size()) fail(no, "short \\u escape");
          append_utf8(out, static_cast<unsigned>(std::strtoul(s.substr(i, 4).c_str(), nullptr, 16)));
          i += 4;
          break;
        }
        default: out.push_back(e);
      }
      continue;
    }
    out.push_back(c);
  }
  fail(no, "unterminated quoted scalar");
}

Json plain_scalar(const std::string& v) {
  if (v.empty() || v == "~" || v == "null" || v == "Null" || v == "NULL") return Json();
  if (v == "true" || v == "True" || v == "TRUE") return Json(true);
  if (v == "false" || v == "False" || v == "FALSE") return Json(false);
  const char* b = v.c_str();
  char* e = nullptr;
  errno = 0;
  long long iv = std::strtoll(b, &e, 10);
  if (*e == '\0' && errno == 0 && (std::isdigit(static_cast<unsigned char>(v[0])) || v[0] == '-' || v[0] == '+'))
    return Json(iv);
  double dv = std::strtod(b, &e);
  if (*e == '\0' && (std::isdigit(static_cast<unsigned char>(v[0])) || v[0] == '-' || v[0] == '+' || v[0] == '.'))
    return Json(dv);
  return Json(v);
}

// Flow collections on one line: [a, "b", {k: v}] / {k: v, k2: [1]}.
Json flow(const std::string& s, size_t& i, int no);

void skip_ws(const std::string& s, size_t& i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
}

Json flow_scalar(const std::string& s, size_t& i, int no, bool key) {
  skip_ws(s, i);
  if (i < s.size() && (s[i] == '"' || s[i] == '\'')) return Json(quoted(s, i, no));
  if (i < s.size() && (s[i] == '[' || s[i] == '{')) return flow(s, i, no);
  size_t a = i;
  while (i < s.size() && s[i] != ',' && s[i] != ']' && s[i] != '}' && !(key && s[i] == ':')) ++i;
  return plain_scalar(trim(s.substr(a, i - a)));
}

Json flow(const std::string& s, size_t& i, int no) {
  char open = s[i++];
  char close = open == '[' ? ']' : '}';
  Json out = open == '[' ? Json::array() : Json::object();
  skip_ws(s, i);
  if (i < s.size() && s[i] == close) {
    ++i;
    return out;
  }
  while (i < s.size()) {
    if (open == '[') {
      out.push_back(flow_scalar(s, i, no, false));
    } else {
      Json k = flow_scalar(s, i, no, true);
      skip_ws(s, i);
      if (i >= s.size() || s[i] != ':') fail(no, "expected ':' in flow mapping");
      ++i;
      out[k.is_string() ? k.as_string() : k.dump()] = flow_scalar(s, i, no, false);
    }
    skip_ws(s, i);
    if (i < s.size() && s[i] == ',') {
      ++i;
      continue;
    }
    if (i < s.size() && s[i] == close) {
      ++i;
      return out;
    }
    break;
  }
  fail(no, std::string("unterminated flow collection, expected '") + close + "'");
}

class Parser {
 public:
  explicit Parser(std::vector<Line> lines) : l_(std::move(lines)) {}

  Json document() {
    if (l_.empty()) return Json();
    Json v = block(l_[0].indent);
    if (i_ < l_.size()) fail(l_[i_].no, "unexpected content (bad indentation?)");
    return v;
  }

 private:
  static bool is_seq_item(const std::string& t) { return t == "-" || (t.size() > 1 && t[0] == '-' && t[1] == ' '); }

  // Position of the "key: " separator (or a trailing ':'), outside quotes; npos if none.
  static size_t key_sep(const std::string& t) {
    char q = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      char c = t[i];
      if (q) {
        if (c == q) q = 0;
        else if (q == '"' && c == '\\') ++i;
        continue;
      }
      if ((c == '"' || c == '\'') && i == 0) {
        q = c;
        continue;
      }
      if (c == '[' || c == '{') return std::string::npos;  // flow value, not a key
      if (c == ':' && (i + 1 == t.size() || t[i + 1] == ' ' || t[i + 1] == '\t')) return i;
    }
    return std::string::npos;
  }

  Json block(int indent) {
    if (i_ >= l_.size()) return Json();
    return is_seq_item(l_[i_].text) ? seq(indent) : map_or_scalar(indent);
  }

  Json map_or_scalar(int indent) {
    const Line& first = l_[i_];
    if (key_sep(first.text) == std::string::npos) {  // a lone scalar document / value
      ++i_;
      return value(first.text, first.no, indent);
    }
    Json out = Json::object();
    while (i_ < l_.size() && l_[i_].indent == indent && !is_seq_item(l_[i_].text)) {
      const Line& ln = l_[i_];
      size_t sep = key_sep(ln.text);
      if (sep == std::string::npos) fail(ln.no, "expected 'key: value'");
      std::string k = trim(ln.text.substr(0, sep));
      if (!k.empty() && (k[0] == '"' || k[0] == '\'')) {
        size_t j = 0;
        k = quoted(k, j, ln.no);
      }
      std::string rest = trim(ln.text.substr(sep + 1));
      int no = ln.no;
      ++i_;
      if (rest.empty()) {
        if (i_ < l_.size() && l_[i_].indent > indent) out[k] = block(l_[i_].indent);
        else if (i_ < l_.size() && l_[i_].indent == indent && is_seq_item(l_[i_].text)) out[k] = seq(indent);
        else out[k] = Json();
      } else {
        out[k] = value(rest, no, indent);
      }
    }
    if (i_ < l_.size() && l_[i_].indent > indent) fail(l_[i_].no, "bad indentation");
    return out;
  }

  Json seq(int indent) {
    Json out = Json::array();
    while (i_ < l_.size() && l_[i_].indent == indent && is_seq_item(l_[i_].text)) {
      Line& ln = l_[i_];
      std::string rest = ln.text.size() > 1 ? trim(ln.text.substr(1)) : "";
      if (rest.empty()) {
        ++i_;
        out.push_back(i_ < l_.size() && l_[i_].indent > indent ? block(l_[i_].indent) : Json());
        continue;
      }
      // "- key: v" / "- - x": re-read the remainder as a block starting at its own column
      size_t col = ln.text.find_first_not_of(" \t", 1);
      if (key_sep(rest) != std::string::npos || is_seq_item(rest)) {
        ln.indent += static_cast<int>(col);
        ln.text = rest;
        out.push_back(block(ln.indent));
      } else {
        ++i_;
        out.push_back(value(rest, ln.no, indent));
      }
    }
    return out;
  }

  // A value on the same line as its key / dash: scalar, flow collection or block scalar header.
  Json value(const std::string& v, int no, int parent_indent) {
    if (v[0] == '"' || v[0] == '\'') {
      size_t j = 0;
      std::string s = quoted(v, j, no);
      if (!trim(v.substr(j)).empty()) fail(no, "trailing characters after quoted scalar");
      return Json(s);
    }
    if (v[0] == '[' || v[0] == '{') {
      size_t j = 0;
      Json f = flow(v, j, no);
      if (!trim(v.substr(j)).empty()) fail(no, "trailing characters after flow collection");
      return f;
    }
    if (v[0] == '|' || v[0] == '>') return block_scalar(v, parent_indent);
    if (v[0] == '&' || v[0] == '*' || v[0] == '!') fail(no, "anchors, aliases and tags are not supported");
    return plain_scalar(v);
  }

  Json block_scalar(const std::string& hdr, int parent_indent) {
    bool folded = hdr[0] == '>';
    bool strip = hdr.find('-') != std::string::npos, keep = hdr.find('+') != std::string::npos;
    std::vector<std::string> body;
    int ind = -1;
    while (i_ < l_.size() && l_[i_].indent > parent_indent) {
      if (ind < 0) ind = l_[i_].indent;
      body.push_back(l_[i_].raw.size() > static_cast<size_t>(ind) ? rtrim(l_[i_].raw.substr(static_cast<size_t>(ind))) : "");
      ++i_;
    }
    std::string out;
    for (size_t k = 0; k < body.size(); ++k) {
      out += body[k];
      if (k + 1 < body.size()) out += folded ? " " : "\n";
    }
    if (!strip && !body.empty()) out += "\n";
    (void)keep;  // blank trailing lines are dropped by the line scanner: keep == clip here
    return Json(out);
  }

  std::vector<Line> l_;
  size_t i_ = 0;
};

}  // namespace

Json yaml_parse(const std::string& text) {
  std::vector<Line> lines;
  size_t pos = 0;
  int no = 0;
  bool started = false;
  while (pos <= text.size()) {
    size_t nl = text.find('\n', pos);
    std::string raw = text.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
    pos = nl == std::string::npos ? text.size() + 1 : nl + 1;
    ++no;
    if (!raw.empty() && raw.back() == '\r') raw.pop_back();
    if (raw.rfind("---", 0) == 0 && (raw.size() == 3 || raw[3] == ' ')) {
      if (started) break;  // first document only
      continue;
    }
    if (raw == "...") break;
    if (raw.rfind("%", 0) == 0) continue;  // directives
    size_t lead = raw.find_first_not_of(" \t");
    if (lead != std::string::npos && raw.find('\t') < lead) fail(no, "tabs are not allowed for indentation");
    std::string body = rtrim(strip_comment(raw));
    size_t a = body.find_first_not_of(' ');
    if (a == std::string::npos) continue;
    started = true;
    lines.push_back(Line{static_cast<int>(a), body.substr(a), no, raw});
  }
  return Parser(std::move(lines)).document();
}

}  // namespace gpupool
