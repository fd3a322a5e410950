#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace wh {
namespace host {

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;
  explicit Parser(const std::string& t) : s(t) {}

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool lit(const char* w) {
    size_t n = std::char_traits<char>::length(w);
    if (s.compare(i, n, w) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= s.size()) fail("bad escape");
      char e = s[i++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          if (i + 4 > s.size()) fail("bad \\u escape");
          unsigned cp = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
          i += 4;
          if (cp >= 0xD800 && cp <= 0xDBFF && i + 6 <= s.size() && s[i] == '\\' &&
              s[i + 1] == 'u') {  // surrogate pair
            unsigned lo = (unsigned)std::strtoul(s.substr(i + 2, 4).c_str(), nullptr, 16);
            i += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (cp < 0x80) {
            out += (char)cp;
          } else if (cp < 0x800) {
            out += (char)(0xC0 | (cp >> 6));
            out += (char)(0x80 | (cp & 0x3F));
          } else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
          } else {
            out += (char)(0xF0 | (cp >> 18));
            out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
          }
          break;
        }
        default: fail("bad escape");
      }
    }
    if (i >= s.size()) fail("unterminated string");
    ++i;
    return out;
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    const char c = s[i];
    if (c == '{') {
      ++i;
      Json o = Json::Obj();
      ws();
      if (s[i] == '}') {
        ++i;
        return o;
      }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (s[i] != ':') fail("expected ':'");
        ++i;
        o.set(k, value());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == '}') { ++i; return o; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Json a = Json::Arr();
      ws();
      if (s[i] == ']') {
        ++i;
        return a;
      }
      while (true) {
        a.push(value());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == ']') { ++i; return a; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') return Json::Str(str());
    if (lit("true")) return Json::Bool(true);
    if (lit("false")) return Json::Bool(false);
    if (lit("null")) return Json::Null();
    if (lit("NaN")) return Json::Num(NAN);
    if (lit("Infinity")) return Json::Num(INFINITY);
    if (lit("-Infinity")) return Json::Num(-INFINITY);
    char* end = nullptr;
    const double d = std::strtod(s.c_str() + i, &end);
    if (end == s.c_str() + i) fail("bad value");
    i = (size_t)(end - s.c_str());
    return Json::Num(d);
  }
};

void dump_str(const std::string& s, std::string* out) {
  *out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': *out += "\\\""; break;
      case '\\': *out += "\\\\"; break;
      case '\n': *out += "\\n"; break;
      case '\r': *out += "\\r"; break;
      case '\t': *out += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          *out += b;
        } else {
          *out += (char)c;
        }
    }
  }
  *out += '"';
}

}  // namespace

Json Json::Parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

bool Json::truthy() const {
  switch (kind_) {
    case kNull: return false;
    case kBool: return b_;
    case kNum: return d_ != 0;
    case kStr: return !s_.empty();
    case kArr: return !a_.empty();
    case kObj: return !o_.empty();
  }
  return false;
}

double Json::num() const {
  if (kind_ == kNum) return d_;
  if (kind_ == kBool) return b_ ? 1 : 0;
  throw std::runtime_error("json: not a number");
}

bool Json::boolean() const { return truthy(); }

const std::string& Json::str() const {
  if (kind_ != kStr) throw std::runtime_error("json: not a string");
  return s_;
}

std::vector<double> Json::nums() const {
  std::vector<double> v;
  for (const auto& x : a_) v.push_back(x.num());
  return v;
}

std::vector<std::string> Json::strs() const {
  std::vector<std::string> v;
  for (const auto& x : a_) v.push_back(x.str());
  return v;
}

const Json& Json::operator[](const std::string& k) const {
  static const Json null;
  if (kind_ != kObj) return null;
  auto it = o_.find(k);
  return it == o_.end() ? null : it->second;
}

Json& Json::set(const std::string& k, Json v) {
  kind_ = kObj;
  o_[k] = std::move(v);
  return *this;
}

Json& Json::push(Json v) {
  kind_ = kArr;
  a_.push_back(std::move(v));
  return *this;
}

std::string Json::Dump() const {
  std::string out;
  switch (kind_) {
    case kNull: out = "null"; break;
    case kBool: out = b_ ? "true" : "false"; break;
    case kNum: {
      if (std::isfinite(d_) && d_ == std::floor(d_) && std::fabs(d_) < 9e15) {
        out = std::to_string((long long)d_);
      } else {
        char b[32];
        std::snprintf(b, sizeof(b), "%.17g", d_);
        out = b;
      }
      break;
    }
    case kStr: dump_str(s_, &out); break;
    case kArr: {
      out = "[";
      for (size_t i = 0; i < a_.size(); ++i) {
        if (i) out += ", ";
        out += a_[i].Dump();
      }
      out += "]";
      break;
    }
    case kObj: {
      out = "{";
      bool first = true;
      for (const auto& kv : o_) {
        if (!first) out += ", ";
        first = false;
        dump_str(kv.first, &out);
        out += ": ";
        out += kv.second.Dump();
      }
      out += "}";
      break;
    }
  }
  return out;
}

}  // namespace host
}  // namespace wh
