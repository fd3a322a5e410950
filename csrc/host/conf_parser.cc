// Protobuf-text-format subset parser for wormhole .conf files (reference
// ArgParser, learn/base/arg_parser.h:13-64: `key = value` / `key: value`,
// '#' comments, quoted strings, nested `name { ... }` messages; argv
// overrides use the same syntax and are merged after the file).
#include <cctype>
#include <memory>
#include <string>
#include <vector>

#include "common.h"

namespace wh {
namespace host {


namespace {

class Lexer {
 public:
  explicit Lexer(const std::string& s) : s_(s) {}
  void skip() {
    while (i_ < s_.size()) {
      char c = s_[i_];
      if (std::isspace((unsigned char)c) || c == ',' || c == ';') {
        if (c == '\n') ++line_;
        ++i_;
      } else if (c == '#') {
        while (i_ < s_.size() && s_[i_] != '\n') ++i_;
      } else {
        break;
      }
    }
  }
  bool eof() {
    skip();
    return i_ >= s_.size();
  }
  char peek() {
    skip();
    return i_ < s_.size() ? s_[i_] : '\0';
  }
  char get() {
    skip();
    return s_[i_++];
  }
  std::string ident() {
    skip();
    size_t b = i_;
    while (i_ < s_.size() && (std::isalnum((unsigned char)s_[i_]) || s_[i_] == '_' ||
                              s_[i_] == '.' || s_[i_] == '[' || s_[i_] == ']'))
      ++i_;
    if (b == i_) err("expected a field name");
    return s_.substr(b, i_ - b);
  }
  std::string token() {
    skip();
    size_t b = i_;
    while (i_ < s_.size() && !std::isspace((unsigned char)s_[i_]) && s_[i_] != '#' &&
           s_[i_] != '}' && s_[i_] != '{' && s_[i_] != ',' && s_[i_] != ';')
      ++i_;
    if (b == i_) err("expected a value");
    return s_.substr(b, i_ - b);
  }
  std::string quoted() {
    const char q = get();
    std::string out;
    while (true) {
      if (i_ >= s_.size()) err("unterminated string");
      char c = s_[i_++];
      if (c == q) break;
      if (c == '\\' && i_ < s_.size()) {
        char e = s_[i_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    // adjacent string literals concatenate (protobuf text format rule)
    while (peek() == '"' || peek() == '\'') out += quoted();
    return out;
  }
  [[noreturn]] void err(const std::string& m) {
    throw std::runtime_error("conf parse error at line " + std::to_string(line_) + ": " + m);
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  int line_ = 1;
};

void parse_block(Lexer& lx, std::vector<ConfItem>* out, bool nested) {
  while (!lx.eof()) {
    if (lx.peek() == '}') {
      if (!nested) lx.err("unbalanced '}'");
      lx.get();
      return;
    }
    ConfItem it;
    it.key = lx.ident();
    char c = lx.peek();
    if (c == ':' || c == '=') {
      lx.get();
      c = lx.peek();
    }
    if (c == '{') {
      lx.get();
      it.kind = 'm';
      parse_block(lx, &it.children, true);
    } else if (c == '"' || c == '\'') {
      it.kind = 's';
      it.value = lx.quoted();
    } else {
      it.kind = 't';
      it.value = lx.token();
    }
    out->push_back(std::move(it));
  }
  if (nested) lx.err("missing '}'");
}

}  // namespace

std::vector<ConfItem> ParseConf(const std::string& text) {
  std::vector<ConfItem> items;
  Lexer lx(text);
  parse_block(lx, &items, false);
  return items;
}

// dmlc::Config-format text ("key = value" per entry, '#' comments, quoted
// values, repeated keys kept in order) -> protobuf text ("key: value", string
// values re-quoted).  The reference's unused alternative front end
// (learn/base/arg2proto.h:13-20: dmlc::Config(in, multi_value=true)
// .ToProtoString() then TextFormat::ParseFromString).  Nested messages are
// not part of that format; a line "name {" is passed through unchanged so
// files in either syntax convert.
std::string Arg2Proto(const std::string& text) {
  std::string out;
  size_t i = 0;
  const size_t n = text.size();
  auto quote = [](const std::string& v) {
    std::string q = "\"";
    for (char c : v) {
      if (c == '"' || c == '\\') q += '\\';
      if (c == '\n') { q += "\\n"; continue; }
      q += c;
    }
    return q + "\"";
  };
  while (i < n) {
    size_t e = text.find('\n', i);
    if (e == std::string::npos) e = n;
    std::string line = text.substr(i, e - i);
    i = e + 1;
    // strip comments outside quotes
    bool inq = false;
    char qc = 0;
    for (size_t k = 0; k < line.size(); ++k) {
      const char c = line[k];
      if (inq) {
        if (c == '\\') ++k;
        else if (c == qc) inq = false;
      } else if (c == '"' || c == '\'') {
        inq = true;
        qc = c;
      } else if (c == '#') {
        line.resize(k);
        break;
      }
    }
    auto trim = [](std::string s) {
      size_t b = 0, t = s.size();
      while (b < t && std::isspace((unsigned char)s[b])) ++b;
      while (t > b && std::isspace((unsigned char)s[t - 1])) --t;
      return s.substr(b, t - b);
    };
    line = trim(line);
    if (line.empty()) continue;
    size_t eq = std::string::npos;
    for (size_t k = 0; k < line.size(); ++k)
      if (line[k] == '=' || line[k] == ':') { eq = k; break; }
    if (eq == std::string::npos) {  // "name {" / "}" of a nested message
      out += line + "\n";
      continue;
    }
    const std::string key = trim(line.substr(0, eq));
    std::string val = trim(line.substr(eq + 1));
    if (key.empty()) throw std::runtime_error("arg2proto: empty key in line: " + line);
    if (val.size() >= 2 && (val[0] == '"' || val[0] == '\'') && val.back() == val[0]) {
      std::string raw;
      for (size_t k = 1; k + 1 < val.size(); ++k) {
        if (val[k] == '\\' && k + 2 < val.size()) {
          const char c = val[++k];
          raw += c == 'n' ? '\n' : c == 't' ? '\t' : c;
        } else {
          raw += val[k];
        }
      }
      out += key + ": " + quote(raw) + "\n";
    } else if (val == "{") {
      out += key + " {\n";
    } else {
      out += key + ": " + val + "\n";
    }
  }
  return out;
}

}  // namespace host
}  // namespace wh
