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

}  // namespace host
}  // namespace wh
