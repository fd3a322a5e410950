// Minimal JSON value for the control-plane messages exchanged between the
// native scheduler and the workers (flat objects of strings, numbers, bools,
// null, number lists and string lists; nesting is supported generally).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace wh {
namespace host {

class Json {
 public:
  enum Kind { kNull, kBool, kNum, kStr, kArr, kObj };
  Json() = default;
  static Json Null() { return Json(); }
  static Json Bool(bool b) { Json j; j.kind_ = kBool; j.b_ = b; return j; }
  static Json Num(double d) { Json j; j.kind_ = kNum; j.d_ = d; return j; }
  static Json Str(const std::string& s) { Json j; j.kind_ = kStr; j.s_ = s; return j; }
  static Json Arr() { Json j; j.kind_ = kArr; return j; }
  static Json Obj() { Json j; j.kind_ = kObj; return j; }
  static Json Parse(const std::string& text);  // throws std::runtime_error

  Kind kind() const { return kind_; }
  bool is_null() const { return kind_ == kNull; }
  bool truthy() const;  // Python truthiness of the value
  double num() const;
  bool boolean() const;
  const std::string& str() const;
  const std::vector<Json>& arr() const { return a_; }
  std::vector<double> nums() const;       // array of numbers
  std::vector<std::string> strs() const;  // array of strings
  bool has(const std::string& k) const { return kind_ == kObj && o_.count(k); }
  const Json& operator[](const std::string& k) const;  // null when absent
  Json& set(const std::string& k, Json v);
  Json& push(Json v);
  std::string Dump() const;

 private:
  Kind kind_ = kNull;
  bool b_ = false;
  double d_ = 0;
  std::string s_;
  std::vector<Json> a_;
  std::map<std::string, Json> o_;
};

}  // namespace host
}  // namespace wh
