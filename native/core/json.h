// Minimal JSON DOM, parser and writer.
//
// Replaces serde_json in the reference (frame payloads, handshake and
// signalling messages: reference tunnel/src/protocol.rs:14-136,
// tunnel/src/signaling.rs:9-65). Objects keep insertion order so emitted
// documents match the reference's field order (serde emits struct fields in
// declaration order).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace p2pt {

class Json {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::vector<std::pair<std::string, Json>>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(unsigned v) : type_(Type::Int), i_(v) {}
  Json(int64_t v) : type_(Type::Int), i_(v) {}
  Json(uint64_t v) : type_(Type::Int), i_(int64_t(v)) {}
  Json(long long v) : type_(Type::Int), i_(int64_t(v)) {}
  Json(double v) : type_(Type::Double), d_(v) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Json(std::string_view s) : type_(Type::String), s_(s) {}
  static Json array() { Json j; j.type_ = Type::Array; return j; }
  static Json object() { Json j; j.type_ = Type::Object; return j; }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Double; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return type_ == Type::Bool ? b_ : dflt; }
  int64_t as_int(int64_t dflt = 0) const {
    return type_ == Type::Int ? i_ : type_ == Type::Double ? int64_t(d_) : dflt;
  }
  double as_double(double dflt = 0) const {
    return type_ == Type::Double ? d_ : type_ == Type::Int ? double(i_) : dflt;
  }
  const std::string& as_string() const { return s_; }
  const Array& as_array() const { return a_; }
  const Object& as_object() const { return o_; }
  Array& arr() { return a_; }
  Object& obj() { return o_; }

  // Object access. get() returns nullptr when absent or not an object.
  const Json* get(std::string_view key) const;
  Json& set(std::string key, Json v);  // replaces existing key (last wins)
  Json& push(Json v) {
    if (type_ != Type::Array) { type_ = Type::Array; a_.clear(); }
    a_.push_back(std::move(v));
    return a_.back();
  }
  size_t size() const { return type_ == Type::Array ? a_.size() : type_ == Type::Object ? o_.size() : 0; }

  std::string dump() const;
  void dump_to(std::string& out) const;

  // Returns false (and sets *err) on malformed input. Rejects trailing garbage.
  static bool parse(std::string_view text, Json& out, std::string* err = nullptr);

 private:
  Type type_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  Array a_;
  Object o_;
};

// JSON string escaping (serde_json compatible: escapes ", \, and control chars).
void json_escape_to(std::string& out, std::string_view s);

}  // namespace p2pt
