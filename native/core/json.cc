#include "core/json.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace p2pt {

const Json* Json::get(std::string_view key) const {
  if (type_ != Type::Object) return nullptr;
  for (auto& kv : o_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

Json& Json::set(std::string key, Json v) {
  if (type_ != Type::Object) {
    type_ = Type::Object;
    o_.clear();
  }
  for (auto& kv : o_) {
    if (kv.first == key) {
      kv.second = std::move(v);
      return kv.second;
    }
  }
  o_.emplace_back(std::move(key), std::move(v));
  return o_.back().second;
}

void json_escape_to(std::string& out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  size_t run = 0;
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(s.data() + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        out += "\\u00";
        out.push_back(hex[c >> 4]);
        out.push_back(hex[c & 15]);
    }
  }
  out.append(s.data() + run, s.size() - run);
  out.push_back('"');
}

void Json::dump_to(std::string& out) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: {
      char buf[32];
      int n = snprintf(buf, sizeof buf, "%lld", static_cast<long long>(i_));
      out.append(buf, size_t(n));
      break;
    }
    case Type::Double: {
      if (!std::isfinite(d_)) {
        out += "null";
        break;
      }
      char buf[40];
      int n = snprintf(buf, sizeof buf, "%.17g", d_);
      out.append(buf, size_t(n));
      break;
    }
    case Type::String: json_escape_to(out, s_); break;
    case Type::Array: {
      out.push_back('[');
      for (size_t i = 0; i < a_.size(); i++) {
        if (i) out.push_back(',');
        a_[i].dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      for (size_t i = 0; i < o_.size(); i++) {
        if (i) out.push_back(',');
        json_escape_to(out, o_[i].first);
        out.push_back(':');
        o_[i].second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump() const {
  std::string s;
  dump_to(s);
  return s;
}

namespace {

struct Parser {
  const char* p;
  const char* end;
  std::string err;
  int depth = 0;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
  }
  bool fail(const char* m) {
    if (err.empty()) err = m;
    return false;
  }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o.push_back(char(cp));
    else if (cp < 0x800) {
      o.push_back(char(0xC0 | (cp >> 6)));
      o.push_back(char(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back(char(0xE0 | (cp >> 12)));
      o.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back(char(0x80 | (cp & 0x3F)));
    } else {
      o.push_back(char(0xF0 | (cp >> 18)));
      o.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back(char(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t& v) {
    if (end - p < 4) return fail("truncated \\u escape");
    v = 0;
    for (int i = 0; i < 4; i++) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= uint32_t(c - '0');
      else if (c >= 'a' && c <= 'f') v |= uint32_t(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= uint32_t(c - 'A' + 10);
      else return fail("bad \\u escape");
    }
    return true;
  }
  bool string(std::string& o) {
    if (p >= end || *p != '"') return fail("expected string");
    p++;
    while (true) {
      const char* s = p;
      while (p < end && *p != '"' && *p != '\\' && static_cast<unsigned char>(*p) >= 0x20) p++;
      o.append(s, size_t(p - s));
      if (p >= end) return fail("unterminated string");
      char c = *p++;
      if (c == '"') return true;
      if (c != '\\') return fail("control character in string");
      if (p >= end) return fail("unterminated escape");
      char e = *p++;
      switch (e) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {
            uint32_t lo;
            if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              if (!hex4(lo)) return false;
              if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              else { utf8(o, 0xFFFD); cp = lo; }
            } else cp = 0xFFFD;
          } else if (cp >= 0xDC00 && cp < 0xE000) cp = 0xFFFD;
          utf8(o, cp);
          break;
        }
        default: return fail("bad escape");
      }
    }
  }
  bool number(Json& out) {
    const char* s = p;
    bool is_float = false;
    if (p < end && *p == '-') p++;
    if (p >= end || !(*p >= '0' && *p <= '9')) return fail("bad number");
    if (*p == '0') p++;
    else while (p < end && *p >= '0' && *p <= '9') p++;
    if (p < end && *p == '.') {
      is_float = true;
      p++;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("bad number");
      while (p < end && *p >= '0' && *p <= '9') p++;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      is_float = true;
      p++;
      if (p < end && (*p == '+' || *p == '-')) p++;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("bad number");
      while (p < end && *p >= '0' && *p <= '9') p++;
    }
    std::string tok(s, size_t(p - s));
    if (!is_float) {
      errno = 0;
      char* ep;
      long long v = strtoll(tok.c_str(), &ep, 10);
      if (errno == 0) {
        out = Json(int64_t(v));
        return true;
      }
    }
    out = Json(strtod(tok.c_str(), nullptr));
    return true;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if (size_t(end - p) < n || memcmp(p, w, n) != 0) return fail("bad literal");
    p += n;
    return true;
  }
  bool value(Json& out) {
    if (++depth > 128) return fail("nesting too deep");
    ws();
    if (p >= end) return fail("unexpected end");
    bool ok = true;
    switch (*p) {
      case '{': {
        p++;
        out = Json::object();
        ws();
        if (p < end && *p == '}') {
          p++;
          break;
        }
        while (true) {
          ws();
          std::string k;
          if (!string(k)) return false;
          ws();
          if (p >= end || *p != ':') return fail("expected ':'");
          p++;
          Json v;
          if (!value(v)) return false;
          out.set(std::move(k), std::move(v));
          ws();
          if (p < end && *p == ',') { p++; continue; }
          if (p < end && *p == '}') { p++; break; }
          return fail("expected ',' or '}'");
        }
        break;
      }
      case '[': {
        p++;
        out = Json::array();
        ws();
        if (p < end && *p == ']') {
          p++;
          break;
        }
        while (true) {
          Json v;
          if (!value(v)) return false;
          out.push(std::move(v));
          ws();
          if (p < end && *p == ',') { p++; continue; }
          if (p < end && *p == ']') { p++; break; }
          return fail("expected ',' or ']'");
        }
        break;
      }
      case '"': {
        std::string s;
        ok = string(s);
        out = Json(std::move(s));
        break;
      }
      case 't': ok = lit("true"); out = Json(true); break;
      case 'f': ok = lit("false"); out = Json(false); break;
      case 'n': ok = lit("null"); out = Json(); break;
      default: ok = number(out);
    }
    depth--;
    return ok;
  }
};

}  // namespace

bool Json::parse(std::string_view text, Json& out, std::string* err) {
  Parser ps{text.data(), text.data() + text.size(), {}};
  Json v;
  bool ok = ps.value(v);
  if (ok) {
    ps.ws();
    if (ps.p != ps.end) ok = ps.fail("trailing characters");
  }
  if (!ok) {
    if (err) *err = ps.err + " at offset " + std::to_string(ps.p - text.data());
    return false;
  }
  out = std::move(v);
  return true;
}

}  // namespace p2pt
