#include "proto/frame.h"

#include <algorithm>
#include <cstdlib>

#include <algorithm>
#include <cstring>

#include "core/crypto.h"

namespace p2pt::proto {

std::optional<MsgType> msg_type_from_u8(uint8_t v) {
  switch (v) {
    case 1: case 2: case 3: case 4:
    case 10: case 11: case 12: case 13: case 14: case 15:
    case 20: case 21: case 22:
    case 99:
      return MsgType(v);
    default:
      return std::nullopt;
  }
}

const char* msg_type_name(MsgType t) {
  switch (t) {
    case MsgType::Hello: return "Hello";
    case MsgType::Agree: return "Agree";
    case MsgType::Ping: return "Ping";
    case MsgType::Pong: return "Pong";
    case MsgType::ReqHeaders: return "ReqHeaders";
    case MsgType::ReqBody: return "ReqBody";
    case MsgType::ReqEnd: return "ReqEnd";
    case MsgType::Cancel: return "Cancel";
    case MsgType::Credit: return "Credit";
    case MsgType::Assoc: return "Assoc";
    case MsgType::ResHeaders: return "ResHeaders";
    case MsgType::ResBody: return "ResBody";
    case MsgType::ResEnd: return "ResEnd";
    case MsgType::Error: return "Error";
  }
  return "?";
}

void Frame::header(uint8_t out[kHeaderLen]) const {
  out[0] = uint8_t(type);
  wr32(out + 1, stream_id);
}

Bytes Frame::encode() const {
  std::vector<uint8_t> v(kHeaderLen + payload.size());
  header(v.data());
  if (!payload.empty()) memcpy(v.data() + kHeaderLen, payload.data(), payload.size());
  return Bytes::take(std::move(v));
}

Bytes Frame::flat_payload() const {
  if (more.empty()) return payload;
  std::vector<uint8_t> v;
  v.reserve(payload_size());
  v.insert(v.end(), payload.data(), payload.data() + payload.size());
  for (auto& b : more) v.insert(v.end(), b.data(), b.data() + b.size());
  return Bytes::take(std::move(v));
}


bool decode_chain(const Bytes& raw, std::vector<Bytes>& more, Frame& out, std::string* err) {
  if (more.empty() || raw.size() < kHeaderLen) {
    Bytes flat = raw;
    if (!more.empty()) {  // a first fragment shorter than the header: one piece
      std::vector<uint8_t> v(raw.data(), raw.data() + raw.size());
      for (auto& b : more) v.insert(v.end(), b.data(), b.data() + b.size());
      flat = Bytes::take(std::move(v));
    }
    out.more.clear();
    return decode(flat, out, err);
  }
  if (!decode(raw, out, err)) return false;
  out.more = std::move(more);
  if (out.type != MsgType::ReqBody && out.type != MsgType::ResBody) {
    out.payload = out.flat_payload();
    out.more.clear();
  }
  return true;
}

bool decode(const Bytes& raw, Frame& out, std::string* err) {
  if (raw.size() < kHeaderLen) {
    if (err) *err = "message too short: " + std::to_string(raw.size()) + " bytes";
    return false;
  }
  auto t = msg_type_from_u8(raw[0]);
  if (!t) {
    if (err) *err = "unknown message type: " + std::to_string(raw[0]);
    return false;
  }
  out.type = *t;
  out.stream_id = rd32(raw.data() + 1);
  out.payload = raw.slice(kHeaderLen);
  return true;
}

namespace {
Json str_array(const std::vector<std::string>& v) {
  Json a = Json::array();
  for (auto& s : v) a.push(Json(s));
  return a;
}

bool get_u32(const Json& j, const char* k, uint32_t& out, std::string* err) {
  const Json* v = j.get(k);
  if (!v || !v->is_int() || v->as_int() < 0 || v->as_int() > int64_t(UINT32_MAX)) {
    if (err) *err = std::string(v ? "invalid type for field `" : "missing field `") + k + "`";
    return false;
  }
  out = uint32_t(v->as_int());
  return true;
}

bool get_str(const Json& j, const char* k, std::string& out, std::string* err) {
  const Json* v = j.get(k);
  if (!v || !v->is_string()) {
    if (err) *err = std::string(v ? "invalid type for field `" : "missing field `") + k + "`";
    return false;
  }
  out = v->as_string();
  return true;
}

bool get_str_array(const Json& j, const char* k, std::vector<std::string>& out, std::string* err) {
  const Json* v = j.get(k);
  if (!v || !v->is_array()) {
    if (err) *err = std::string(v ? "invalid type for field `" : "missing field `") + k + "`";
    return false;
  }
  out.clear();
  for (auto& e : v->as_array()) {
    if (!e.is_string()) {
      if (err) *err = std::string("invalid element in `") + k + "`";
      return false;
    }
    out.push_back(e.as_string());
  }
  return true;
}

bool get_headers(const Json& j, HeaderMap& out, std::string* err) {
  const Json* v = j.get("headers");
  if (!v || !v->is_object()) {
    if (err) *err = v ? "invalid type for field `headers`" : "missing field `headers`";
    return false;
  }
  out.clear();
  for (auto& kv : v->as_object()) {
    if (!kv.second.is_string()) {
      if (err) *err = "header value must be a string";
      return false;
    }
    out.emplace_back(kv.first, kv.second.as_string());
  }
  return true;
}

Json headers_json(const HeaderMap& h) {
  Json o = Json::object();
  for (auto& kv : h) o.set(kv.first, Json(kv.second));
  return o;
}

Frame json_frame(MsgType t, uint32_t sid, const Json& j) {
  std::string s = j.dump();
  return Frame{t, sid, Bytes::copy(s)};
}
}  // namespace

bool json_parse_bytes(const Bytes& b, Json& out, std::string* err) { return Json::parse(b.view(), out, err); }

Json Hello::to_json() const {
  Json j = Json::object();
  j.set("proto", Json(proto));
  j.set("min_version", Json(min_version));
  j.set("max_version", Json(max_version));
  j.set("features", str_array(features));
  if (!psk_nonce.empty()) j.set("psk_nonce", Json(psk_nonce));
  if (!psk_mac.empty()) j.set("psk_mac", Json(psk_mac));
  if (assoc) j.set("assoc", Json(assoc));
  return j;
}

// Optional unsigned member (absent is fine).
static bool opt_u32(const Json& j, const char* k, uint32_t& out, std::string* err) {
  if (!j.get(k)) return true;
  return get_u32(j, k, out, err);
}

// Optional string member (absent is fine; present must be a string).
static bool opt_str(const Json& j, const char* k, std::string& out, std::string* err) {
  const Json* v = j.get(k);
  if (!v) return true;
  if (!v->is_string()) {
    if (err) *err = std::string("field '") + k + "' must be a string";
    return false;
  }
  out = v->as_string();
  return true;
}

bool Hello::from_json(const Json& j, Hello& out, std::string* err) {
  if (!j.is_object()) {
    if (err) *err = "expected object";
    return false;
  }
  return get_str(j, "proto", out.proto, err) && get_u32(j, "min_version", out.min_version, err) &&
         get_u32(j, "max_version", out.max_version, err) && get_str_array(j, "features", out.features, err) &&
         opt_str(j, "psk_nonce", out.psk_nonce, err) && opt_str(j, "psk_mac", out.psk_mac, err) &&
         opt_u32(j, "assoc", out.assoc, err);
}

Json Agree::to_json() const {
  Json j = Json::object();
  j.set("version", Json(version));
  j.set("features", str_array(features));
  if (!psk_mac.empty()) j.set("psk_mac", Json(psk_mac));
  if (assoc) j.set("assoc", Json(assoc));
  return j;
}

bool Agree::from_json(const Json& j, Agree& out, std::string* err) {
  if (!j.is_object()) {
    if (err) *err = "expected object";
    return false;
  }
  return get_u32(j, "version", out.version, err) && get_str_array(j, "features", out.features, err) &&
         opt_str(j, "psk_mac", out.psk_mac, err) && opt_u32(j, "assoc", out.assoc, err);
}

std::string psk_mac(const std::string& secret, const char* role, const std::string& nonce,
                    const std::string& binding) {
  std::string msg = std::string("p2pt-psk|") + role + "|" + nonce + "|" + binding;
  auto mac = hmac_sha256(secret.data(), secret.size(), msg.data(), msg.size());
  return hex_encode(mac.data(), mac.size());
}

// TUNNEL_FEATURES=<comma list> replaces the list (e.g. "sse" to behave
// exactly like a reference peer in interop and A/B tests).
const std::vector<std::string>& our_features() {
  static const std::vector<std::string> f = [] {
    std::vector<std::string> v{"sse", "cancel", "flow", "multistream", "assoc"};
    if (const char* e = getenv("TUNNEL_FEATURES")) {
      v.clear();
      std::string s = e;
      for (size_t a = 0; a <= s.size();) {
        size_t c = s.find(',', a);
        if (c == std::string::npos) c = s.size();
        if (c > a) v.push_back(s.substr(a, c - a));
        a = c + 1;
      }
    }
    return v;
  }();
  return f;
}

bool agree_from_hello(const Hello& h, Agree& out, std::string* err, const std::vector<std::string>& ours) {
  if (h.proto != kProtocolName) {
    if (err) *err = "unknown protocol: " + h.proto;
    return false;
  }
  const uint32_t our_min = 1, our_max = kProtocolVersion;
  uint32_t lo = std::max(h.min_version, our_min);
  uint32_t hi = std::min(h.max_version, our_max);
  if (lo > hi) {
    if (err)
      *err = "no compatible version: peer=[" + std::to_string(h.min_version) + "," + std::to_string(h.max_version) +
             "], ours=[" + std::to_string(our_min) + "," + std::to_string(our_max) + "]";
    return false;
  }
  out.version = hi;
  out.features.clear();
  for (auto& f : h.features)
    if (std::find(ours.begin(), ours.end(), f) != ours.end()) out.features.push_back(f);
  return true;
}

void header_set(HeaderMap& h, std::string name, std::string value) {
  for (auto& kv : h)
    if (kv.first == name) {
      kv.second = std::move(value);
      return;
    }
  h.emplace_back(std::move(name), std::move(value));
}

const std::string* header_get(const HeaderMap& h, std::string_view name) {
  for (auto& kv : h)
    if (kv.first == name) return &kv.second;
  return nullptr;
}

Json RequestHeaders::to_json() const {
  Json j = Json::object();
  j.set("stream_id", Json(stream_id));
  j.set("method", Json(method));
  j.set("path", Json(path));
  j.set("headers", headers_json(headers));
  return j;
}

bool RequestHeaders::from_json(const Json& j, RequestHeaders& out, std::string* err) {
  if (!j.is_object()) {
    if (err) *err = "expected object";
    return false;
  }
  return get_u32(j, "stream_id", out.stream_id, err) && get_str(j, "method", out.method, err) &&
         get_str(j, "path", out.path, err) && get_headers(j, out.headers, err);
}

Json ResponseHeaders::to_json() const {
  Json j = Json::object();
  j.set("stream_id", Json(stream_id));
  j.set("status", Json(unsigned(status)));
  j.set("headers", headers_json(headers));
  return j;
}

bool ResponseHeaders::from_json(const Json& j, ResponseHeaders& out, std::string* err) {
  if (!j.is_object()) {
    if (err) *err = "expected object";
    return false;
  }
  uint32_t st = 0;
  if (!get_u32(j, "stream_id", out.stream_id, err) || !get_u32(j, "status", st, err) ||
      !get_headers(j, out.headers, err))
    return false;
  if (st > 65535) {
    if (err) *err = "status out of range";
    return false;
  }
  out.status = uint16_t(st);
  return true;
}

Frame make_hello(const Hello& h) { return json_frame(MsgType::Hello, 0, h.to_json()); }
Frame make_agree(const Agree& a) { return json_frame(MsgType::Agree, 0, a.to_json()); }
Frame make_req_headers(const RequestHeaders& h) { return json_frame(MsgType::ReqHeaders, h.stream_id, h.to_json()); }
Frame make_res_headers(const ResponseHeaders& h) { return json_frame(MsgType::ResHeaders, h.stream_id, h.to_json()); }
Frame make_body(MsgType t, uint32_t sid, Bytes data) { return Frame{t, sid, std::move(data)}; }
Frame make_empty(MsgType t, uint32_t sid) { return Frame{t, sid, Bytes()}; }
Frame make_error(uint32_t sid, const std::string& msg) { return Frame{MsgType::Error, sid, Bytes::copy(msg)}; }
Frame make_credit(uint32_t sid, uint32_t bytes) {
  uint8_t b[4];
  wr32(b, bytes);
  return Frame{MsgType::Credit, sid, slab_copy(b, 4)};
}
uint32_t credit_bytes(const Frame& f) { return f.payload.size() == 4 ? rd32(f.payload.data()) : 0; }

static std::string trim_trailing_slashes(const std::string& s) {
  size_t n = s.size();
  while (n > 0 && s[n - 1] == '/') n--;
  return s.substr(0, n);
}

std::string build_upstream_url(const std::string& upstream_base, const std::string& advertise_prefix,
                               const std::string& request_path) {
  std::string base = trim_trailing_slashes(upstream_base);
  std::string prefix = trim_trailing_slashes(advertise_prefix);
  if (prefix.empty() || prefix == "/") return base + request_path;
  if (request_path.compare(0, prefix.size(), prefix) == 0) {
    std::string stripped = request_path.substr(prefix.size());
    if (stripped.empty()) stripped = "/";
    return base + stripped;
  }
  return base + request_path;
}

uint64_t FlowWindow::on_grant(uint64_t n, uint64_t now_us, uint64_t rtt_us) {
  if (!epoch_t0) {  // the first grant opens the first measuring epoch
    epoch_t0 = now_us ? now_us : 1;
    return 0;
  }
  epoch_bytes += n;
  if (epoch_bytes < uint64_t(win)) return 0;
  uint64_t extra = 0;
  const uint64_t elapsed = std::max<uint64_t>(now_us - epoch_t0, 1);
  bool grow;
  if (rtt_us) {
    // Credit-bound: taken within two round trips, and two bandwidth-delay
    // products at the rate it was taken exceed the window (on a LAN a
    // window lasts many round trips: growing there only adds buffering).
    const double bdp2 = 2.0 * double(epoch_bytes) / double(elapsed) * double(rtt_us);
    grow = elapsed < 2 * rtt_us + kFlowGrowSlackUs && bdp2 > double(win);
  } else {
    grow = elapsed < kFlowGrowUs;
  }
  if (win < kFlowMaxWindow && grow) {
    extra = uint64_t(std::min(win, kFlowMaxWindow - win));
    win += int64_t(extra);
  }
  epoch_bytes = 0;
  epoch_t0 = now_us ? now_us : 1;
  return extra;
}

}  // namespace p2pt::proto
