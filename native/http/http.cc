#include "http/http.h"

#include <cstring>
#include <ctime>

namespace p2pt::http {

bool iequals(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); i++)
    if (tolower(static_cast<unsigned char>(a[i])) != tolower(static_cast<unsigned char>(b[i]))) return false;
  return true;
}

std::string to_lower(std::string_view s) {
  std::string o(s);
  for (auto& c : o) c = char(tolower(static_cast<unsigned char>(c)));
  return o;
}

bool is_visible_ascii(std::string_view v) {
  for (unsigned char c : v)
    if (!((c >= 32 && c < 127) || c == '\t')) return false;
  return true;
}

const std::string* Head::get(std::string_view name) const {
  for (auto& h : headers)
    if (iequals(h.name, name)) return &h.value;
  return nullptr;
}

bool Head::has_token(std::string_view name, std::string_view token) const {
  for (auto& h : headers) {
    if (!iequals(h.name, name)) continue;
    std::string_view v = h.value;
    while (!v.empty()) {
      size_t c = v.find(',');
      std::string_view t = v.substr(0, c);
      while (!t.empty() && (t.front() == ' ' || t.front() == '\t')) t.remove_prefix(1);
      while (!t.empty() && (t.back() == ' ' || t.back() == '\t')) t.remove_suffix(1);
      if (iequals(t, token)) return true;
      if (c == std::string_view::npos) break;
      v.remove_prefix(c + 1);
    }
  }
  return false;
}

namespace {

bool is_tchar(char c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
         strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

// Find end of head ("\r\n\r\n" or bare "\n\n"); returns offset past it or npos.
size_t find_head_end(std::string_view buf) {
  for (size_t i = 0; i < buf.size(); i++) {
    if (buf[i] != '\n') continue;
    if (i + 1 < buf.size() && buf[i + 1] == '\n') return i + 2;
    if (i + 2 < buf.size() && buf[i + 1] == '\r' && buf[i + 2] == '\n') return i + 3;
  }
  return std::string_view::npos;
}

bool parse_headers(std::string_view lines, std::vector<Header>& out, std::string* err) {
  while (!lines.empty()) {
    size_t nl = lines.find('\n');
    std::string_view line = lines.substr(0, nl);
    lines = nl == std::string_view::npos ? std::string_view() : lines.substr(nl + 1);
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    if (line.empty()) break;
    if ((line[0] == ' ' || line[0] == '\t')) {
      if (out.empty()) {
        if (err) *err = "invalid header continuation";
        return false;
      }
      // obs-fold: join with a space (RFC 9112 §5.2)
      std::string_view cont = line;
      while (!cont.empty() && (cont.front() == ' ' || cont.front() == '\t')) cont.remove_prefix(1);
      out.back().value += ' ';
      out.back().value.append(cont);
      continue;
    }
    size_t colon = line.find(':');
    if (colon == std::string_view::npos || colon == 0) {
      if (err) *err = "invalid header line";
      return false;
    }
    std::string_view name = line.substr(0, colon);
    for (char c : name)
      if (!is_tchar(c)) {
        if (err) *err = "invalid header name";
        return false;
      }
    std::string_view v = line.substr(colon + 1);
    while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.remove_suffix(1);
    out.push_back(Header{std::string(name), std::string(v)});
  }
  return true;
}

bool parse_version(std::string_view v, int& minor) {
  if (v.size() != 8 || v.substr(0, 7) != "HTTP/1.") return false;
  if (v[7] < '0' || v[7] > '9') return false;
  minor = v[7] - '0';
  return true;
}

}  // namespace

ParseResult parse_request_head(std::string_view buf, Head& out, size_t& consumed, std::string* err) {
  // Skip leading empty lines (RFC 9112 §2.2).
  size_t skip = 0;
  while (skip < buf.size() && (buf[skip] == '\r' || buf[skip] == '\n')) skip++;
  std::string_view b = buf.substr(skip);
  size_t end = find_head_end(b);
  if (end == std::string_view::npos) {
    if (b.size() > kMaxHeadBytes) {
      if (err) *err = "request head too large";
      return ParseResult::Error;
    }
    return ParseResult::Incomplete;
  }
  std::string_view head = b.substr(0, end);
  size_t nl = head.find('\n');
  std::string_view line = head.substr(0, nl);
  if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
  size_t s1 = line.find(' ');
  size_t s2 = s1 == std::string_view::npos ? s1 : line.find(' ', s1 + 1);
  if (s1 == std::string_view::npos || s2 == std::string_view::npos) {
    if (err) *err = "invalid request line";
    return ParseResult::Error;
  }
  out = Head{};
  out.method = std::string(line.substr(0, s1));
  out.target = std::string(line.substr(s1 + 1, s2 - s1 - 1));
  for (char c : out.method)
    if (!is_tchar(c)) {
      if (err) *err = "invalid method";
      return ParseResult::Error;
    }
  if (out.target.empty() || !parse_version(line.substr(s2 + 1), out.version_minor)) {
    if (err) *err = "invalid request line";
    return ParseResult::Error;
  }
  if (!parse_headers(head.substr(nl + 1), out.headers, err)) return ParseResult::Error;
  consumed = skip + end;
  return ParseResult::Done;
}

ParseResult parse_response_head(std::string_view buf, Head& out, size_t& consumed, std::string* err) {
  size_t end = find_head_end(buf);
  if (end == std::string_view::npos) {
    if (buf.size() > kMaxHeadBytes) {
      if (err) *err = "response head too large";
      return ParseResult::Error;
    }
    return ParseResult::Incomplete;
  }
  std::string_view head = buf.substr(0, end);
  size_t nl = head.find('\n');
  std::string_view line = head.substr(0, nl);
  if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
  out = Head{};
  size_t s1 = line.find(' ');
  if (s1 == std::string_view::npos || !parse_version(line.substr(0, s1), out.version_minor)) {
    if (err) *err = "invalid status line";
    return ParseResult::Error;
  }
  std::string_view rest = line.substr(s1 + 1);
  if (rest.size() < 3) {
    if (err) *err = "invalid status code";
    return ParseResult::Error;
  }
  int st = 0;
  for (int i = 0; i < 3; i++) {
    if (rest[i] < '0' || rest[i] > '9') {
      if (err) *err = "invalid status code";
      return ParseResult::Error;
    }
    st = st * 10 + (rest[i] - '0');
  }
  out.status = st;
  if (rest.size() > 4) out.reason = std::string(rest.substr(4));
  if (!parse_headers(head.substr(nl + 1), out.headers, err)) return ParseResult::Error;
  consumed = end;
  return ParseResult::Done;
}

static bool parse_content_length(const Head& h, uint64_t& len, bool& present, std::string* err) {
  present = false;
  for (auto& hd : h.headers) {
    if (!iequals(hd.name, "content-length")) continue;
    // Accept "n" or "n, n" with identical values.
    std::string_view v = hd.value;
    uint64_t val = 0;
    bool any = false;
    size_t i = 0;
    for (; i < v.size() && v[i] >= '0' && v[i] <= '9'; i++) {
      any = true;
      val = val * 10 + uint64_t(v[i] - '0');
      if (val > (uint64_t(1) << 50)) break;
    }
    if (!any || (i < v.size() && v[i] != ',')) {
      if (err) *err = "invalid content-length";
      return false;
    }
    if (present && val != len) {
      if (err) *err = "conflicting content-length";
      return false;
    }
    present = true;
    len = val;
  }
  return true;
}

// The transfer codings of every Transfer-Encoding field line, in order
// (RFC 9112 §6.1: the list is the concatenation of the field lines).
static std::vector<std::string_view> te_codings(const Head& h) {
  std::vector<std::string_view> out;
  for (auto& hd : h.headers) {
    if (!iequals(hd.name, "transfer-encoding")) continue;
    std::string_view v = hd.value;
    for (;;) {
      size_t c = v.find(',');
      std::string_view t = v.substr(0, c);
      while (!t.empty() && (t.front() == ' ' || t.front() == '\t')) t.remove_prefix(1);
      while (!t.empty() && (t.back() == ' ' || t.back() == '\t')) t.remove_suffix(1);
      if (!t.empty()) out.push_back(t);
      if (c == std::string_view::npos) break;
      v.remove_prefix(c + 1);
    }
  }
  return out;
}

BodyDecoder::Mode request_body_mode(const Head& h, uint64_t& length, std::string* err) {
  length = 0;
  if (h.get("transfer-encoding")) {
    // RFC 9112 §6.1 / §6.3: a request whose final coding is not chunked cannot
    // be framed (400, then close); Transfer-Encoding next to Content-Length is
    // a smuggling vector, rejected rather than read as chunked. Chunked is the
    // only coding relayed (serve re-frames the body for the upstream), so any
    // other coding before it is refused too.
    auto te = te_codings(h);
    if (te.empty() || !iequals(te.back(), "chunked")) {
      if (err) *err = "transfer-encoding without chunked as the final coding";
      return BodyDecoder::Mode::UntilClose;  // caller treats err as fatal
    }
    if (h.get("content-length")) {
      if (err) *err = "both transfer-encoding and content-length";
      return BodyDecoder::Mode::UntilClose;
    }
    if (te.size() != 1) {
      if (err) *err = "unsupported transfer-encoding";
      return BodyDecoder::Mode::UntilClose;
    }
    return BodyDecoder::Mode::Chunked;
  }
  bool present;
  if (!parse_content_length(h, length, present, err)) return BodyDecoder::Mode::UntilClose;
  if (present && length > 0) return BodyDecoder::Mode::Length;
  return BodyDecoder::Mode::None;
}

BodyDecoder::Mode response_body_mode(const Head& h, const std::string& method, uint64_t& length) {
  length = 0;
  if (method == "HEAD" || h.status == 204 || h.status == 304 || (h.status >= 100 && h.status < 200))
    return BodyDecoder::Mode::None;
  if (h.get("transfer-encoding")) {
    // RFC 9112 §6.3 (3): chunked last => chunked; otherwise read until close.
    // Transfer-Encoding overrides Content-Length.
    auto te = te_codings(h);
    return !te.empty() && iequals(te.back(), "chunked") ? BodyDecoder::Mode::Chunked : BodyDecoder::Mode::UntilClose;
  }
  bool present;
  if (parse_content_length(h, length, present, nullptr) && present)
    return length ? BodyDecoder::Mode::Length : BodyDecoder::Mode::None;
  return BodyDecoder::Mode::UntilClose;
}

void BodyDecoder::reset(Mode m, uint64_t length) {
  mode_ = m;
  remaining_ = length;
  done_ = (m == Mode::None) || (m == Mode::Length && length == 0);
  cstate_ = CState::Size;
  line_.clear();
  err_.clear();
}

bool BodyDecoder::on_eof() {
  if (done_) return true;
  if (mode_ == Mode::UntilClose) {
    done_ = true;
    return true;
  }
  err_ = mode_ == Mode::Length ? "connection closed before message completed"
                               : "connection closed inside chunked body";
  return false;
}

size_t BodyDecoder::feed(const uint8_t* buf, size_t n, const std::function<void(const uint8_t*, size_t)>& sink) {
  if (done_) return 0;
  switch (mode_) {
    case Mode::None: done_ = true; return 0;
    case Mode::UntilClose:
      if (n) sink(buf, n);
      return n;
    case Mode::Length: {
      size_t take = n < remaining_ ? n : size_t(remaining_);
      if (take) sink(buf, take);
      remaining_ -= take;
      if (!remaining_) done_ = true;
      return take;
    }
    case Mode::Chunked: break;
  }
  size_t i = 0;
  while (i < n && !done_) {
    switch (cstate_) {
      case CState::Size:
      case CState::Trailer:
      case CState::DataCrlf: {
        const uint8_t* nl = static_cast<const uint8_t*>(memchr(buf + i, '\n', n - i));
        if (!nl) {
          line_.append(reinterpret_cast<const char*>(buf + i), n - i);
          if (line_.size() > 4096) {
            err_ = "chunk line too long";
            return SIZE_MAX;
          }
          return n;
        }
        size_t len = size_t(nl - (buf + i));
        line_.append(reinterpret_cast<const char*>(buf + i), len);
        i += len + 1;
        if (!line_.empty() && line_.back() == '\r') line_.pop_back();
        if (cstate_ == CState::DataCrlf) {
          if (!line_.empty()) {
            err_ = "missing CRLF after chunk data";
            return SIZE_MAX;
          }
          cstate_ = CState::Size;
        } else if (cstate_ == CState::Size) {
          uint64_t sz = 0;
          size_t k = 0;
          for (; k < line_.size(); k++) {
            char c = line_[k];
            int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                                                     : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
            if (d < 0) break;
            sz = sz * 16 + uint64_t(d);
            if (sz > (uint64_t(1) << 48)) {
              err_ = "chunk size too large";
              return SIZE_MAX;
            }
          }
          if (k == 0 || (k < line_.size() && line_[k] != ';' && line_[k] != ' ' && line_[k] != '\t')) {
            err_ = "invalid chunk size line";
            return SIZE_MAX;
          }
          if (sz == 0) cstate_ = CState::Trailer;
          else {
            remaining_ = sz;
            cstate_ = CState::Data;
          }
        } else {  // Trailer: ends at the empty line
          if (line_.empty()) done_ = true;
        }
        line_.clear();
        break;
      }
      case CState::Data: {
        size_t take = (n - i) < remaining_ ? (n - i) : size_t(remaining_);
        sink(buf + i, take);
        i += take;
        remaining_ -= take;
        if (!remaining_) cstate_ = CState::DataCrlf;
        break;
      }
    }
  }
  return i;
}

const char* reason_phrase(int s) {
  switch (s) {
    case 100: return "Continue";
    case 101: return "Switching Protocols";
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 206: return "Partial Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 304: return "Not Modified";
    case 307: return "Temporary Redirect";
    case 308: return "Permanent Redirect";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 408: return "Request Timeout";
    case 409: return "Conflict";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "";
  }
}

std::string http_date_now() {
  time_t t = time(nullptr);
  struct tm tm;
  gmtime_r(&t, &tm);
  char buf[64];
  strftime(buf, sizeof buf, "%a, %d %b %Y %H:%M:%S GMT", &tm);
  return buf;
}

std::string Url::host_header() const {
  bool dflt = ((scheme == "http" || scheme == "ws") && port == 80) || ((scheme == "https" || scheme == "wss") && port == 443);
  std::string h = host.find(':') != std::string::npos ? "[" + host + "]" : host;
  return dflt ? h : h + ":" + std::to_string(port);
}

bool parse_url(const std::string& url, Url& out, std::string* err) {
  size_t p = url.find("://");
  if (p == std::string::npos) {
    if (err) *err = "relative URL without a base: " + url;
    return false;
  }
  out = Url{};
  out.scheme = to_lower(url.substr(0, p));
  if (out.scheme == "http" || out.scheme == "ws") out.port = 80;
  else if (out.scheme == "https" || out.scheme == "wss") out.port = 443;
  else {
    if (err) *err = "unsupported URL scheme: " + out.scheme;
    return false;
  }
  std::string rest = url.substr(p + 3);
  size_t slash = rest.find_first_of("/?#");
  std::string auth = rest.substr(0, slash);
  std::string path = slash == std::string::npos ? "/" : rest.substr(slash);
  if (!path.empty() && path[0] == '?') path = "/" + path;
  size_t hash = path.find('#');
  if (hash != std::string::npos) path = path.substr(0, hash);
  if (path.empty()) path = "/";
  size_t at = auth.rfind('@');
  if (at != std::string::npos) auth = auth.substr(at + 1);
  if (!auth.empty() && auth[0] == '[') {
    size_t rb = auth.find(']');
    if (rb == std::string::npos) {
      if (err) *err = "invalid IPv6 host";
      return false;
    }
    out.host = auth.substr(1, rb - 1);
    if (rb + 1 < auth.size() && auth[rb + 1] == ':') out.port = uint16_t(atoi(auth.c_str() + rb + 2));
  } else {
    size_t colon = auth.rfind(':');
    if (colon != std::string::npos) {
      out.host = auth.substr(0, colon);
      int pt = atoi(auth.c_str() + colon + 1);
      if (pt <= 0 || pt > 65535) {
        if (err) *err = "invalid port";
        return false;
      }
      out.port = uint16_t(pt);
    } else {
      out.host = auth;
    }
  }
  if (out.host.empty()) {
    if (err) *err = "empty host";
    return false;
  }
  out.path = path;
  return true;
}

}  // namespace p2pt::http
