// HTTP/1.x message parsing and serialisation.
//
// Replaces hyper's HTTP/1 server (proxy side, reference proxy.rs:212) and
// reqwest's HTTP/1 client (serve side, reference serve.rs:62, :203-263).
// Incremental: heads are parsed once complete; bodies are decoded
// piecewise (Content-Length, chunked, or close-delimited for HTTP/1.0
// upstreams such as the reference's mock, tmp/mock_llm.py:97).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <string_view>
#include <vector>

namespace p2pt::http {

struct Header {
  std::string name;   // as received
  std::string value;  // trimmed
};

struct Head {
  // request
  std::string method;
  std::string target;
  // response
  int status = 0;
  std::string reason;
  // both
  int version_minor = 1;  // HTTP/1.x
  std::vector<Header> headers;

  const std::string* get(std::string_view name_ci) const;  // first match, case-insensitive
  bool has_token(std::string_view name_ci, std::string_view token_ci) const;
};

enum class ParseResult { Incomplete, Done, Error };

constexpr size_t kMaxHeadBytes = 64 * 1024;

// Parses a request head from the start of `buf`; on Done sets `consumed`.
ParseResult parse_request_head(std::string_view buf, Head& out, size_t& consumed, std::string* err);
ParseResult parse_response_head(std::string_view buf, Head& out, size_t& consumed, std::string* err);

class BodyDecoder {
 public:
  enum class Mode { None, Length, Chunked, UntilClose };
  void reset(Mode m, uint64_t length = 0);
  // Consume from buf; decoded data pieces go to `sink`. Returns bytes consumed,
  // or SIZE_MAX on a framing error (see error()).
  size_t feed(const uint8_t* buf, size_t n, const std::function<void(const uint8_t*, size_t)>& sink);
  // Peer closed the connection: true if that legitimately ends the body.
  bool on_eof();
  bool done() const { return done_; }
  Mode mode() const { return mode_; }
  const std::string& error() const { return err_; }

 private:
  enum class CState { Size, Data, DataCrlf, Trailer };
  Mode mode_ = Mode::None;
  bool done_ = true;
  uint64_t remaining_ = 0;
  CState cstate_ = CState::Size;
  std::string line_;
  std::string err_;
};

// Body framing for a request we received (RFC 9112 §6).
BodyDecoder::Mode request_body_mode(const Head& h, uint64_t& length, std::string* err);
// Body framing for a response to `method`.
BodyDecoder::Mode response_body_mode(const Head& h, const std::string& method, uint64_t& length);

const char* reason_phrase(int status);
bool iequals(std::string_view a, std::string_view b);
std::string to_lower(std::string_view s);
// Visible-ASCII header value check (hyper's HeaderValue::to_str()).
bool is_visible_ascii(std::string_view v);
std::string http_date_now();

// Parsed absolute URL (http/https only).
struct Url {
  std::string scheme;  // "http" / "https" / "ws" / "wss"
  std::string host;    // without brackets
  uint16_t port = 0;
  std::string path;    // path + query, at least "/"
  std::string host_header() const;  // host[:port] (port omitted if default)
  bool tls() const { return scheme == "https" || scheme == "wss"; }
};
bool parse_url(const std::string& url, Url& out, std::string* err);

}  // namespace p2pt::http
