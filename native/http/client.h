// Streaming HTTP/1.1 client for the serve side's upstream requests.
//
// Replaces reqwest (reference serve.rs:62, :203-263): method + all headers
// except host/connection/transfer-encoding are forwarded (serve.rs:207-212),
// the body is sent with a Content-Length, and the response body is delivered
// piecewise as it arrives (reqwest's bytes_stream(), serve.rs:263) so SSE
// tokens are relayed one read at a time. Supports Content-Length, chunked and
// close-delimited (HTTP/1.0) responses, https:// via OpenSSL, and keep-alive
// connection pooling per origin. Reading can be paused for back-pressure.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "core/net.h"
#include "http/http.h"

namespace p2pt::http {

struct ClientRequest {
  std::string method;
  std::string url;
  std::vector<Header> headers;  // already filtered by the caller
  std::vector<Bytes> body;      // gathered, not concatenated
  uint64_t body_len = 0;
  bool force_content_length = false;  // send content-length even when 0
  // Streamed request body: `body` holds what is known at start, the rest comes
  // through ClientCall::write_body()/end_body(). Sent with content-length when
  // `content_length` >= 0, chunked otherwise; always on a fresh connection
  // (a stale pooled socket could not replay a body that is already gone).
  bool stream_body = false;
  int64_t content_length = -1;
};

struct ClientCallbacks {
  // Request bytes handed to the socket (connection established or reused).
  std::function<void(bool reused)> on_sent;
  std::function<void(const Head&)> on_head;
  // Body bytes; large pieces are views of the socket's receive buffer.
  std::function<void(Bytes)> on_data;
  // err empty => complete body received. `before_head` tells whether any
  // response head had been delivered (502 vs mid-stream ERROR semantics).
  std::function<void(const std::string& err, bool before_head)> on_done;
  // No TCP (or TLS) connection to the origin could be established: the
  // request never reached it (fires right before on_done). Safe to retry on
  // another origin.
  std::function<void()> on_connect_failed;
  // Streamed body: the socket's backlog drained below body_low_water after
  // having been above it (the producer may send more).
  std::function<void()> on_body_drain;
  size_t body_low_water = 64 * 1024;
};

class ClientConnPool;

class ClientCall : public std::enable_shared_from_this<ClientCall> {
 public:
  void pause();
  void resume();
  void cancel();
  bool finished() const { return finished_; }
  // Streamed request body (ClientRequest::stream_body).
  void write_body(Bytes b);
  void end_body();
  // Request-body bytes accepted but not yet handed to the kernel.
  size_t body_backlog() const;
  ~ClientCall();

 private:
  friend class HttpClient;
  void start();
  void attach(std::shared_ptr<TcpConn> c, bool reused);
  void on_data(const uint8_t* p, size_t n);
  void on_close(const std::string& err);
  void finish(const std::string& err);
  void process();

  Reactor* r_ = nullptr;
  std::shared_ptr<ClientConnPool> pool_;
  ClientRequest req_;
  ClientCallbacks cb_;
  Url url_;
  std::string pool_key_;
  std::shared_ptr<TcpConn> conn_;
  bool reused_ = false;
  bool got_any_ = false;
  bool head_done_ = false;
  bool finished_ = false;
  bool paused_ = false;
  bool keep_alive_ = false;
  bool counted_ = false;
  bool chunked_body_ = false;
  bool body_ended_ = false;
  uint64_t queued_body_ = 0;  // streamed pieces waiting for the connection
  void write_piece(const Bytes& b);
  Head head_;
  BodyDecoder body_;
  std::string buf_;
  uint64_t timeout_timer_ = 0;
};

class HttpClient {
 public:
  explicit HttpClient(Reactor& r);
  ~HttpClient();
  // Starts the request; callbacks run on the reactor thread. The returned
  // handle may be dropped (the call keeps itself alive until done).
  std::shared_ptr<ClientCall> request(ClientRequest req, ClientCallbacks cb);
  size_t idle_connections() const;
  // Keep >= min_ready established spare connections to url's origin (grows to
  // the recent peak concurrency, max 64). 0 disables.
  bool prewarm(const std::string& url, size_t min_ready, uint64_t idle_ttl_ms = 1000, std::string* err = nullptr);
  size_t warm_connections(const std::string& url) const;

 private:
  Reactor& r_;
  std::shared_ptr<ClientConnPool> pool_;
};

}  // namespace p2pt::http
