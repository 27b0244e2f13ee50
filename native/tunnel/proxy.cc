#include "tunnel/proxy.h"

#include <algorithm>
#include <cstdio>

#include "core/crypto.h"
#include "core/log.h"
#include "core/net.h"
#include "http/http.h"
#include "tunnel/metrics.h"

namespace p2pt {

static const char* kT = "tunnel::proxy";

// One accepted client connection. Requests on a connection are handled one
// at a time (HTTP/1.1 keep-alive; pipelined requests wait in the buffer).
class ProxyConn : public std::enable_shared_from_this<ProxyConn> {
 public:
  ProxyConn(std::weak_ptr<ProxySession> s, std::shared_ptr<TcpConn> c) : sess_(std::move(s)), conn_(std::move(c)) {}
  ~ProxyConn() { cancel_timer(); }

  void start() {
    std::weak_ptr<ProxyConn> w = shared_from_this();
    conn_->on_data([w](const uint8_t* p, size_t n) {
      if (auto s = w.lock()) s->on_data(p, n);
    });
    conn_->on_close([w](const std::string& err) {
      if (auto s = w.lock()) s->on_client_closed(err);
    });
  }

  void on_res_headers(const proto::ResponseHeaders& rh) {
    if (!conn_ || conn_->closed() || aborted_) return;
    if (state_ != State::Awaiting && state_ != State::ReadingBody) {
      LOG_WARN(kT, "unexpected duplicate headers for stream %u", sid_);
      return;
    }
    cancel_timer();
    trace::event("proxy", sid_, "res_headers");
    write_response_head(rh);
  }

  void on_res_body(const Bytes& payload) {
    if (!conn_ || conn_->closed() || aborted_) return;
    if (!head_written_) {
      LOG_WARN(kT, "received body chunk before headers for stream %u", sid_);
      return;
    }
    if (!first_body_) {
      first_body_ = true;
      trace::event("proxy", sid_, "first_body");
    }
    if (payload.empty() || no_body_) return;
    body_sent_ += payload.size();
    if (chunked_) {
      char hdr[24];
      int n = snprintf(hdr, sizeof hdr, "%zx\r\n", payload.size());
      conn_->write(Bytes::copy(hdr, size_t(n)));
      conn_->write(payload);  // zero-copy from the received message
      conn_->write(Bytes::copy("\r\n", 2));
    } else {
      conn_->write(payload);
    }
  }

  void on_res_end() {
    if (!conn_ || conn_->closed() || aborted_) return;
    trace::event("proxy", sid_, "res_end");
    if (!head_written_) {
      fail_before_head("response ended before headers");
      return;
    }
    if (chunked_ && !no_body_) conn_->write(Bytes::copy("0\r\n\r\n", 5));
    response_done();
  }

  void on_res_error(const std::string& msg) {
    if (!conn_ || conn_->closed() || aborted_) return;
    if (!head_written_) {
      fail_before_head(msg);
      return;
    }
    // Q10: ending the body normally would hand the client a truncated body
    // that looks complete; abort the connection instead.
    LOG_WARN(kT, "tunnel error mid-stream for %u: %s", sid_, msg.c_str());
    // The head and body bytes already queued are flushed first so the client
    // sees the status and the partial body, then the connection ends without
    // the length/terminating chunk it was promised.
    stream_registered_ = false;
    aborted_ = true;
    conn_->pause_reading();
    conn_->close_after_flush();
  }

  void resume_reading() {
    if (conn_ && !conn_->closed() && !pipelined_hold_) conn_->resume_reading();
    if (conn_ && !inbuf_.empty()) process();
  }

 private:
  enum class State { Head, ReadingBody, Awaiting, Responding };

  void on_data(const uint8_t* p, size_t n) {
    if (state_ == State::ReadingBody && inbuf_.empty() && conn_) {
      // Request body straight from the socket buffer: REQ_BODY frames are
      // views of it (no staging copy into inbuf_).
      auto keep = shared_from_this();
      size_t used = 0;
      bool more = feed_body(p, n, &used);
      if (used == SIZE_MAX) return;
      if (used < n) inbuf_.append(reinterpret_cast<const char*>(p + used), n - used);
      if (more) process();
      return;
    }
    inbuf_.append(reinterpret_cast<const char*>(p), n);
    process();
  }

  void process() {
    auto keep = shared_from_this();
    while (conn_ && !conn_->closed()) {
      if (state_ == State::Head) {
        if (inbuf_.empty()) return;
        if (!parse_head()) return;
        continue;
      }
      if (state_ == State::ReadingBody) {
        if (inbuf_.empty()) return;
        size_t used = 0;
        bool more = feed_body(reinterpret_cast<const uint8_t*>(inbuf_.data()), inbuf_.size(), &used);
        if (used != SIZE_MAX) inbuf_.erase(0, used);
        if (!more) return;
        continue;
      }
      // Awaiting / Responding: further bytes belong to the next (pipelined)
      // request; hold them and stop reading until this response completes.
      if (inbuf_.size() > 1 << 20 && !pipelined_hold_) {
        pipelined_hold_ = true;
        conn_->pause_reading();
      }
      return;
    }
  }

  bool parse_head() {
    auto sess = sess_.lock();
    if (!sess) return false;
    http::Head h;
    size_t used = 0;
    std::string err;
    auto res = http::parse_request_head(inbuf_, h, used, &err);
    if (res == http::ParseResult::Incomplete) return false;
    if (res == http::ParseResult::Error) {
      simple_and_close(400, "text/plain", "Bad Request");
      return false;
    }
    inbuf_.erase(0, used);
    req_ = std::move(h);
    reset_response_state();
    keep_alive_ = req_.version_minor >= 1 ? !req_.has_token("connection", "close")
                                          : req_.has_token("connection", "keep-alive");
    uint64_t len = 0;
    auto mode = http::request_body_mode(req_, len, &err);
    if (!err.empty()) {
      simple_and_close(400, "text/plain", "Failed to read body");
      return false;
    }
    if (!sess->ready()) {
      // Only reachable with --listen-early (reference's dead 503 path, proxy.rs:257-263).
      body_.reset(mode, len);
      state_ = State::ReadingBody;
      reject_not_ready_ = true;
      if (body_.done()) finish_request_body();
      return true;
    }
    sid_ = sess->next_stream_id();
    metrics::counter_add("tunnel_streams_opened_total");
    trace::event("proxy", sid_, "accept");
    std::string path = req_.target;
    if (path.rfind("http://", 0) == 0 || path.rfind("https://", 0) == 0) {
      size_t s = path.find('/', path.find("://") + 3);
      path = s == std::string::npos ? "/" : path.substr(s);
    } else if (path == "*") {
      path = "/";
    }
    proto::RequestHeaders rh;
    rh.stream_id = sid_;
    rh.method = req_.method;
    rh.path = path;
    for (auto& hd : req_.headers)
      if (http::is_visible_ascii(hd.value)) proto::header_set(rh.headers, http::to_lower(hd.name), hd.value);
    LOG_DEBUG(kT, "proxying %s %s (stream %u)", rh.method.c_str(), rh.path.c_str(), sid_);
    proto::Frame hf = proto::make_req_headers(rh);
    if (hf.wire_size() > proto::kMaxFrameSize) {
      // Q15: the reference sends oversized headers unchecked.
      simple_and_close(431, "text/plain", "Request header fields too large for the tunnel");
      return false;
    }
    sess->register_stream(sid_, weak_from_this());
    stream_registered_ = true;
    sess->send(std::move(hf));
    if (req_.version_minor >= 1 && req_.has_token("expect", "100-continue"))
      conn_->write(std::string("HTTP/1.1 100 Continue\r\n\r\n"));
    body_.reset(mode, len);
    state_ = State::ReadingBody;
    if (body_.done()) finish_request_body();
    return true;
  }

  // Feeds request-body bytes; *used = bytes consumed (SIZE_MAX on a framing
  // error, after which the connection is closed). Returns whether processing
  // should continue (the body completed).
  bool feed_body(const uint8_t* data, size_t len, size_t* used_out) {
    *used_out = 0;
    auto sess = sess_.lock();
    if (!sess) return false;
    uint32_t sid = sid_;
    bool reject = reject_not_ready_;
    size_t cs = sess->body_chunk();
    auto conn = conn_;
    size_t used = body_.feed(data, len, [&](const uint8_t* d, size_t n) {
      if (reject) return;
      Bytes b = conn ? conn->rx_view(d, n) : Bytes::copy(d, n);
      for (size_t off = 0; off < n; off += cs)
        sess->send(proto::make_body(proto::MsgType::ReqBody, sid, b.slice(off, cs)));
    });
    *used_out = used;
    if (used == SIZE_MAX) {
      simple_and_close(400, "text/plain", "Failed to read body");
      return false;
    }
    if (body_.done()) {
      finish_request_body();
      return true;
    }
    if (sess->congested() && !conn_->reading_paused()) {
      conn_->pause_reading();
      sess->add_paused_reader(weak_from_this());
    }
    return false;
  }

  void finish_request_body() {
    auto sess = sess_.lock();
    if (!sess) return;
    if (reject_not_ready_) {
      reject_not_ready_ = false;
      state_ = State::Responding;
      write_simple(503, "text/plain", "Tunnel not ready");
      response_done();
      return;
    }
    sess->send(proto::make_empty(proto::MsgType::ReqEnd, sid_));
    trace::event("proxy", sid_, "req_end");
    if (state_ == State::ReadingBody) state_ = head_written_ ? State::Responding : State::Awaiting;
    if (!head_written_) {
      std::weak_ptr<ProxyConn> w = shared_from_this();
      timer_ = sess->reactor().call_later_ms(sess->config().header_timeout_ms, [w] {
        if (auto s = w.lock()) {
          s->timer_ = 0;
          s->on_header_timeout();
        }
      });
    }
    if (response_complete_) response_done();
  }

  void on_header_timeout() {
    if (head_written_) return;
    if (auto sess = sess_.lock()) sess->unregister_stream(sid_);
    stream_registered_ = false;
    metrics::counter_add("tunnel_streams_timeout_total");
    state_ = State::Responding;
    write_simple(504, "", "Tunnel response timeout");
    response_done();
  }

  void fail_before_head(const std::string& msg) {
    cancel_timer();
    stream_registered_ = false;
    metrics::counter_add("tunnel_streams_errors_total");
    write_simple(502, "text/plain", "Tunnel error: " + msg);
    if (state_ == State::ReadingBody) {
      // Response went out before the request body finished: drop the rest.
      keep_alive_ = false;
    }
    state_ = State::Responding;
    response_done();
  }

  void write_response_head(const proto::ResponseHeaders& rh) {
    head_written_ = true;
    if (state_ == State::Awaiting) state_ = State::Responding;
    int status = rh.status;
    if (status < 100 || status > 999) status = 502;
    no_body_ = req_.method == "HEAD" || status == 204 || status == 304 || (status >= 100 && status < 200);
    std::string out;
    out.reserve(256);
    char line[64];
    snprintf(line, sizeof line, "HTTP/1.1 %d %s\r\n", status, http::reason_phrase(status));
    out += line;
    bool has_cl = false, has_date = false;
    for (auto& kv : rh.headers) {
      if (http::iequals(kv.first, "transfer-encoding") || http::iequals(kv.first, "connection")) continue;
      if (http::iequals(kv.first, "content-length")) has_cl = true;
      if (http::iequals(kv.first, "date")) has_date = true;
      out += kv.first;
      out += ": ";
      out += kv.second;
      out += "\r\n";
    }
    if (!has_date) out += "date: " + http::http_date_now() + "\r\n";
    chunked_ = false;
    if (!no_body_ && !has_cl) {
      if (req_.version_minor >= 1) {
        chunked_ = true;
        out += "transfer-encoding: chunked\r\n";
      } else {
        keep_alive_ = false;  // close-delimited body for HTTP/1.0 clients
      }
    }
    if (!keep_alive_) out += "connection: close\r\n";
    else if (req_.version_minor == 0) out += "connection: keep-alive\r\n";
    out += "\r\n";
    conn_->write(std::move(out));
  }

  void write_simple(int status, const std::string& ctype, const std::string& body) {
    if (state_ == State::ReadingBody) keep_alive_ = false;
    std::string out;
    char line[64];
    snprintf(line, sizeof line, "HTTP/1.1 %d %s\r\n", status, http::reason_phrase(status));
    out += line;
    if (!ctype.empty()) out += "content-type: " + ctype + "\r\n";
    out += "content-length: " + std::to_string(body.size()) + "\r\n";
    out += "date: " + http::http_date_now() + "\r\n";
    if (!keep_alive_) out += "connection: close\r\n";
    out += "\r\n";
    if (req_.method != "HEAD") out += body;
    head_written_ = true;
    conn_->write(std::move(out));
  }

  void simple_and_close(int status, const std::string& ctype, const std::string& body) {
    keep_alive_ = false;
    write_simple(status, ctype, body);
    state_ = State::Responding;
    conn_->close_after_flush();
  }

  void response_done() {
    cancel_timer();
    if (stream_registered_) {
      if (auto sess = sess_.lock()) sess->unregister_stream(sid_);
      stream_registered_ = false;
    }
    if (state_ == State::ReadingBody) {
      // Response finished before the request body: complete it first.
      response_complete_ = true;
      return;
    }
    if (!keep_alive_) {
      conn_->close_after_flush();
      return;
    }
    state_ = State::Head;
    req_ = http::Head{};
    if (pipelined_hold_) {
      pipelined_hold_ = false;
      conn_->resume_reading();
    }
    if (!inbuf_.empty()) {
      std::weak_ptr<ProxyConn> w = shared_from_this();
      if (auto sess = sess_.lock())
        sess->reactor().post([w] {
          if (auto s = w.lock()) s->process();
        });
    }
  }

  void reset_response_state() {
    head_written_ = false;
    chunked_ = false;
    no_body_ = false;
    first_body_ = false;
    response_complete_ = false;
    body_sent_ = 0;
  }

  void on_client_closed(const std::string& err) {
    auto keep = shared_from_this();
    cancel_timer();
    auto sess = sess_.lock();
    if (stream_registered_ && sess) {
      LOG_DEBUG(kT, "HTTP client disconnected for stream %u%s%s", sid_, err.empty() ? "" : ": ", err.c_str());
      if (sess->cancel_feature()) {
        sess->send(proto::make_empty(proto::MsgType::Cancel, sid_));
        sess->unregister_stream(sid_);
      }
      stream_registered_ = false;
    }
    conn_.reset();
    if (sess) sess->conns_.erase(this);
  }

  void cancel_timer() {
    if (timer_) {
      if (auto sess = sess_.lock()) sess->reactor().cancel(timer_);
      timer_ = 0;
    }
  }

  std::weak_ptr<ProxySession> sess_;
  std::shared_ptr<TcpConn> conn_;
  std::string inbuf_;
  State state_ = State::Head;
  http::Head req_;
  http::BodyDecoder body_;
  uint32_t sid_ = 0;
  bool stream_registered_ = false;
  bool keep_alive_ = true;
  bool head_written_ = false;
  bool aborted_ = false;
  bool chunked_ = false;
  bool no_body_ = false;
  bool first_body_ = false;
  bool response_complete_ = false;
  bool pipelined_hold_ = false;
  bool reject_not_ready_ = false;
  uint64_t body_sent_ = 0;
  uint64_t timer_ = 0;
  friend class ProxySession;
};

// ---------------------------------------------------------------- session

std::shared_ptr<ProxySession> ProxySession::start(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg,
                                                  std::function<void(const std::string&)> done) {
  auto s = std::shared_ptr<ProxySession>(new ProxySession(r, ch, std::move(cfg)));
  s->done_ = std::move(done);
  std::weak_ptr<ProxySession> w = s;
  ch->on_message = [w](Bytes b) {
    if (auto x = w.lock()) x->on_message(std::move(b));
  };
  ch->on_closed = [w](const std::string& why) {
    if (auto x = w.lock()) x->stop("data channel closed: " + why);
  };
  ch->on_buffered_low = [w] {
    if (auto x = w.lock()) x->sched_->pump();
  };
  if (ch->is_open()) {
    LOG_INFO(kT, "data channel already open");
    s->on_open();
  } else {
    LOG_INFO(kT, "waiting for data channel to be ready...");
    ch->on_open = [w] {
      if (auto x = w.lock()) x->on_open();
    };
  }
  return s;
}

ProxySession::ProxySession(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg)
    : r_(r), ch_(std::move(ch)), cfg_(std::move(cfg)) {
  sched_ = std::make_unique<FrameScheduler>(ch_);
}

ProxySession::~ProxySession() {
  if (agree_timer_) r_.cancel(agree_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  if (ch_) {
    ch_->on_message = nullptr;
    ch_->on_closed = nullptr;
    ch_->on_open = nullptr;
    ch_->on_buffered_low = nullptr;
  }
  auto conns = std::move(conns_);
  for (auto& kv : conns)
    if (kv.second->conn_) {
      kv.second->conn_->on_close(nullptr);
      kv.second->conn_->close();
    }
}

void ProxySession::stop(const std::string& why) {
  if (stopped_) return;
  stopped_ = true;
  if (agree_timer_) r_.cancel(agree_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  agree_timer_ = ping_timer_ = 0;
  listener_.reset();  // like the reference, the listener dies with the session
  // Fail in-flight requests so clients are not left hanging.
  auto streams = std::move(streams_);
  streams_.clear();
  for (auto& kv : streams)
    if (auto c = kv.second.lock()) c->on_res_error("tunnel disconnected");
  auto done = std::move(done_);
  done_ = nullptr;
  if (done) done(why);
}

void ProxySession::on_open() {
  if (stopped_ || hello_sent_) return;
  LOG_INFO(kT, "data channel ready, performing handshake...");
  proto::Hello hello;
  hello.features = proto::our_features();
  if (!cfg_.secret.empty()) {  // psk extension: prove the shared secret on this channel
    uint8_t nonce[16];
    random_bytes(nonce, sizeof nonce);
    psk_nonce_ = hex_encode(nonce, sizeof nonce);
    hello.features.push_back("psk");
    hello.psk_nonce = psk_nonce_;
    hello.psk_mac = proto::psk_mac(cfg_.secret, "hello", psk_nonce_, ch_->channel_binding());
  }
  sched_->send(proto::make_hello(hello));
  hello_sent_ = true;
  LOG_INFO(kT, "sent HELLO");
  std::weak_ptr<ProxySession> w = shared_from_this();
  agree_timer_ = r_.call_later_ms(cfg_.handshake_timeout_ms, [w] {
    if (auto s = w.lock()) {
      s->agree_timer_ = 0;
      s->stop("handshake timeout: no AGREE received within 5 minutes");
    }
  });
  sched_->set_watermarks(cfg_.high_water, cfg_.low_water, [w] {
    if (auto s = w.lock()) s->on_relief();
  });
}

void ProxySession::on_message(Bytes raw) {
  if (stopped_) return;
  proto::Frame f;
  std::string err;
  if (!ready_) {
    if (!proto::decode(raw, f, &err)) {
      stop(err);
      return;
    }
    metrics::frame_recv(uint8_t(f.type), raw.size());
    on_agree(f);
    return;
  }
  if (!proto::decode(raw, f, &err)) {
    LOG_WARN(kT, "failed to decode tunnel message: %s", err.c_str());
    return;
  }
  metrics::frame_recv(uint8_t(f.type), raw.size());
  route(f);
}

void ProxySession::on_agree(const proto::Frame& f) {
  if (agree_timer_) {
    r_.cancel(agree_timer_);
    agree_timer_ = 0;
  }
  if (f.type != proto::MsgType::Agree) {
    stop(std::string("expected AGREE, got ") + proto::msg_type_name(f.type));
    return;
  }
  Json j;
  std::string err;
  proto::Agree agree;
  if (!proto::json_parse_bytes(f.payload, j, &err) || !proto::Agree::from_json(j, agree, &err)) {
    stop(err);
    return;
  }
  LOG_INFO(kT, "received AGREE: %s", j.dump().c_str());
  if (!cfg_.secret.empty()) {
    bool agreed = std::find(agree.features.begin(), agree.features.end(), "psk") != agree.features.end();
    if (!agreed ||
        !equal_ct(agree.psk_mac, proto::psk_mac(cfg_.secret, "agree", psk_nonce_, ch_->channel_binding()))) {
      LOG_ERROR(kT, "authentication failed: peer did not prove the shared secret");
      metrics::counter_add("tunnel_auth_failures_total");
      stop("authentication failed: peer did not prove the shared secret");
      return;
    }
  }
  cancel_feature_ = std::find(agree.features.begin(), agree.features.end(), "cancel") != agree.features.end();
  ready_ = true;
  last_pong_ms_ = Reactor::now_ms();
  send_ping();
  if (!listener_ && !cfg_.listen_early) {
    if (!bind_listener()) return;
  }
}

bool ProxySession::bind_listener() {
  std::string err;
  std::weak_ptr<ProxySession> w = shared_from_this();
  listener_ = TcpListener::bind(
      r_, cfg_.listen,
      [w](int fd, SockAddr) {
        if (auto s = w.lock()) s->accept(fd);
        else ::close(fd);
      },
      &err);
  if (!listener_) {
    stop(err);
    return false;
  }
  std::string addr = listener_->local_addr().str();
  LOG_INFO(kT, "proxy listening on http://%s", addr.c_str());
  if (cfg_.on_listening) cfg_.on_listening(addr);
  return true;
}

void ProxySession::accept(int fd) {
  if (stopped_) {
    ::close(fd);
    return;
  }
  trace::event("proxy", uint32_t(fd), "tcp_accept");
  auto tc = TcpConn::adopt(r_, fd);
  auto pc = std::make_shared<ProxyConn>(weak_from_this(), tc);
  conns_[pc.get()] = pc;
  pc->start();
}

void ProxySession::send_ping() {
  if (stopped_) return;
  if (cfg_.pong_timeout_ms && Reactor::now_ms() - last_pong_ms_ > cfg_.pong_timeout_ms) {
    stop("keepalive: no PONG within " + std::to_string(cfg_.pong_timeout_ms) + " ms");
    return;
  }
  sched_->send(proto::make_empty(proto::MsgType::Ping, 0));
  LOG_DEBUG(kT, "sent keepalive ping");
  std::weak_ptr<ProxySession> w = shared_from_this();
  ping_timer_ = r_.call_later_ms(cfg_.ping_interval_ms, [w] {
    if (auto s = w.lock()) {
      s->ping_timer_ = 0;
      s->send_ping();
    }
  });
}

void ProxySession::route(const proto::Frame& f) {
  using proto::MsgType;
  switch (f.type) {
    case MsgType::ResHeaders: {
      Json j;
      std::string err;
      proto::ResponseHeaders rh;
      if (!proto::json_parse_bytes(f.payload, j, &err) || !proto::ResponseHeaders::from_json(j, rh, &err)) {
        LOG_ERROR(kT, "failed to parse response headers: %s", err.c_str());
        return;
      }
      LOG_DEBUG(kT, "response headers for stream %u: status=%u", rh.stream_id, rh.status);
      auto it = streams_.find(rh.stream_id);  // routed by the JSON stream_id (proxy.rs:131)
      if (it != streams_.end())
        if (auto c = it->second.lock()) c->on_res_headers(rh);
      break;
    }
    case MsgType::ResBody: {
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end())
        if (auto c = it->second.lock()) c->on_res_body(f.payload);
      break;
    }
    case MsgType::ResEnd: {
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end()) {
        auto c = it->second.lock();
        streams_.erase(it);
        if (c) c->on_res_end();
      }
      break;
    }
    case MsgType::Error: {
      std::string msg = f.payload.str();
      LOG_ERROR(kT, "tunnel error for stream %u: %s", f.stream_id, msg.c_str());
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end()) {
        auto c = it->second.lock();
        streams_.erase(it);
        if (c) c->on_res_error(msg);
      }
      break;
    }
    case MsgType::Ping:
      sched_->send(proto::make_empty(MsgType::Pong, 0));
      LOG_DEBUG(kT, "received ping, sent pong");
      break;
    case MsgType::Pong:
      last_pong_ms_ = Reactor::now_ms();
      LOG_DEBUG(kT, "received pong");
      break;
    default:
      LOG_DEBUG(kT, "proxy ignoring message type %s", proto::msg_type_name(f.type));
  }
}

void ProxySession::on_relief() {
  auto readers = std::move(paused_readers_);
  paused_readers_.clear();
  for (auto& w : readers)
    if (auto c = w.lock()) c->resume_reading();
}

}  // namespace p2pt
