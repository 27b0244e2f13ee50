#include "tunnel/proxy.h"

#include <algorithm>
#include <cstdio>

#include "core/crypto.h"
#include "core/log.h"
#include "core/net.h"
#include "http/http.h"
#include "tunnel/assoc.h"
#include "tunnel/metrics.h"

namespace p2pt {

static const char* kT = "tunnel::proxy";

// The client connections of one reactor thread (the association thread's own
// or a worker's): stream registration, frames towards the session, and the
// RES_* frames the session routes back. Created, used and destroyed on its
// reactor's thread only.
class ProxyWorker : public std::enable_shared_from_this<ProxyWorker> {
 public:
  ProxyWorker(Reactor& r, Reactor& assoc, std::weak_ptr<ProxySession> sess,
              std::shared_ptr<ProxySession::Shared> shared, size_t index)
      : r_(r), assoc_(assoc), sess_(std::move(sess)), shared_(std::move(shared)), index_(index) {}
  ~ProxyWorker();
  void init() {
    std::weak_ptr<ProxySession> w = sess_;
    size_t k = index_;
    out_ = std::make_unique<Pipe<ProxySession::Ev>>(r_, assoc_, [w, k](ProxySession::Ev& ev) {
      if (auto s = w.lock()) s->on_event(k, ev);
    });
  }
  void handle(ProxySession::Cmd& c);
  // Fails every registered stream (the tunnel went away).
  void fail_all(const std::string& why);

  // ---- used by ProxyConn
  uint32_t next_stream_id() { return shared_->next_sid.fetch_add(1, std::memory_order_relaxed); }
  void register_stream(uint32_t sid, std::weak_ptr<ProxyConn> c) {
    streams_[sid] = std::move(c);
    out_->push(ProxySession::Ev{ProxySession::Ev::Route, sid});
  }
  void unregister_stream(uint32_t sid) {
    if (streams_.erase(sid)) out_->push(ProxySession::Ev{ProxySession::Ev::Unroute, sid});
  }
  void send(proto::Frame f) {
    ProxySession::Ev ev(ProxySession::Ev::Frame, f.stream_id);
    const bool urgent = f.type == proto::MsgType::ReqHeaders || f.type == proto::MsgType::ReqEnd;
    ev.frame = std::move(f);
    out_->push(std::move(ev), urgent);
  }
  bool ready() const { return shared_->ready.load(std::memory_order_relaxed); }
  size_t body_chunk() const { return shared_->body_chunk; }
  bool cancel_feature() const { return shared_->cancel_feature.load(std::memory_order_relaxed); }
  bool flow() const { return shared_->flow.load(std::memory_order_relaxed); }
  uint64_t rtt_us() const { return shared_->rtt_us.load(std::memory_order_relaxed); }
  const ProxyConfig& config() const { return shared_->cfg; }
  Reactor& reactor() { return r_; }
  void conn_closed(ProxyConn* c);
  // Where a connection's next request runs (ProxyRouter): kStay, kWorker
  // (the association thread's inline connection with a bulk request hands
  // its socket to a worker: bulk I/O off the association thread), or the
  // index of the association to hand the connection to.
  static constexpr int kStay = -1, kWorker = -2;
  int placement(ProxyConn* c, bool bulk);
  // Interactive requests in flight on this association (router).
  void interactive(int delta) { shared_->router->interactive(shared_->assoc_index, delta); }
  bool first_association() const { return shared_->assoc_index == 0; }
  void migrate(ProxyConn* c, int fd, Bytes unparsed);
  void hand_off(ProxyConn* c, int fd, Bytes unparsed, size_t dest);
  bool bulk_route(const std::string& key) { return shared_->router->bulk_route(key); }
  void note_route(const std::string& key, uint64_t bytes, bool streaming) {
    shared_->router->note_route(key, bytes, streaming);
  }

 private:
  void adopt(int fd, Bytes unparsed = Bytes(), uint64_t accepted_us = 0, bool counted = false);
  Reactor& r_;
  Reactor& assoc_;
  std::weak_ptr<ProxySession> sess_;
  std::shared_ptr<ProxySession::Shared> shared_;
  size_t index_;
  std::unique_ptr<Pipe<ProxySession::Ev>> out_;
  std::unordered_map<uint32_t, std::weak_ptr<ProxyConn>> streams_;
  std::unordered_map<ProxyConn*, std::shared_ptr<ProxyConn>> conns_;
};

// One accepted client connection. Requests on a connection are handled one
// at a time (HTTP/1.1 keep-alive; pipelined requests wait in the buffer).
class ProxyConn : public std::enable_shared_from_this<ProxyConn> {
 public:
  ProxyConn(std::weak_ptr<ProxyWorker> s, std::shared_ptr<TcpConn> c) : sess_(std::move(s)), conn_(std::move(c)) {}
  ~ProxyConn() {
    cancel_timer();
    end_interactive();
  }

  // TUNNEL_TRACE: when the listener accepted this connection and when its
  // connection thread took it over, stamped under its first request's id.
  void set_conn_times(uint64_t accepted_us, uint64_t adopted_us) {
    accepted_us_ = accepted_us;
    adopted_us_ = adopted_us;
  }

  void start() {
    std::weak_ptr<ProxyConn> w = shared_from_this();
    conn_->on_data([w](const uint8_t* p, size_t n) {
      if (auto s = w.lock()) s->on_data(p, n);
    });
    conn_->on_close([w](const std::string& err) {
      if (auto s = w.lock()) s->on_client_closed(err);
    });
    conn_->on_drain(
        [w] {
          if (auto s = w.lock()) s->maybe_grant();
        },
        kGrantLow);
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

  // `more`: the rest of a body frame that arrived in transport fragments
  // (each piece written zero-copy, one chunk for the whole frame).
  void on_res_body(const Bytes& payload, const std::vector<Bytes>* more = nullptr) {
    if (!conn_ || conn_->closed() || aborted_) return;
    if (!head_written_) {
      LOG_WARN(kT, "received body chunk before headers for stream %u", sid_);
      return;
    }
    if (!first_body_) {
      first_body_ = true;
      trace::event("proxy", sid_, "first_body");
    }
    size_t total = payload.size();
    if (more)
      for (auto& b : *more) total += b.size();
    if (!total || no_body_) return;
    body_sent_ += total;
    if (more && !more->empty()) {
      if (chunked_) {
        char hdr[24];
        int n = snprintf(hdr, sizeof hdr, "%zx\r\n", total);
        conn_->write(slab_copy(hdr, size_t(n)));
      }
      conn_->write(payload);
      for (auto& b : *more) conn_->write(b);
      if (chunked_) conn_->write(slab_copy("\r\n", 2));
      if (stream_registered_ && sess_flow()) {
        owed_ += total;
        maybe_grant();
      }
      return;
    }
    if (chunked_) {
      char hdr[24];
      int n = snprintf(hdr, sizeof hdr, "%zx\r\n", payload.size());
      if (payload.size() <= 1024) {
        // A token event: chunk header, data and CRLF as one small slab piece.
        char ev[1024 + 32];
        memcpy(ev, hdr, size_t(n));
        memcpy(ev + n, payload.data(), payload.size());
        memcpy(ev + n + payload.size(), "\r\n", 2);
        conn_->write(slab_copy(ev, size_t(n) + payload.size() + 2));
      } else {
        conn_->write(slab_copy(hdr, size_t(n)));
        conn_->write(payload);  // zero-copy from the received message
        conn_->write(slab_copy("\r\n", 2));
      }
    } else {
      conn_->write(payload);
    }
    if (stream_registered_ && sess_flow()) {
      owed_ += payload.size();
      maybe_grant();
    }
  }

  // "flow": RES_BODY bytes the client has taken (our output backlog for it is
  // small again) are credit for serve to send more of this stream.
  void maybe_grant() {
    if (owed_ < proto::kFlowGrantMin || !conn_ || conn_->closed() || conn_->pending_out() > kGrantLow) return;
    auto sess = sess_.lock();
    if (!sess) return;
    const uint64_t grow = rwin_.on_grant(owed_, Reactor::now_us(), sess->rtt_us());
    if (grow) metrics::counter_add("tunnel_flow_window_growths_total");
    const uint64_t g = owed_ + grow;
    sess->send(proto::make_credit(sid_, uint32_t(std::min<uint64_t>(g, UINT32_MAX))));
    owed_ = 0;
  }

  // "flow": serve granted more REQ_BODY bytes for this upload.
  void on_credit(uint32_t n) {
    send_credit_ += n;
    if (credit_paused_ && send_credit_ > 0) {
      credit_paused_ = false;
      if (trace::enabled()) waits_.end(0);
      update_reading();
      if (conn_ && !inbuf_.empty()) process();
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

  // Per-stream back-pressure from the session: this upload's frames pile up.
  void flow_pause() {
    flow_paused_ = true;
    if (trace::enabled()) waits_.begin(1);
    update_reading();
  }
  void flow_resume() {
    flow_paused_ = false;
    if (trace::enabled()) waits_.end(1);
    update_reading();
    if (conn_ && !inbuf_.empty()) process();
  }

  // The client socket is read unless a pipelined request waits, the session
  // holds this upload back, or serve's credit for it ran out.
  void update_reading() {
    if (!conn_ || conn_->closed()) return;
    if (pipelined_hold_ || flow_paused_ || credit_paused_) conn_->pause_reading();
    else conn_->resume_reading();
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
    if (sess->ready() && !pipelined_hold_) {
      // Move the connection, head and all, before any stream exists for it:
      // a bulk request to another association or off the association thread,
      // an interactive one on an extra association back to the first.
      uint64_t blen = 0;
      std::string e2;
      const bool big_upload =
          http::request_body_mode(h, blen, &e2) == http::BodyDecoder::Mode::Length && blen >= Placement::kBulkBytes;
      const bool bulk = big_upload || sess->bulk_route(BulkRoutes::key(h.method, h.target));
      const int dest = sess->placement(this, bulk);
      if (dest == ProxyWorker::kStay && !bulk && !interactive_) {
        interactive_ = true;  // counted until it ends (ProxyRouter::pick_bulk, pick_interactive)
        sess->interactive(+1);
      }
      if (dest != ProxyWorker::kStay) {
        int fd = conn_->release_fd();
        if (fd >= 0) {
          Bytes rest = Bytes::copy(inbuf_);
          inbuf_.clear();
          auto keep = shared_from_this();
          conn_.reset();
          if (dest == ProxyWorker::kWorker) sess->migrate(this, fd, std::move(rest));
          else sess->hand_off(this, fd, std::move(rest), size_t(dest));
          return false;
        }
      }
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
    if (adopted_us_) {  // the connection's first request
      if (accepted_us_) trace::event_at("proxy", sid_, "tcp_accept", accepted_us_);
      trace::event_at("proxy", sid_, "conn_adopt", adopted_us_);
      accepted_us_ = adopted_us_ = 0;
    }
    if (req_.method == "GET") trace::event("proxy", sid_, "get");  // tells bulk downloads apart in the traces
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
    send_credit_ = proto::flow_window();
    credit_paused_ = false;
    owed_ = 0;
    rwin_ = proto::FlowWindow{};
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
    bool reject = reject_not_ready_ || discard_body_;
    size_t cs = sess->body_chunk();
    auto conn = conn_;
    bool flow = sess->flow() && !discard_body_;
    size_t used = body_.feed(data, len, [&](const uint8_t* d, size_t n) {
      if (reject) return;
      if (!body_seen_) {
        body_seen_ = true;
        trace::event("proxy", sid, "body_first");
      }
      Bytes b = conn ? conn->rx_view(d, n) : Bytes::copy(d, n);
      for (size_t off = 0; off < n; off += cs)
        sess->send(proto::make_body(proto::MsgType::ReqBody, sid, b.slice(off, cs)));
      if (flow) send_credit_ -= int64_t(n);
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
    if (flow && send_credit_ <= 0 && !credit_paused_) {  // wait for serve's credit
      credit_paused_ = true;
      if (trace::enabled()) waits_.begin(0);
      update_reading();
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
    if (!discard_body_) {
      sess->send(proto::make_empty(proto::MsgType::ReqEnd, sid_));
      trace::event("proxy", sid_, "req_end");
      if (trace::enabled()) waits_.emit(sid_);
    }
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
    res_streaming_ = false;
    for (auto& kv : rh.headers) {
      if (http::iequals(kv.first, "transfer-encoding") || http::iequals(kv.first, "connection")) continue;
      if (http::iequals(kv.first, "content-type")) res_streaming_ = BulkRoutes::streaming_type(kv.second);
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

  void end_interactive() {
    if (!interactive_) return;
    interactive_ = false;
    if (auto sess = sess_.lock()) sess->interactive(-1);
  }

  void response_done() {
    cancel_timer();
    end_interactive();
    if (head_written_ && !req_.method.empty())
      if (auto sess = sess_.lock()) sess->note_route(BulkRoutes::key(req_.method, req_.target), body_sent_, res_streaming_);
    if (stream_registered_) {
      if (auto sess = sess_.lock()) sess->unregister_stream(sid_);
      stream_registered_ = false;
    }
    if (state_ == State::ReadingBody) {
      // Response finished before the request body (a 413, an upstream that
      // answered a streamed upload early): read and discard the rest of the
      // body so a client that sends everything before reading still gets to
      // the response. The stream is unregistered, so no Credit or Resume for
      // it will come: its pauses end here, and nothing more is forwarded.
      response_complete_ = true;
      discard_body_ = true;
      if (flow_paused_ || credit_paused_) {
        flow_paused_ = false;
        credit_paused_ = false;
        update_reading();
      }
      if (conn_ && !inbuf_.empty()) {
        std::weak_ptr<ProxyConn> w = shared_from_this();
        if (auto sess = sess_.lock())
          sess->reactor().post([w] {
            if (auto s = w.lock()) s->process();
          });
      }
      return;
    }
    if (!keep_alive_) {
      conn_->close_after_flush();
      return;
    }
    state_ = State::Head;
    req_ = http::Head{};
    // Pauses belonged to the stream that just ended (its Resume may never
    // come: the session drops a finished stream's pause state).
    if (pipelined_hold_ || flow_paused_ || credit_paused_) {
      pipelined_hold_ = false;
      flow_paused_ = false;
      credit_paused_ = false;
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
    body_seen_ = false;
    response_complete_ = false;
    discard_body_ = false;
    body_sent_ = 0;
  }

  void on_client_closed(const std::string& err) {
    auto keep = shared_from_this();
    cancel_timer();
    end_interactive();
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
    if (sess) sess->conn_closed(this);
  }

  void cancel_timer() {
    if (timer_) {
      if (auto sess = sess_.lock()) sess->reactor().cancel(timer_);
      timer_ = 0;
    }
  }

  std::weak_ptr<ProxyWorker> sess_;  // this connection's thread
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
  bool body_seen_ = false;  // TUNNEL_TRACE: the request's first body byte was stamped
  uint64_t accepted_us_ = 0, adopted_us_ = 0;
  bool response_complete_ = false;
  bool discard_body_ = false;    // response done mid-upload: drain the body, forward nothing
  bool pipelined_hold_ = false;
  bool reject_not_ready_ = false;
  bool flow_paused_ = false;
  bool credit_paused_ = false;   // "flow": upload out of serve's credit
  // TUNNEL_TRACE: the longest wait of this upload for serve's credit (0) and
  // for the session's per-stream back-pressure (1), stamped at req_end as
  // credit_wait/credit_go and flow_wait/flow_go.
  struct Waits {
    uint64_t start[2] = {0, 0}, best_from[2] = {0, 0}, best_to[2] = {0, 0};
    void begin(int k) { start[k] = Reactor::now_us(); }
    void end(int k) {
      if (!start[k]) return;
      const uint64_t now = Reactor::now_us();
      if (now - start[k] > best_to[k] - best_from[k]) {
        best_from[k] = start[k];
        best_to[k] = now;
      }
      start[k] = 0;
    }
    void emit(uint32_t sid) {
      static const char* names[2][2] = {{"credit_wait", "credit_go"}, {"flow_wait", "flow_go"}};
      for (int k = 0; k < 2; k++) {
        if (best_to[k]) {
          trace::event_at("proxy", sid, names[k][0], best_from[k]);
          trace::event_at("proxy", sid, names[k][1], best_to[k]);
        }
      }
      *this = Waits{};
    }
  } waits_;
  int64_t send_credit_ = proto::flow_window();
  uint64_t owed_ = 0;            // "flow": RES_BODY bytes delivered, not yet granted back
  proto::FlowWindow rwin_;       // "flow": RES_BODY window autotuning
  static constexpr size_t kGrantLow = 64 * 1024;
  bool sess_flow() const {
    auto s = sess_.lock();
    return s && s->flow();
  }
  uint64_t body_sent_ = 0;
  bool res_streaming_ = false;  // SSE / NDJSON response (never a bulk route)
  uint64_t timer_ = 0;
  bool counted_ = false;      // the router counts this connection on its association
  bool interactive_ = false;  // an interactive request in flight, counted on this association (router)
  friend class ProxyWorker;
};

ProxyWorker::~ProxyWorker() {
  auto conns = std::move(conns_);
  for (auto& kv : conns)
    if (kv.second->conn_) {
      kv.second->conn_->on_close(nullptr);
      kv.second->conn_->close();
    }
  out_.reset();
}

void ProxyWorker::adopt(int fd, Bytes unparsed, uint64_t accepted_us, bool counted) {
  auto tc = TcpConn::adopt(r_, fd);
  auto pc = std::make_shared<ProxyConn>(weak_from_this(), tc);
  pc->counted_ = counted;
  if (trace::enabled()) pc->set_conn_times(accepted_us, Reactor::now_us());
  conns_[pc.get()] = pc;
  pc->start();
  if (!unparsed.empty()) pc->on_data(unparsed.data(), unparsed.size());
}

void ProxyWorker::migrate(ProxyConn* c, int fd, Bytes unparsed) {
  if (!conns_.erase(c)) {
    ::close(fd);
    return;
  }
  ProxySession::Ev ev(ProxySession::Ev::Migrate, c->counted_ ? 1 : 0);
  ev.fd = fd;
  ev.frame.payload = std::move(unparsed);
  out_->push(std::move(ev));
}

int ProxyWorker::placement(ProxyConn* c, bool bulk) {
  const size_t own = shared_->assoc_index;
  auto& rt = *shared_->router;
  if (bulk && own == 0) {
    // The first association takes bulk too while no interactive request runs
    // on it (a bulk-only load, e.g. the 64 x 1 MB echo, then uses every
    // association); counted there like on the others.
    const int k = rt.pick_bulk(c->counted_);
    if (k > 0) return k;
    if (k == 0 && !c->counted_) {
      rt.count(0);
      c->counted_ = true;
    }
  }
  if (!bulk && own == 0 && c->counted_) {  // an interactive request on a connection counted as bulk here
    rt.release(0);
    c->counted_ = false;
  }
  if (!bulk) {
    // Interactive traffic runs on the first association, spilling over to
    // the others only under node-scale load (ProxyRouter::kSpill).
    const int k = rt.pick_interactive(own);
    return k >= 0 && size_t(k) != own ? k : kStay;
  }
  if (index_ == 0 && shared_->workers > 0) return kWorker;
  return kStay;
}

void ProxyWorker::hand_off(ProxyConn* c, int fd, Bytes unparsed, size_t dest) {
  const bool counted = c->counted_;
  if (!conns_.erase(c)) {
    ::close(fd);
    return;
  }
  out_->push(ProxySession::Ev{ProxySession::Ev::ConnClosed, 0});  // leaves this session's placement
  if (counted) shared_->router->release(shared_->assoc_index);
  metrics::counter_add("tunnel_assoc_handoffs_total");
  shared_->router->hand(dest, fd, std::move(unparsed));
}

void ProxyWorker::conn_closed(ProxyConn* c) {
  if (c->counted_) {
    c->counted_ = false;
    shared_->router->release(shared_->assoc_index);
  }
  if (conns_.erase(c)) out_->push(ProxySession::Ev{ProxySession::Ev::ConnClosed, 0});
}

void ProxyWorker::fail_all(const std::string& why) {
  auto streams = std::move(streams_);
  streams_.clear();
  LOG_DEBUG(kT, "worker %zu: failing %zu in-flight stream(s): %s", index_, streams.size(), why.c_str());
  for (auto& kv : streams)
    if (auto c = kv.second.lock()) c->on_res_error(why);
}

void ProxyWorker::handle(ProxySession::Cmd& c) {
  using Cmd = ProxySession::Cmd;
  if (c.kind == Cmd::Adopt) {
    adopt(c.fd, std::move(c.data), c.t_us, c.counted);
    return;
  }
  auto it = streams_.find(c.sid);
  if (it == streams_.end()) return;
  auto conn = it->second.lock();
  if (c.urgent) r_.flush_soon();  // the client write of a response's start, now
  switch (c.kind) {
    case Cmd::Headers:
      if (conn) conn->on_res_headers(*c.rh);
      break;
    case Cmd::Body:
      if (conn) conn->on_res_body(c.data, &c.more);
      break;
    case Cmd::End:
      streams_.erase(it);
      if (conn) conn->on_res_end();
      break;
    case Cmd::Error:
      streams_.erase(it);
      if (conn) conn->on_res_error(c.data.str());
      break;
    case Cmd::Pause:
      if (conn) conn->flow_pause();
      break;
    case Cmd::Resume:
      if (conn) conn->flow_resume();
      break;
    case Cmd::Credit:
      if (conn) conn->on_credit(c.bytes);
      break;
    case Cmd::Adopt:
      break;
  }
}

// ---------------------------------------------------------------- session

std::shared_ptr<ProxySession> ProxySession::start(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg,
                                                  std::function<void(const std::string&)> done, WorkerPool* pool) {
  auto s = std::shared_ptr<ProxySession>(new ProxySession(r, ch, std::move(cfg)));
  s->done_ = std::move(done);
  s->pool_ = pool;
  s->shared_->router->attach(s->cfg_.assoc_index, &r, s);
  s->init_links(pool);
  std::weak_ptr<ProxySession> w = s;
  ch->on_message = [w](Bytes b) {
    if (auto x = w.lock()) x->on_message(std::move(b));
  };
  ch->on_message_chain = [w](Bytes b, std::vector<Bytes>& more) {
    if (auto x = w.lock()) x->on_message(std::move(b), &more);
  };
  ch->on_closed = [w](const std::string& why) {
    if (auto x = w.lock()) x->stop("data channel closed: " + why);
  };
  ch->on_buffered_low = [w] {
    if (auto x = w.lock()) x->sched_->pump();
  };
  s->sched_->on_progress = [w] {
    if (auto x = w.lock()) x->check_paused();
  };
  auto gauge = [w](double (*f)(ProxySession&)) {
    return [w, f]() -> double {
      auto x = w.lock();
      return x ? f(*x) : 0.0;
    };
  };
  // Gauges read the session from the metrics thread (the first
  // association's): an extra association's session runs on another thread.
  if (s->cfg_.assoc_index == 0) {
    metrics::gauge_fn("tunnel_streams_inflight", gauge([](ProxySession& x) { return double(x.routes_.size()); }));
    metrics::gauge_fn("tunnel_streams_paused", gauge([](ProxySession& x) { return double(x.paused_.size()); }));
    metrics::gauge_fn("tunnel_scheduler_queued_bytes",
                      gauge([](ProxySession& x) { return double(x.sched_->queued_bytes()); }));
    metrics::gauge_fn("tunnel_channel_buffered_bytes",
                      gauge([](ProxySession& x) { return double(x.ch_->buffered_amount()); }));
  }
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
    : r_(r), ch_(std::move(ch)), cfg_(std::move(cfg)), shared_(std::make_shared<Shared>()) {
  sched_ = std::make_unique<FrameScheduler>(ch_);
  shared_->cfg = cfg_;
  shared_->cfg.on_listening = nullptr;
  shared_->cfg.router = nullptr;
  shared_->assoc_index = cfg_.assoc_index;
  shared_->router = cfg_.router ? cfg_.router : std::make_shared<ProxyRouter>();
  // Stream ids are per channel; an extra association's start at k << 28 so
  // the trace (TUNNEL_TRACE) and the logs tell the associations' streams apart.
  if (cfg_.assoc_index) shared_->next_sid = uint32_t(cfg_.assoc_index << 28) + 1;
}

void ProxySession::init_links(WorkerPool* pool) {
  size_t n = 1 + (pool ? pool->size() : 0);
  place_ = std::make_unique<Placement>(n, cfg_.inline_streams);
  shared_->workers = n - 1;
  std::weak_ptr<ProxySession> self = shared_from_this();
  for (size_t k = 0; k < n; k++) {
    Reactor& wr = k == 0 ? r_ : pool->reactor(k - 1);
    auto worker = std::make_shared<ProxyWorker>(wr, r_, self, shared_, k);
    std::weak_ptr<ProxyWorker> ww = worker;
    Link l;
    l.r = &wr;
    l.to = std::make_unique<Pipe<Cmd>>(r_, wr, [ww](Cmd& c) {
      if (auto x = ww.lock()) x->handle(c);
    });
    if (k == 0) worker->init();
    else wr.post_threadsafe([worker] { worker->init(); });  // init before any Cmd batch (FIFO)
    l.worker = std::move(worker);
    links_.push_back(std::move(l));
  }
}

// Drops the links: pending commands are discarded; each worker fails its
// in-flight streams (`fail_why`, if any) and is destroyed on its own thread
// one loop iteration later, after those error responses were written.
void ProxySession::release_links(const std::string& fail_why) {
  auto links = std::move(links_);
  links_.clear();
  for (size_t k = 0; k < links.size(); k++) {
    links[k].to.reset();
    // The task owns the only reference (moved in), so the worker is destroyed
    // on its own thread, never by this loop's scope.
    auto finish = [w = std::move(links[k].worker), fail_why]() mutable {
      if (!fail_why.empty()) w->fail_all(fail_why);
      Reactor& wr = w->reactor();
      wr.post([w]() mutable { w.reset(); });
      w.reset();
    };
    if (k == 0) finish();
    else links[k].r->post_threadsafe(std::move(finish));
  }
}

ProxySession::~ProxySession() {
  // No more connections handed to this session (its reactor may go next:
  // an extra association's thread is joined after its session is dropped).
  shared_->router->detach(cfg_.assoc_index);
  assoc_.reset();  // extra associations first (joins their threads)
  if (agree_timer_) r_.cancel(agree_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  if (wd_timer_) r_.cancel(wd_timer_);
  wd_timer_ = 0;
  if (ch_) {
    ch_->on_message = nullptr;
    ch_->on_message_chain = nullptr;
    ch_->on_closed = nullptr;
    ch_->on_open = nullptr;
    ch_->on_buffered_low = nullptr;
  }
  // Dropped without stop() (an extra association torn down from its own
  // side: its link drops the session): its in-flight requests still get an
  // error, or their clients wait on a response that never comes.
  release_links(stopped_ ? "" : "tunnel disconnected");
}

void ProxySession::stop(const std::string& why) {
  if (stopped_) return;
  stopped_ = true;
  ready_ = false;
  shared_->ready = false;
  if (agree_timer_) r_.cancel(agree_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  if (wd_timer_) r_.cancel(wd_timer_);
  wd_timer_ = 0;
  agree_timer_ = ping_timer_ = 0;
  shared_->router->set_ready(cfg_.assoc_index, false);
  assoc_.reset();
  listener_.reset();  // like the reference, the listener dies with the session
  routes_.clear();
  paused_.clear();
  // Fail in-flight requests so clients are not left hanging.
  release_links("tunnel disconnected");
  auto done = std::move(done_);
  done_ = nullptr;
  if (done) done(why);
}

void ProxySession::on_open() {
  if (stopped_ || hello_sent_) return;
  LOG_INFO(kT, "data channel ready, performing handshake...");
  shared_->body_chunk = sched_->body_chunk();  // path MTU known now; read by connection threads later
  proto::Hello hello;
  hello.features = proto::our_features();
  if (cfg_.assoc_index == 0 && cfg_.assoc > 1 && cfg_.assoc_pc) hello.assoc = std::min(cfg_.assoc, proto::kMaxAssoc);
  else hello.features.erase(std::remove(hello.features.begin(), hello.features.end(), "assoc"), hello.features.end());
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
    if (auto s = w.lock()) s->check_paused();
  });
}

void ProxySession::on_message(Bytes raw, std::vector<Bytes>* more) {
  if (stopped_) return;
  proto::Frame f;
  std::string err;
  std::vector<Bytes> none;
  const bool ok = proto::decode_chain(raw, more ? *more : none, f, &err);
  if (!ready_) {
    if (!ok) {
      stop(err);
      return;
    }
    metrics::frame_recv(uint8_t(f.type), f.wire_size());
    on_agree(f);
    return;
  }
  if (!ok) {
    LOG_WARN(kT, "failed to decode tunnel message: %s", err.c_str());
    return;
  }
  metrics::frame_recv(uint8_t(f.type), f.wire_size());
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
  shared_->cancel_feature =
      std::find(agree.features.begin(), agree.features.end(), "cancel") != agree.features.end();
  shared_->flow = std::find(agree.features.begin(), agree.features.end(), "flow") != agree.features.end();
  if (std::find(agree.features.begin(), agree.features.end(), "multistream") != agree.features.end())
    ch_->set_lanes(proto::kLanes);
  ready_ = true;
  shared_->ready = true;
  last_pong_ms_ = Reactor::now_ms();
  send_ping();
  watchdog();
  shared_->router->set_ready(cfg_.assoc_index, true);
  if (cfg_.assoc_index != 0) {
    LOG_INFO(kT, "association %zu ready", cfg_.assoc_index);
    return;  // an extra association: client connections come from the first one's router
  }
  if (!listener_ && !cfg_.listen_early) {
    if (!bind_listener()) return;
  }
  const bool agreed = std::find(agree.features.begin(), agree.features.end(), "assoc") != agree.features.end();
  if (agreed && agree.assoc > 1 && cfg_.assoc > 1 && cfg_.assoc_pc) {
    // Only where one association's thread is the limit: a same-host or LAN
    // path. On a WAN path the limit is the path (its RTT and loss), and
    // parallel associations would only take N congestion windows' share of
    // a shared bottleneck (bench/bench_fairness.py's criterion).
    const uint64_t a = ch_->path_rtt_us(), b = ch_->rtt_hint_us();
    const uint64_t rtt = a && b ? std::min(a, b) : a | b;
    if (rtt && rtt <= kAssocMaxRttUs) start_assoc(std::min(agree.assoc, cfg_.assoc));
    else LOG_INFO(kT, "extra associations not used: path RTT %.1f ms (> %.1f ms or unknown)", double(rtt) / 1e3,
                  double(kAssocMaxRttUs) / 1e3);
  }
}

// "assoc": offers the extra PeerConnections over this channel; each gets a
// proxy session of its own on its own thread, fed by this one's router.
void ProxySession::start_assoc(uint32_t count) {
  ProxyConfig c = cfg_;
  c.assoc = 1;
  c.router = shared_->router;
  c.on_listening = nullptr;
  WorkerPool* pool = pool_;
  auto factory = [c, pool](Reactor& r, std::shared_ptr<MessageChannel> ch, size_t k,
                           std::function<void(const std::string&)> done) -> std::shared_ptr<void> {
    ProxyConfig ck = c;
    ck.assoc_index = k;
    return ProxySession::start(r, std::move(ch), ck, std::move(done), pool);
  };
  std::weak_ptr<ProxySession> w = shared_from_this();
  auto send = [w](proto::Frame f) {
    if (auto s = w.lock(); s && !s->stopped_) s->sched_->send(std::move(f));
  };
  auto router = shared_->router;
  auto state = [router](size_t k, bool up, const std::string&) {
    if (!up) router->set_ready(k, false);
  };
  LOG_INFO(kT, "associations agreed: %u", count);
  assoc_ = AssocGroup::create(r_, true, count, *cfg_.assoc_pc, cfg_.busy_poll_us, factory, send, state);
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

void ProxySession::adopt_handed(int fd, Bytes unparsed, bool counted) {
  if (stopped_ || !ready_ || links_.empty()) {
    // This association is gone or not ready: back to the first one (which
    // closes the connection if it is gone itself).
    if (counted) shared_->router->release(cfg_.assoc_index);
    if (cfg_.assoc_index != 0) shared_->router->hand(0, fd, std::move(unparsed));
    else ::close(fd);
    return;
  }
  Cmd c{Cmd::Adopt};
  c.fd = fd;
  c.data = std::move(unparsed);
  c.counted = counted;
  if (trace::enabled()) c.t_us = Reactor::now_us();
  command(place_->pick(cfg_.assoc_index != 0), std::move(c));
}

void ProxySession::accept(int fd) {
  if (stopped_ || links_.empty()) {
    ::close(fd);
    return;
  }
  size_t k = place_->pick();
  Cmd c{Cmd::Adopt};
  c.fd = fd;
  if (trace::enabled()) c.t_us = Reactor::now_us();
  command(k, std::move(c));
}

// Send-path stall watchdog: once a second, frames or channel bytes that are
// waiting without any having moved since the last tick are logged with the
// scheduler / data channel / SCTP state (and counted), so a stalled tunnel
// says why, and the scheduler is pumped once more.
void ProxySession::watchdog() {
  if (stopped_) return;
  if (sched_ && sched_->stalled_tick()) {
    if (++wd_stalled_s_ == 1) metrics::counter_add("tunnel_send_stalls_total");
    if (wd_stalled_s_ <= 3 || wd_stalled_s_ % 10 == 0)
      LOG_WARN(kT, "send path stalled for %d s: %s", wd_stalled_s_, sched_->debug_state().c_str());
    sched_->pump();  // heals a missed channel wake-up; a no-op when the transport is the one waiting
  } else {
    wd_stalled_s_ = 0;
  }
  std::weak_ptr<ProxySession> w = shared_from_this();
  wd_timer_ = r_.call_later_ms(1000, [w] {
    if (auto s = w.lock()) {
      s->wd_timer_ = 0;
      s->watchdog();
    }
  });
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

void ProxySession::on_event(size_t thread, Ev& ev) {
  if (stopped_) return;
  switch (ev.kind) {
    case Ev::Route:
      routes_[ev.sid] = Route{thread, false};
      return;
    case Ev::Unroute:
      routes_.erase(ev.sid);
      paused_.erase(ev.sid);
      return;
    case Ev::ConnClosed:
      place_->release(thread);
      return;
    case Ev::Migrate: {
      place_->release(thread);
      metrics::counter_add("tunnel_conns_migrated_total");
      Cmd c{Cmd::Adopt};
      c.fd = ev.fd;
      c.data = std::move(ev.frame.payload);
      c.counted = ev.sid != 0;
      command(place_->pick(true), std::move(c));
      return;
    }
    case Ev::Frame:
      break;
  }
  bool body = ev.frame.type == proto::MsgType::ReqBody;
  uint32_t sid = ev.frame.stream_id;
  // A request goes out on the transport now, not after the rest of this
  // loop turn (Reactor::flush_soon).
  if (ev.frame.type == proto::MsgType::ReqHeaders || ev.frame.type == proto::MsgType::ReqEnd) r_.flush_soon();
  sched_->send(std::move(ev.frame));
  if (!body) return;
  auto it = routes_.find(sid);
  if (it == routes_.end() || it->second.paused) return;
  // Per-stream back-pressure for uploads: pause just this client's reads.
  size_t q = sched_->stream_queued(sid);
  if (q > cfg_.stream_budget || (q > FrameScheduler::kInteractive && sched_->over_high())) {
    it->second.paused = true;
    paused_.insert(sid);
    command(it->second.thread, Cmd{Cmd::Pause, sid});
  }
}

void ProxySession::check_paused() {
  if (paused_.empty() || stopped_ || sched_->over_high()) return;
  for (auto p = paused_.begin(); p != paused_.end();) {
    uint32_t sid = *p;
    auto it = routes_.find(sid);
    if (it == routes_.end()) {
      p = paused_.erase(p);
      continue;
    }
    if (sched_->stream_queued(sid) <= cfg_.stream_budget / 4) {
      it->second.paused = false;
      p = paused_.erase(p);
      command(it->second.thread, Cmd{Cmd::Resume, sid});
      continue;
    }
    ++p;
  }
}

void ProxySession::route(const proto::Frame& f) {
  using proto::MsgType;
  switch (f.type) {
    case MsgType::ResHeaders: {
      Json j;
      std::string err;
      auto rh = std::make_shared<proto::ResponseHeaders>();
      if (!proto::json_parse_bytes(f.payload, j, &err) || !proto::ResponseHeaders::from_json(j, *rh, &err)) {
        LOG_ERROR(kT, "failed to parse response headers: %s", err.c_str());
        return;
      }
      LOG_DEBUG(kT, "response headers for stream %u: status=%u", rh->stream_id, rh->status);
      uint32_t sid = rh->stream_id;  // routed by the JSON stream_id (proxy.rs:131)
      auto it = routes_.find(sid);
      if (it != routes_.end()) {
        Cmd c{Cmd::Headers, sid};
        c.urgent = true;
        c.rh = std::move(rh);
        command(it->second.thread, std::move(c));
      }
      break;
    }
    case MsgType::ResBody: {
      auto it = routes_.find(f.stream_id);
      if (shared_->flow.load(std::memory_order_relaxed))
        shared_->rtt_us.store(ch_ ? ch_->rtt_hint_us() : 0, std::memory_order_relaxed);
      if (it != routes_.end()) {
        const bool first = !it->second.body_seen;
        if (first) {
          it->second.body_seen = true;
          trace::event("proxy", f.stream_id, "chan_rx");
          trace::rx_stamps("proxy", f.stream_id);
        }
        Cmd c{Cmd::Body, f.stream_id};
        c.urgent = first;
        c.data = f.more.empty() ? links_[it->second.thread].to->stage(f.payload) : f.payload;
        c.more = f.more;
        command(it->second.thread, std::move(c));
      }
      break;
    }
    case MsgType::ResEnd: {
      auto it = routes_.find(f.stream_id);
      if (it != routes_.end()) {
        size_t k = it->second.thread;
        routes_.erase(it);
        paused_.erase(f.stream_id);
        command(k, Cmd{Cmd::End, f.stream_id});
      }
      break;
    }
    case MsgType::Error: {
      std::string msg = f.payload.str();
      LOG_ERROR(kT, "tunnel error for stream %u: %s", f.stream_id, msg.c_str());
      auto it = routes_.find(f.stream_id);
      if (it != routes_.end()) {
        size_t k = it->second.thread;
        routes_.erase(it);
        paused_.erase(f.stream_id);
        Cmd c{Cmd::Error, f.stream_id};
        c.data = f.payload;
        command(k, std::move(c));
      }
      break;
    }
    case MsgType::Credit: {
      auto it = routes_.find(f.stream_id);
      if (it != routes_.end() && shared_->flow) {
        Cmd c{Cmd::Credit, f.stream_id};
        c.bytes = proto::credit_bytes(f);
        command(it->second.thread, std::move(c));
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
    case MsgType::Assoc:
      if (assoc_) assoc_->on_frame(f);
      break;
    default:
      LOG_DEBUG(kT, "proxy ignoring message type %s", proto::msg_type_name(f.type));
  }
}

// ---------------------------------------------------------------- router

void ProxyRouter::attach(size_t k, Reactor* r, std::weak_ptr<ProxySession> s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (t_.size() <= k) t_.resize(k + 1);
  t_[k].r = r;
  t_[k].s = std::move(s);
}

void ProxyRouter::set_ready(size_t k, bool ready) {
  std::lock_guard<std::mutex> lk(mu_);
  if (k < t_.size()) t_[k].ready = ready;
}

int ProxyRouter::pick_bulk(bool counted_on_first) {
  std::lock_guard<std::mutex> lk(mu_);
  int best = -1;
  for (size_t k = 1; k < t_.size(); k++)
    if (t_[k].ready && (best < 0 || t_[k].conns < t_[size_t(best)].conns)) best = int(k);
  if (best < 0) return -1;  // no extra association: placement as without the extension
  // The first association is a candidate while no interactive request has run
  // on it for quiet_us_ (ties go to an extra one; a connection already counted
  // there stays unless another association has fewer). A bulk-only load uses
  // every association; next to interactive traffic the first one stays clear.
  const bool quiet = !last_interactive_us_ || Reactor::now_us() - last_interactive_us_ >= quiet_us_;
  if (!t_.empty() && t_[0].ready && t_[0].interactive == 0 && quiet) {
    const size_t c0 = t_[0].conns - (counted_on_first && t_[0].conns ? 1 : 0);
    if (c0 < t_[size_t(best)].conns || (counted_on_first && c0 <= t_[size_t(best)].conns)) return 0;
  }
  return best;
}

void ProxyRouter::count(size_t k) {
  std::lock_guard<std::mutex> lk(mu_);
  if (k < t_.size()) t_[k].conns++;
}

void ProxyRouter::interactive(size_t k, int delta) {
  std::lock_guard<std::mutex> lk(mu_);
  if (k >= t_.size()) return;
  if (k == 0) last_interactive_us_ = std::max<uint64_t>(Reactor::now_us(), 1);
  if (delta > 0) t_[k].interactive += size_t(delta);
  else t_[k].interactive -= std::min(t_[k].interactive, size_t(-delta));
}

int ProxyRouter::pick_interactive(size_t own) {
  std::lock_guard<std::mutex> lk(mu_);
  if (t_.empty()) return -1;
  if (own != 0 && own < t_.size() && t_[own].ready) {
    // A connection that spilled over stays until the first association is
    // well below the threshold again (hysteresis: no move per request while
    // the load hovers around it).
    return t_[0].ready && t_[0].interactive < kSpill / 2 ? 0 : int(own);
  }
  if (t_[0].interactive < kSpill || t_.size() < 2 || (load_gate_ && load(0) < kSpillLoad))
    return t_[0].ready || own == 0 ? 0 : -1;
  // Node-scale load on a busy first association thread: the ready extra
  // association with the fewest interactive requests whose thread still has
  // idle time (with the load gate, the default). When every thread is busy (a
  // CPU-bound process: 1024 streams on the pool box's 16-CPU quota), spreading
  // only adds per-association overhead — smaller batches, more packets and
  // SACKs per token — so the request stays on the first (profiles/r06/b13,
  // b20: events 0.855 / 0.851 of direct gated vs 0.841 / 0.838 without).
  int best = 0;
  for (size_t k = 1; k < t_.size(); k++)
    if (t_[k].ready && (!load_gate_ || load(k) < kSpillLoad) &&
        (best == 0 || t_[k].interactive < t_[size_t(best)].interactive))
      best = int(k);
  return best;
}

void ProxyRouter::hand(size_t k, int fd, Bytes unparsed) {
  auto self = shared_from_this();
  std::lock_guard<std::mutex> lk(mu_);
  // An extra association that is gone (detached) sends the connection to the
  // first one instead.
  if (k > 0 && (k >= t_.size() || !t_[k].r)) k = 0;
  if (k >= t_.size() || !t_[k].r) {
    ::close(fd);
    return;
  }
  if (k > 0) t_[k].conns++;
  // Posted under mu_: detach() takes mu_ before the association's reactor
  // goes away, so nothing is posted to a destroyed reactor.
  t_[k].r->post_threadsafe([self, s = t_[k].s, k, fd, unparsed = std::move(unparsed)]() mutable {
    if (auto x = s.lock()) {
      x->adopt_handed(fd, std::move(unparsed), k > 0);
      return;
    }
    if (k > 0) {  // its session is gone: back to the first association
      self->release(k);
      self->hand(0, fd, std::move(unparsed));
    } else {
      ::close(fd);
    }
  });
}

void ProxyRouter::detach(size_t k) {
  std::lock_guard<std::mutex> lk(mu_);
  if (k >= t_.size()) return;
  t_[k].r = nullptr;
  t_[k].s.reset();
  t_[k].ready = false;
}

double ProxyRouter::load(size_t k) const {
  if (load_fn_) return load_fn_(k);
  return k < t_.size() && t_[k].r ? t_[k].r->load() : 1.0;
}

void ProxyRouter::release(size_t k) {
  std::lock_guard<std::mutex> lk(mu_);
  if (k < t_.size() && t_[k].conns) t_[k].conns--;
}

size_t ProxyRouter::connections(size_t k) {
  std::lock_guard<std::mutex> lk(mu_);
  return k < t_.size() ? t_[k].conns : 0;
}

bool ProxyRouter::bulk_route(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  return routes_.bulk(key);
}

void ProxyRouter::note_route(const std::string& key, uint64_t bytes, bool streaming) {
  std::lock_guard<std::mutex> lk(mu_);
  routes_.note(key, bytes, streaming);
}

}  // namespace p2pt
