#include "tunnel/serve.h"

#include <algorithm>

#include "core/crypto.h"
#include "core/log.h"
#include "tunnel/metrics.h"

namespace p2pt {

static const char* kT = "tunnel::serve";

std::shared_ptr<ServeSession> ServeSession::start(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg,
                                                  std::function<void(const std::string&)> done) {
  auto s = std::shared_ptr<ServeSession>(new ServeSession(r, ch, std::move(cfg)));
  s->done_ = std::move(done);
  std::weak_ptr<ServeSession> w = s;
  ch->on_message = [w](Bytes b) {
    if (auto x = w.lock()) x->on_message(std::move(b));
  };
  ch->on_closed = [w](const std::string& why) {
    if (auto x = w.lock()) {
      LOG_INFO(kT, "data channel closed, serve ending");
      x->stop("data channel closed: " + why);
    }
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

ServeSession::ServeSession(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg)
    : r_(r), ch_(std::move(ch)), cfg_(std::move(cfg)), client_(r) {
  sched_ = std::make_unique<FrameScheduler>(ch_);
  for (size_t a = 0; a <= cfg_.upstream.size();) {
    size_t c = cfg_.upstream.find(',', a);
    if (c == std::string::npos) c = cfg_.upstream.size();
    if (c > a) upstreams_.push_back(cfg_.upstream.substr(a, c - a));
    a = c + 1;
  }
  if (upstreams_.empty()) upstreams_.push_back(cfg_.upstream);
  outstanding_.assign(upstreams_.size(), 0);
  std::weak_ptr<ServeSession> w;  // set after construction via on_open
  ch_->on_buffered_low = [this] { sched_->pump(); };
}

ServeSession::~ServeSession() {
  if (hello_timer_) r_.cancel(hello_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  for (auto& kv : inflight_)
    if (kv.second.call) kv.second.call->cancel();
  if (ch_) {
    ch_->on_message = nullptr;
    ch_->on_closed = nullptr;
    ch_->on_open = nullptr;
    ch_->on_buffered_low = nullptr;
  }
}

void ServeSession::stop(const std::string& why) {
  if (stopped_) return;
  stopped_ = true;
  if (hello_timer_) r_.cancel(hello_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  hello_timer_ = ping_timer_ = 0;
  auto inflight = std::move(inflight_);
  inflight_.clear();
  std::fill(outstanding_.begin(), outstanding_.end(), 0);
  for (auto& kv : inflight)
    if (kv.second.call) kv.second.call->cancel();
  streams_.clear();
  auto done = std::move(done_);
  done_ = nullptr;
  if (done) done(why);
}

void ServeSession::on_open() {
  if (stopped_ || hello_timer_ || handshaken_) return;
  LOG_INFO(kT, "data channel ready, performing handshake...");
  std::weak_ptr<ServeSession> w = shared_from_this();
  hello_timer_ = r_.call_later_ms(cfg_.handshake_timeout_ms, [w] {
    if (auto s = w.lock()) {
      s->hello_timer_ = 0;
      s->stop("handshake timeout: no HELLO received within 5 minutes");
    }
  });
  sched_->set_watermarks(cfg_.high_water, cfg_.low_water, [w] {
    if (auto s = w.lock()) s->on_backpressure_relief();
  });
}

void ServeSession::on_message(Bytes raw) {
  if (stopped_) return;
  proto::Frame f;
  std::string err;
  if (!handshaken_) {
    if (!proto::decode(raw, f, &err)) {
      stop(err);
      return;
    }
    metrics::frame_recv(uint8_t(f.type), raw.size());
    on_hello(f);
    return;
  }
  if (!proto::decode(raw, f, &err)) {
    LOG_WARN(kT, "failed to decode tunnel message: %s", err.c_str());
    return;
  }
  metrics::frame_recv(uint8_t(f.type), raw.size());
  handle_frame(f);
}

void ServeSession::on_hello(const proto::Frame& f) {
  if (hello_timer_) {
    r_.cancel(hello_timer_);
    hello_timer_ = 0;
  }
  if (f.type != proto::MsgType::Hello) {
    stop(std::string("expected HELLO, got ") + proto::msg_type_name(f.type));
    return;
  }
  Json j;
  std::string err;
  proto::Hello hello;
  if (!proto::json_parse_bytes(f.payload, j, &err) || !proto::Hello::from_json(j, hello, &err)) {
    stop(err);
    return;
  }
  LOG_INFO(kT, "received HELLO: %s", j.dump().c_str());
  proto::Agree agree;
  std::vector<std::string> ours = proto::our_features();
  const std::string binding = ch_->channel_binding();
  if (!cfg_.secret.empty()) {
    // psk extension: the proxy must prove the shared secret on this channel.
    bool offered = std::find(hello.features.begin(), hello.features.end(), "psk") != hello.features.end();
    if (!offered || hello.psk_nonce.size() < 32 ||
        !equal_ct(hello.psk_mac, proto::psk_mac(cfg_.secret, "hello", hello.psk_nonce, binding))) {
      LOG_ERROR(kT, "authentication failed: HELLO without a valid shared-secret proof");
      metrics::counter_add("tunnel_auth_failures_total");
      stop("authentication failed: HELLO without a valid shared-secret proof");
      return;
    }
    ours.push_back("psk");
  }
  if (!proto::agree_from_hello(hello, agree, &err, ours)) {
    stop("handshake failed: " + err);
    return;
  }
  if (!cfg_.secret.empty()) agree.psk_mac = proto::psk_mac(cfg_.secret, "agree", hello.psk_nonce, binding);
  cancel_feature_ = std::find(agree.features.begin(), agree.features.end(), "cancel") != agree.features.end();
  sched_->send(proto::make_agree(agree));
  handshaken_ = true;
  LOG_INFO(kT, "sent AGREE, tunnel ready");
  if (cfg_.upstream_prewarm) {
    for (auto& u : upstreams_) {
      std::string perr;
      if (!client_.prewarm(u, cfg_.upstream_prewarm, cfg_.upstream_prewarm_ttl_ms, &perr))
        LOG_DEBUG(kT, "upstream prewarm disabled for %s: %s", u.c_str(), perr.c_str());
    }
  }
  last_pong_ms_ = Reactor::now_ms();
  send_ping();  // tokio::time::interval's first tick is immediate
}

void ServeSession::send_ping() {
  if (stopped_) return;
  if (cfg_.pong_timeout_ms && Reactor::now_ms() - last_pong_ms_ > cfg_.pong_timeout_ms) {
    stop("keepalive: no PONG within " + std::to_string(cfg_.pong_timeout_ms) + " ms");
    return;
  }
  sched_->send(proto::make_empty(proto::MsgType::Ping, 0));
  LOG_DEBUG(kT, "sent keepalive ping");
  std::weak_ptr<ServeSession> w = shared_from_this();
  ping_timer_ = r_.call_later_ms(cfg_.ping_interval_ms, [w] {
    if (auto s = w.lock()) {
      s->ping_timer_ = 0;
      s->send_ping();
    }
  });
}

void ServeSession::handle_frame(const proto::Frame& f) {
  using proto::MsgType;
  switch (f.type) {
    case MsgType::ReqHeaders: {
      Json j;
      std::string err;
      proto::RequestHeaders h;
      if (!proto::json_parse_bytes(f.payload, j, &err) || !proto::RequestHeaders::from_json(j, h, &err)) {
        // Reference ends the whole session here (serve.rs:113, Q3); we reject
        // just this stream.
        LOG_WARN(kT, "malformed REQ_HEADERS for stream %u: %s", f.stream_id, err.c_str());
        send_simple_response(f.stream_id, 400, "Bad Request: malformed request headers");
        return;
      }
      LOG_DEBUG(kT, "request %u %s %s", h.stream_id, h.method.c_str(), h.path.c_str());
      trace::event("serve", h.stream_id, "req_headers");
      uint32_t sid = h.stream_id;  // keyed by the JSON stream_id (serve.rs:118)
      Pending p;
      p.headers = std::move(h);
      streams_[sid] = std::move(p);
      break;
    }
    case MsgType::ReqBody: {
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end() && !f.payload.empty()) {
        it->second.body_len += f.payload.size();
        it->second.body.push_back(f.payload);  // zero-copy: keeps the message alive
      }
      break;
    }
    case MsgType::ReqEnd: {
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end()) {
        Pending p = std::move(it->second);
        streams_.erase(it);
        trace::event("serve", f.stream_id, "req_end");
        start_request(f.stream_id, std::move(p));
      }
      break;
    }
    case MsgType::Cancel: {
      auto it = inflight_.find(f.stream_id);
      if (it != inflight_.end()) {
        LOG_DEBUG(kT, "stream %u cancelled by peer", f.stream_id);
        auto call = it->second.call;
        release_upstream(it->second);
        inflight_.erase(it);
        if (call) call->cancel();
        metrics::counter_add("tunnel_streams_cancelled_total");
      }
      streams_.erase(f.stream_id);
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
      LOG_DEBUG(kT, "serve ignoring message type %s", proto::msg_type_name(f.type));
  }
}

void ServeSession::send_simple_response(uint32_t sid, uint16_t status, const std::string& body) {
  proto::ResponseHeaders rh;
  rh.stream_id = sid;
  rh.status = status;
  rh.headers.emplace_back("content-type", "text/plain");
  sched_->send(proto::make_res_headers(rh));
  sched_->send(proto::make_body(proto::MsgType::ResBody, sid, Bytes::copy(body)));
  sched_->send(proto::make_empty(proto::MsgType::ResEnd, sid));
}

static bool valid_method(const std::string& m) {
  if (m.empty()) return false;
  for (char c : m)
    if (!(isalnum(static_cast<unsigned char>(c)) || strchr("!#$%&'*+-.^_`|~", c))) return false;
  return true;
}

size_t ServeSession::pick_upstream() {
  size_t n = upstreams_.size(), best = rr_ % n;
  for (size_t k = 1; k < n; k++) {
    size_t i = (rr_ + k) % n;
    if (outstanding_[i] < outstanding_[best]) best = i;
  }
  rr_ = best + 1;
  return best;
}

void ServeSession::start_request(uint32_t sid, Pending p) {
  const size_t up = pick_upstream();
  std::string url = proto::build_upstream_url(upstreams_[up], cfg_.advertise, p.headers.path);
  LOG_DEBUG(kT, "forwarding %s %s -> %s", p.headers.method.c_str(), p.headers.path.c_str(), url.c_str());
  if (!valid_method(p.headers.method)) {
    LOG_ERROR(kT, "failed to handle request: invalid HTTP method");
    send_simple_response(sid, 400, "Bad Request: invalid HTTP method");
    return;
  }
  http::ClientRequest req;
  req.method = p.headers.method;
  req.url = url;
  bool had_cl = false;
  for (auto& kv : p.headers.headers) {
    const std::string& k = kv.first;
    if (http::iequals(k, "host") || http::iequals(k, "connection") || http::iequals(k, "transfer-encoding"))
      continue;
    if (http::iequals(k, "content-length")) {
      had_cl = true;  // recomputed from the body we actually received
      continue;
    }
    req.headers.push_back(http::Header{k, kv.second});
  }
  req.body = std::move(p.body);
  req.body_len = p.body_len;
  req.force_content_length = had_cl;

  std::weak_ptr<ServeSession> w = shared_from_this();
  metrics::counter_add("tunnel_upstream_requests_total");
  http::ClientCallbacks cb;
  cb.on_sent = [sid](bool) { trace::event("serve", sid, "upstream_sent"); };
  cb.on_head = [w, sid](const http::Head& h) {
    auto s = w.lock();
    if (!s || s->stopped_) return;
    proto::ResponseHeaders rh;
    rh.stream_id = sid;
    rh.status = uint16_t(h.status);
    for (auto& hd : h.headers)
      if (http::is_visible_ascii(hd.value)) proto::header_set(rh.headers, http::to_lower(hd.name), hd.value);
    s->sched_->send(proto::make_res_headers(rh));
    trace::event("serve", sid, "res_headers");
  };
  auto first = std::make_shared<bool>(true);
  cb.on_data = [w, sid, first](Bytes chunk) {
    auto s = w.lock();
    if (!s || s->stopped_) return;
    if (*first) {
      *first = false;
      trace::event("serve", sid, "first_body");
    }
    // `chunk` views the upstream socket's receive buffer (large reads) or is a
    // private copy (small ones, e.g. SSE tokens); frames slice it, no copy.
    size_t n = chunk.size();
    size_t cs = s->sched_->body_chunk();
    for (size_t off = 0; off < n; off += cs)
      s->sched_->send(proto::make_body(proto::MsgType::ResBody, sid, chunk.slice(off, cs)));
    if (s->sched_->over_high() && !s->upstream_paused_) {
      s->upstream_paused_ = true;
      for (auto& kv : s->inflight_)
        if (kv.second.call) kv.second.call->pause();
    }
  };
  cb.on_done = [w, sid, url](const std::string& err, bool before_head) {
    auto s = w.lock();
    if (!s) return;
    auto it = s->inflight_.find(sid);
    if (it == s->inflight_.end()) return;  // cancelled
    s->release_upstream(it->second);
    s->inflight_.erase(it);
    if (s->stopped_) return;
    if (!err.empty()) {
      if (before_head) {
        LOG_ERROR(kT, "upstream request failed: %s", err.c_str());
        metrics::counter_add("tunnel_upstream_errors_total");
        s->send_simple_response(sid, 502, "Bad Gateway: " + err);
        return;
      }
      LOG_ERROR(kT, "upstream stream error for stream %u: %s", sid, err.c_str());
      s->sched_->send(proto::make_error(sid, "upstream error: " + err));
    }
    s->sched_->send(proto::make_empty(proto::MsgType::ResEnd, sid));
    trace::event("serve", sid, "res_end");
    LOG_DEBUG(kT, "response %u complete", sid);
  };
  Inflight fl;
  fl.up = up;
  inflight_[sid] = fl;
  outstanding_[up]++;
  auto call = client_.request(std::move(req), std::move(cb));
  auto it = inflight_.find(sid);
  if (it != inflight_.end()) {
    it->second.call = call;
    if (upstream_paused_) call->pause();
  }
}

void ServeSession::on_backpressure_relief() {
  if (!upstream_paused_) return;
  upstream_paused_ = false;
  for (auto& kv : inflight_)
    if (kv.second.call) kv.second.call->resume();
}

}  // namespace p2pt
