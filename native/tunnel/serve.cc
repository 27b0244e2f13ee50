#include "tunnel/serve.h"

#include <algorithm>

#include "core/crypto.h"
#include "core/log.h"
#include "tunnel/assoc.h"
#include "tunnel/metrics.h"

namespace p2pt {

static const char* kT = "tunnel::serve";

// Runs upstream calls on one reactor (the association thread's own or a
// worker's) and reports frames back to the session through a Pipe. Created,
// used and destroyed on its reactor's thread only.
class ServeWorker : public std::enable_shared_from_this<ServeWorker> {
 public:
  ServeWorker(Reactor& r, Reactor& assoc, std::weak_ptr<ServeSession> sess, const ServeConfig& cfg,
              std::vector<std::string> upstreams, bool is_inline)
      : r_(r), assoc_(assoc), sess_(std::move(sess)), cfg_(cfg), upstreams_(std::move(upstreams)),
        inline_(is_inline) {}

  ~ServeWorker() {
    auto calls = std::move(calls_);
    for (auto& kv : calls)
      if (kv.second.call) kv.second.call->cancel();
    client_.reset();
    out_.reset();
  }

  void init() {
    client_ = std::make_unique<http::HttpClient>(r_);
    std::weak_ptr<ServeSession> w = sess_;
    out_ = std::make_unique<Pipe<ServeSession::Ev>>(r_, assoc_, [w](ServeSession::Ev& ev) {
      if (auto s = w.lock()) s->on_event(ev);
    });
  }

  void handle(ServeSession::Cmd& c) {
    using Cmd = ServeSession::Cmd;
    switch (c.kind) {
      case Cmd::Start:
        start(c.sid, std::move(c.req), c.body_chunk, c.retryable, c.grant);
        r_.flush_soon();  // the upstream request is written now, not after this turn's token work
        break;
      case Cmd::Cancel: {
        auto it = calls_.find(c.sid);
        if (it == calls_.end()) break;
        auto call = it->second.call;
        calls_.erase(it);
        if (call) call->cancel();
        break;
      }
      case Cmd::Pause:
      case Cmd::Resume: {
        auto it = calls_.find(c.sid);
        if (it != calls_.end() && it->second.call) {
          if (c.kind == Cmd::Pause) it->second.call->pause();
          else it->second.call->resume();
        }
        break;
      }
      case Cmd::Prewarm: prewarm(); break;
      case Cmd::Body:
      case Cmd::BodyEnd: {
        auto it = calls_.find(c.sid);
        if (it == calls_.end() || !it->second.call) break;
        if (c.kind == Cmd::BodyEnd) {
          it->second.call->end_body();
          break;
        }
        it->second.owed += c.data.size();
        it->second.call->write_body(std::move(c.data));
        for (auto& b : c.more) {
          it->second.owed += b.size();
          it->second.call->write_body(std::move(b));
        }
        maybe_grant(c.sid, it->second);
        break;
      }
    }
  }

 private:
  void prewarm() {
    if (prewarmed_ || !cfg_.upstream_prewarm) return;
    prewarmed_ = true;
    for (auto& u : upstreams_) {
      std::string perr;
      if (!client_->prewarm(u, cfg_.upstream_prewarm, cfg_.upstream_prewarm_ttl_ms, &perr))
        LOG_DEBUG(kT, "upstream prewarm disabled for %s: %s", u.c_str(), perr.c_str());
    }
  }

  struct CallState {
    std::shared_ptr<http::ClientCall> call;
    bool grant = false;  // "flow": hand consumed streamed-body bytes back as credit
    uint64_t owed = 0;
  };

  // Streamed request body: the bytes the upstream socket took off our hands
  // are credit the session can give back to the proxy ("flow").
  void maybe_grant(uint32_t sid, CallState& cs) {
    if (!cs.grant || !cs.owed || !cs.call || cs.call->body_backlog() > 64 * 1024) return;
    ServeSession::Ev ev(ServeSession::Ev::Credit, sid);
    ev.bytes = uint32_t(std::min<uint64_t>(cs.owed, UINT32_MAX));
    cs.owed -= ev.bytes;
    out_->push(std::move(ev));
  }

  // urgent: the start of a response (headers, first body): handed to the
  // association thread at once, not at the end of this loop turn.
  void emit(uint32_t sid, proto::Frame f, bool urgent = false) {
    ServeSession::Ev ev(ServeSession::Ev::Frame, sid);
    if (f.type == proto::MsgType::ResBody && f.more.empty()) f.payload = out_->stage(f.payload);
    ev.frame = std::move(f);
    out_->push(std::move(ev), urgent);
  }

  void simple_response(uint32_t sid, uint16_t status, const std::string& body) {
    proto::ResponseHeaders rh;
    rh.stream_id = sid;
    rh.status = status;
    rh.headers.emplace_back("content-type", "text/plain");
    emit(sid, proto::make_res_headers(rh));
    emit(sid, proto::make_body(proto::MsgType::ResBody, sid, Bytes::copy(body)));
    emit(sid, proto::make_empty(proto::MsgType::ResEnd, sid));
  }

  void start(uint32_t sid, http::ClientRequest req, size_t body_chunk, bool retryable, bool grant) {
    if (!inline_) prewarm();  // workers warm their own pools on first use
    std::weak_ptr<ServeWorker> w = shared_from_this();
    http::ClientCallbacks cb;
    if (req.stream_body) {
      cb.on_body_drain = [w, sid] {
        auto s = w.lock();
        if (!s) return;
        auto it = s->calls_.find(sid);
        if (it != s->calls_.end()) s->maybe_grant(sid, it->second);
      };
    }
    // Unreachable upstream: with other upstreams to try, the request goes back
    // to the session untouched (it never left this host).
    std::shared_ptr<ServeSession::Unreachable> back;
    if (retryable) {
      back = std::make_shared<ServeSession::Unreachable>();
      back->req = req;  // header strings + body views: no body copy
    }
    auto unreachable = std::make_shared<bool>(false);
    cb.on_connect_failed = [unreachable] { *unreachable = true; };
    cb.on_sent = [sid](bool) { trace::event("serve", sid, "upstream_sent"); };
    cb.on_head = [w, sid](const http::Head& h) {
      auto s = w.lock();
      if (!s) return;
      proto::ResponseHeaders rh;
      rh.stream_id = sid;
      rh.status = uint16_t(h.status);
      for (auto& hd : h.headers)
        if (http::is_visible_ascii(hd.value)) proto::header_set(rh.headers, http::to_lower(hd.name), hd.value);
      s->emit(sid, proto::make_res_headers(rh), true);
      trace::event("serve", sid, "res_headers");
    };
    auto first = std::make_shared<bool>(true);
    size_t cs = body_chunk ? body_chunk : proto::kMaxBodyChunk;
    cb.on_data = [w, sid, first, cs](Bytes chunk) {
      auto s = w.lock();
      if (!s) return;
      const bool urgent = *first;
      if (*first) {
        *first = false;
        trace::event("serve", sid, "first_body");
      }
      // `chunk` views the upstream socket's receive buffer (large reads) or is a
      // private copy (small ones, e.g. SSE tokens); frames slice it, no copy.
      size_t n = chunk.size();
      for (size_t off = 0; off < n; off += cs)
        s->emit(sid, proto::make_body(proto::MsgType::ResBody, sid, chunk.slice(off, cs)), urgent && off + cs >= n);
    };
    cb.on_done = [w, sid, back, unreachable](const std::string& err, bool before_head) {
      auto s = w.lock();
      if (!s) return;
      auto it = s->calls_.find(sid);
      if (it == s->calls_.end()) return;  // cancelled
      s->calls_.erase(it);
      ServeSession::Ev done(ServeSession::Ev::Done, sid);
      done.responded = !before_head;
      if (*unreachable && before_head) {
        if (back) {  // the session retries elsewhere or answers 502 itself
          back->err = err;
          done.unreachable = back;
          s->out_->push(std::move(done));
          return;
        }
        done.unreachable = std::make_shared<ServeSession::Unreachable>();  // health bookkeeping only
        done.unreachable->err = err;
      }
      if (!err.empty() && before_head) {
        LOG_ERROR(kT, "upstream request failed: %s", err.c_str());
        metrics::counter_add("tunnel_upstream_errors_total");
        s->simple_response(sid, 502, "Bad Gateway: " + err);
      } else {
        if (!err.empty()) {
          LOG_ERROR(kT, "upstream stream error for stream %u: %s", sid, err.c_str());
          s->emit(sid, proto::make_error(sid, "upstream error: " + err));
        }
        s->emit(sid, proto::make_empty(proto::MsgType::ResEnd, sid));
        trace::event("serve", sid, "res_end");
        LOG_DEBUG(kT, "response %u complete", sid);
      }
      s->out_->push(std::move(done));
    };
    CallState& st = calls_[sid];  // present while the call runs (on_done may fire inside request())
    st.grant = grant;
    auto call = client_->request(std::move(req), std::move(cb));
    auto it = calls_.find(sid);
    if (it != calls_.end()) {
      it->second.call = call;
    }
  }

  Reactor& r_;
  Reactor& assoc_;
  std::weak_ptr<ServeSession> sess_;
  ServeConfig cfg_;
  std::vector<std::string> upstreams_;
  bool inline_;
  bool prewarmed_ = false;
  std::unique_ptr<http::HttpClient> client_;
  std::unique_ptr<Pipe<ServeSession::Ev>> out_;
  std::unordered_map<uint32_t, CallState> calls_;
};

std::shared_ptr<ServeSession> ServeSession::start(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg,
                                                  std::function<void(const std::string&)> done, WorkerPool* pool) {
  auto s = std::shared_ptr<ServeSession>(new ServeSession(r, ch, std::move(cfg)));
  s->done_ = std::move(done);
  s->pool_ = pool;
  s->init_links(pool);
  std::weak_ptr<ServeSession> w = s;
  ch->on_message = [w](Bytes b) {
    if (auto x = w.lock()) x->on_message(std::move(b));
  };
  ch->on_message_chain = [w](Bytes b, std::vector<Bytes>& more) {
    if (auto x = w.lock()) x->on_message(std::move(b), &more);
  };
  ch->on_closed = [w](const std::string& why) {
    if (auto x = w.lock()) {
      LOG_INFO(kT, "data channel closed, serve ending");
      x->stop("data channel closed: " + why);
    }
  };
  ch->on_buffered_low = [w] {
    if (auto x = w.lock()) x->sched_->pump();
  };
  s->sched_->on_progress = [w] {
    if (auto x = w.lock()) x->check_paused();
  };
  auto gauge = [w](double (*f)(ServeSession&)) {
    return [w, f]() -> double {
      auto x = w.lock();
      return x ? f(*x) : 0.0;
    };
  };
  // Gauges read the session from the metrics thread (the first
  // association's): an extra association's session runs on another thread.
  if (s->cfg_.assoc_index == 0) {
    metrics::gauge_fn("tunnel_streams_inflight", gauge([](ServeSession& x) { return double(x.inflight_.size()); }));
    metrics::gauge_fn("tunnel_streams_paused", gauge([](ServeSession& x) { return double(x.paused_.size()); }));
    metrics::gauge_fn("tunnel_scheduler_queued_bytes",
                      gauge([](ServeSession& x) { return double(x.sched_->queued_bytes()); }));
    metrics::gauge_fn("tunnel_channel_buffered_bytes",
                      gauge([](ServeSession& x) { return double(x.ch_->buffered_amount()); }));
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

ServeSession::ServeSession(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg)
    : r_(r), ch_(std::move(ch)), cfg_(std::move(cfg)) {
  sched_ = std::make_unique<FrameScheduler>(ch_);
  for (size_t a = 0; a <= cfg_.upstream.size();) {
    size_t c = cfg_.upstream.find(',', a);
    if (c == std::string::npos) c = cfg_.upstream.size();
    if (c > a) ups_.push_back(Upstream{cfg_.upstream.substr(a, c - a)});
    a = c + 1;
  }
  if (ups_.empty()) ups_.push_back(Upstream{cfg_.upstream});
}

void ServeSession::init_links(WorkerPool* pool) {
  size_t n = 1 + (pool ? pool->size() : 0);
  place_ = std::make_unique<Placement>(n, cfg_.inline_streams);
  std::weak_ptr<ServeSession> self = shared_from_this();
  std::vector<std::string> bases;
  for (auto& u : ups_) bases.push_back(u.base);
  for (size_t k = 0; k < n; k++) {
    Reactor& wr = k == 0 ? r_ : pool->reactor(k - 1);
    auto worker = std::make_shared<ServeWorker>(wr, r_, self, cfg_, bases, k == 0);
    std::weak_ptr<ServeWorker> ww = worker;
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

// Drops the links: pending commands are discarded and each worker object is
// destroyed on its own thread (cancelling its upstream calls there).
void ServeSession::release_links() {
  auto links = std::move(links_);
  links_.clear();
  for (size_t k = 0; k < links.size(); k++) {
    links[k].to.reset();
    if (k == 0) {
      links[k].worker.reset();
    } else {
      // Moved, not copied, into the task: the last reference must drop on the
      // worker's own thread (its Pipe unhooks from that thread's reactor).
      links[k].r->post_threadsafe([w = std::move(links[k].worker)]() mutable { w.reset(); });
    }
  }
}

ServeSession::~ServeSession() {
  assoc_.reset();  // extra associations first (joins their threads)
  if (hello_timer_) r_.cancel(hello_timer_);
  if (ping_timer_) r_.cancel(ping_timer_);
  if (wd_timer_) r_.cancel(wd_timer_);
  wd_timer_ = 0;
  release_links();
  if (ch_) {
    ch_->on_message = nullptr;
    ch_->on_message_chain = nullptr;
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
  if (wd_timer_) r_.cancel(wd_timer_);
  wd_timer_ = 0;
  hello_timer_ = ping_timer_ = 0;
  assoc_.reset();
  inflight_.clear();
  paused_.clear();
  for (auto& u : ups_) u.outstanding = 0;
  streams_.clear();
  release_links();
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
    if (auto s = w.lock()) s->check_paused();
  });
}

void ServeSession::on_message(Bytes raw, std::vector<Bytes>* more) {
  if (stopped_) return;
  proto::Frame f;
  std::string err;
  std::vector<Bytes> none;
  const bool ok = proto::decode_chain(raw, more ? *more : none, f, &err);
  if (!handshaken_) {
    if (!ok) {
      stop(err);
      return;
    }
    metrics::frame_recv(uint8_t(f.type), f.wire_size());
    on_hello(f);
    return;
  }
  if (!ok) {
    LOG_WARN(kT, "failed to decode tunnel message: %s", err.c_str());
    return;
  }
  metrics::frame_recv(uint8_t(f.type), f.wire_size());
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
  const bool may_assoc = cfg_.assoc_index == 0 && cfg_.assoc > 1 && cfg_.assoc_pc;
  if (!may_assoc) ours.erase(std::remove(ours.begin(), ours.end(), "assoc"), ours.end());
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
  flow_ = std::find(agree.features.begin(), agree.features.end(), "flow") != agree.features.end();
  if (std::find(agree.features.begin(), agree.features.end(), "assoc") != agree.features.end())
    agree.assoc = assoc_agree(hello.assoc, cfg_.assoc);
  sched_->send(proto::make_agree(agree));
  if (agree.assoc > 1) start_assoc(agree.assoc);
  if (std::find(agree.features.begin(), agree.features.end(), "multistream") != agree.features.end())
    ch_->set_lanes(proto::kLanes);
  handshaken_ = true;
  LOG_INFO(kT, "sent AGREE, tunnel ready");
  if (cfg_.upstream_prewarm) command(0, Cmd{Cmd::Prewarm});
  last_pong_ms_ = Reactor::now_ms();
  send_ping();  // tokio::time::interval's first tick is immediate
  watchdog();
}

// "assoc": answers the proxy's extra PeerConnections as their offers arrive
// (ASSOC frames); each gets a serve session of its own on its own thread,
// with this session's upstreams and worker pool.
void ServeSession::start_assoc(uint32_t count) {
  ServeConfig c = cfg_;
  c.assoc = 1;
  WorkerPool* pool = pool_;
  auto factory = [c, pool](Reactor& r, std::shared_ptr<MessageChannel> ch, size_t k,
                           std::function<void(const std::string&)> done) -> std::shared_ptr<void> {
    ServeConfig ck = c;
    ck.assoc_index = k;
    return ServeSession::start(r, std::move(ch), ck, std::move(done), pool);
  };
  std::weak_ptr<ServeSession> w = shared_from_this();
  auto send = [w](proto::Frame f) {
    if (auto s = w.lock(); s && !s->stopped_) s->sched_->send(std::move(f));
  };
  LOG_INFO(kT, "associations agreed: %u", count);
  assoc_ = AssocGroup::create(r_, false, count, *cfg_.assoc_pc, cfg_.busy_poll_us, factory, send);
}

// Send-path stall watchdog: once a second, frames or channel bytes that are
// waiting without any having moved since the last tick are logged with the
// scheduler / data channel / SCTP state (and counted), so a stalled tunnel
// says why, and the scheduler is pumped once more.
void ServeSession::watchdog() {
  if (stopped_) return;
  if (sched_ && sched_->stalled_tick()) {
    if (++wd_stalled_s_ == 1) metrics::counter_add("tunnel_send_stalls_total");
    if (wd_stalled_s_ <= 3 || wd_stalled_s_ % 10 == 0)
      LOG_WARN(kT, "send path stalled for %d s: %s", wd_stalled_s_, sched_->debug_state().c_str());
    sched_->pump();  // heals a missed channel wake-up; a no-op when the transport is the one waiting
  } else {
    wd_stalled_s_ = 0;
  }
  std::weak_ptr<ServeSession> w = shared_from_this();
  wd_timer_ = r_.call_later_ms(1000, [w] {
    if (auto s = w.lock()) {
      s->wd_timer_ = 0;
      s->watchdog();
    }
  });
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
      trace::rx_stamps("serve", h.stream_id);
      uint32_t sid = h.stream_id;  // keyed by the JSON stream_id (serve.rs:118)
      Pending p;
      if (const std::string* cl = proto::header_get(h.headers, "content-length")) {
        char* end = nullptr;
        unsigned long long v = strtoull(cl->c_str(), &end, 10);
        if (end && *end == 0 && !cl->empty()) p.declared = int64_t(v);
      }
      p.headers = std::move(h);
      Pending& slot = streams_[sid] = std::move(p);
      if (cfg_.max_request_body && slot.declared > int64_t(cfg_.max_request_body)) {
        reject_too_large(sid);
        break;
      }
      // A declared body at or above the streaming threshold: the upstream call
      // starts now (connect and head while the body is still crossing) and the
      // body follows frame by frame (cut-through) instead of waiting for REQ_END.
      if (slot.declared > 0 && uint64_t(slot.declared) >= cfg_.stream_body_threshold) {
        Pending moved = std::move(slot);
        streams_.erase(sid);
        start_request(sid, std::move(moved), true);
      }
      break;
    }
    case MsgType::ReqBody: {
      const size_t n = f.payload_size();
      if (!n) break;
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end()) {
        Pending& p = it->second;
        if (flow_) grant(f.stream_id, p.owed, n);  // buffered here: bounded by the threshold
        if (p.rejected) break;
        p.body_len += n;
        p.body.push_back(f.payload);  // zero-copy: keeps the message (or its fragments) alive
        for (auto& b : f.more) p.body.push_back(b);
        if (cfg_.max_request_body && p.body_len > cfg_.max_request_body) {
          reject_too_large(f.stream_id);
          break;
        }
        // Large bodies go to the upstream as they arrive instead of piling up.
        if (p.body_len >= cfg_.stream_body_threshold) {
          Pending moved = std::move(p);
          streams_.erase(it);
          start_request(f.stream_id, std::move(moved), true);
        }
        break;
      }
      auto fl = inflight_.find(f.stream_id);
      if (fl != inflight_.end() && fl->second.uploading) {
        fl->second.uploaded += n;
        if (cfg_.max_request_body && fl->second.uploaded > cfg_.max_request_body) {
          LOG_WARN(kT, "stream %u: request body over %llu bytes, aborting", f.stream_id,
                   static_cast<unsigned long long>(cfg_.max_request_body));
          Inflight gone = fl->second;
          release_upstream(gone);
          place_->release(gone.thread);
          inflight_.erase(fl);
          paused_.erase(f.stream_id);
          command(gone.thread, Cmd{Cmd::Cancel, f.stream_id});
          sched_->send(proto::make_error(f.stream_id, "request body exceeds the tunnel's limit"));
          sched_->send(proto::make_empty(MsgType::ResEnd, f.stream_id));
          break;
        }
        Cmd c{Cmd::Body, f.stream_id};
        c.data = f.payload;
        c.more = f.more;
        command(fl->second.thread, std::move(c));
      }
      break;
    }
    case MsgType::ReqEnd: {
      auto it = streams_.find(f.stream_id);
      if (it != streams_.end()) {
        Pending p = std::move(it->second);
        streams_.erase(it);
        if (p.rejected) break;
        trace::event("serve", f.stream_id, "req_end");
        start_request(f.stream_id, std::move(p), false);
        break;
      }
      auto fl = inflight_.find(f.stream_id);
      if (fl != inflight_.end() && fl->second.uploading) {
        fl->second.uploading = false;
        trace::event("serve", f.stream_id, "req_end");
        command(fl->second.thread, Cmd{Cmd::BodyEnd, f.stream_id});
      }
      break;
    }
    case MsgType::Credit: {
      auto it = inflight_.find(f.stream_id);
      if (!flow_ || it == inflight_.end()) break;
      it->second.credit += proto::credit_bytes(f);
      if (it->second.fc && it->second.credit > 0) {
        it->second.fc = false;
        set_paused(f.stream_id, it->second);
      }
      break;
    }
    case MsgType::Cancel: {
      auto it = inflight_.find(f.stream_id);
      if (it != inflight_.end()) {
        LOG_DEBUG(kT, "stream %u cancelled by peer", f.stream_id);
        Inflight fl = it->second;
        release_upstream(fl);
        place_->release(fl.thread);
        inflight_.erase(it);
        paused_.erase(f.stream_id);
        command(fl.thread, Cmd{Cmd::Cancel, f.stream_id});
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
    case MsgType::Assoc:
      if (assoc_) assoc_->on_frame(f);
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

// Fewest requests in flight among the healthy upstreams (ties round-robin);
// when every upstream is ejected, the one whose ejection ends first (a probe).
size_t ServeSession::pick_upstream(size_t avoid) {
  size_t n = ups_.size(), best = SIZE_MAX;
  uint64_t now = Reactor::now_ms();
  for (size_t k = 0; k < n; k++) {
    size_t i = (rr_ + k) % n;
    if (i == avoid && n > 1) continue;
    if (ups_[i].down_until_ms > now) continue;
    if (best == SIZE_MAX || ups_[i].outstanding < ups_[best].outstanding) best = i;
  }
  if (best == SIZE_MAX) {
    for (size_t i = 0; i < n; i++)
      if (best == SIZE_MAX || ups_[i].down_until_ms < ups_[best].down_until_ms) best = i;
  }
  rr_ = best + 1;
  return best;
}

bool ServeSession::any_healthy(size_t except) const {
  uint64_t now = Reactor::now_ms();
  for (size_t i = 0; i < ups_.size(); i++)
    if (i != except && ups_[i].down_until_ms <= now) return true;
  return false;
}

void ServeSession::send_start(uint32_t sid, Inflight& fl, http::ClientRequest req) {
  req.url = proto::build_upstream_url(ups_[fl.up].base, cfg_.advertise, fl.path);
  Cmd c{Cmd::Start, sid};
  c.req = std::move(req);
  c.body_chunk = sched_->body_chunk();
  c.retryable = ups_.size() > 1 && fl.tries + 1u < ups_.size() && !c.req.stream_body;
  c.grant = flow_ && c.req.stream_body;
  ups_[fl.up].outstanding++;
  command(fl.thread, std::move(c));
}

// "flow": give `n` consumed body bytes back to the sender of `sid`, batched
// (kFlowGrantMin) so small uploads cost no extra frames.
void ServeSession::grant(uint32_t sid, uint64_t& owed, uint64_t n, bool force) {
  owed += n;
  if (!owed || (!force && owed < proto::kFlowGrantMin)) return;
  uint32_t g = uint32_t(std::min<uint64_t>(owed, UINT32_MAX));
  owed -= g;
  sched_->send(proto::make_credit(sid, g));
}

void ServeSession::reject_too_large(uint32_t sid) {
  auto it = streams_.find(sid);
  if (it == streams_.end() || it->second.rejected) return;
  LOG_WARN(kT, "stream %u: request body over %llu bytes, answering 413", sid,
           static_cast<unsigned long long>(cfg_.max_request_body));
  metrics::counter_add("tunnel_requests_too_large_total");
  it->second.rejected = true;
  it->second.body.clear();
  it->second.body_len = 0;
  send_simple_response(sid, 413, "Payload Too Large");
}

void ServeSession::start_request(uint32_t sid, Pending p, bool streaming) {
  if (!valid_method(p.headers.method)) {
    LOG_ERROR(kT, "failed to handle request: invalid HTTP method");
    send_simple_response(sid, 400, "Bad Request: invalid HTTP method");
    return;
  }
  if (inflight_.count(sid)) {
    LOG_WARN(kT, "stream %u reused while its response is in flight; ignoring the new request", sid);
    return;
  }
  http::ClientRequest req;
  req.method = p.headers.method;
  LOG_DEBUG(kT, "forwarding %s %s", p.headers.method.c_str(), p.headers.path.c_str());
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
  if (streaming) {  // the rest of the body arrives after the call started
    req.stream_body = true;
    req.content_length = p.declared;
  }
  metrics::counter_add("tunnel_upstream_requests_total");
  Inflight& fl = inflight_[sid];
  fl.up = pick_upstream();
  fl.route = BulkRoutes::key(req.method, p.headers.path);
  fl.thread = place_->pick(p.body_len >= Placement::kBulkBytes || p.declared >= int64_t(Placement::kBulkBytes) ||
                           bulk_routes_.bulk(fl.route));
  fl.path = std::move(p.headers.path);
  fl.uploading = streaming;
  fl.uploaded = p.body_len;
  if (flow_ && p.owed) grant(sid, p.owed, 0, true);  // what was buffered is consumed
  send_start(sid, fl, std::move(req));
}

void ServeSession::on_event(Ev& ev) {
  if (stopped_) return;
  auto it = inflight_.find(ev.sid);
  if (it == inflight_.end()) return;  // cancelled: drop its late frames
  if (ev.kind == Ev::Done) {
    Inflight& fl = it->second;
    release_upstream(fl);
    Upstream& u = ups_[fl.up];
    if (ev.unreachable) {
      u.fails++;
      uint64_t ms = std::min<uint64_t>(1000ull << std::min<uint32_t>(u.fails - 1, 5), 30000);
      u.down_until_ms = Reactor::now_ms() + ms;
      metrics::counter_add("tunnel_upstream_ejections_total");
      if (ups_.size() > 1)
        LOG_WARN(kT, "upstream %s unreachable, ejected for %llu ms: %s", u.base.c_str(),
                 static_cast<unsigned long long>(ms), ev.unreachable->err.c_str());
      // Never connected, nothing sent: try another healthy upstream.
      if (!ev.unreachable->req.method.empty() && any_healthy(fl.up)) {
        fl.tries++;
        fl.up = pick_upstream(fl.up);
        metrics::counter_add("tunnel_upstream_retries_total");
        send_start(ev.sid, fl, std::move(ev.unreachable->req));
        return;
      }
      if (!ev.unreachable->req.method.empty()) {  // handed back, but nowhere left to go
        LOG_ERROR(kT, "upstream request failed: %s", ev.unreachable->err.c_str());
        metrics::counter_add("tunnel_upstream_errors_total");
        send_simple_response(ev.sid, 502, "Bad Gateway: " + ev.unreachable->err);
      }
    } else if (ev.responded) {
      u.fails = 0;
      u.down_until_ms = 0;
      bulk_routes_.note(fl.route, fl.res_bytes, fl.res_streaming);
    }
    place_->release(fl.thread);
    inflight_.erase(it);
    paused_.erase(ev.sid);
    return;
  }
  if (ev.kind == Ev::Credit) {  // the upstream took streamed request-body bytes
    if (flow_) {
      const uint64_t grow = it->second.upwin.on_grant(ev.bytes, Reactor::now_us(), ch_ ? ch_->rtt_hint_us() : 0);
      if (grow) metrics::counter_add("tunnel_flow_window_growths_total");
      const uint64_t g = ev.bytes + grow;
      sched_->send(proto::make_credit(ev.sid, uint32_t(std::min<uint64_t>(g, UINT32_MAX))));
    }
    return;
  }
  Inflight& fl = it->second;
  bool body = ev.frame.type == proto::MsgType::ResBody;
  size_t n = ev.frame.payload.size();
  if (ev.frame.type == proto::MsgType::ResHeaders) fl.res_streaming = BulkRoutes::streaming_type(ev.frame.payload.view());
  if (body && fl.res_bytes == 0) trace::event("serve", ev.sid, "sched_in");  // first body frame reaches the scheduler
  // The start of a response goes out on the transport now, not after the
  // rest of this loop turn (Reactor::flush_soon).
  if (ev.frame.type == proto::MsgType::ResHeaders || (body && fl.res_bytes == 0)) r_.flush_soon();
  sched_->send(std::move(ev.frame));
  if (!body) return;
  fl.res_bytes += n;
  // "flow": the proxy hands credit back as its client drains; out of credit,
  // this stream's upstream read pauses (a slow client cannot grow the proxy).
  if (flow_) {
    fl.credit -= int64_t(n);
    if (fl.credit <= 0 && !fl.fc) {
      fl.fc = true;
      metrics::counter_add("tunnel_stream_credit_stalls_total");
    }
  }
  // Per-stream back-pressure: only the stream whose frames pile up stops
  // reading its upstream; a congested channel (over the global high water)
  // also pauses every stream that has a backlog, but never an interactive
  // (SSE-like) one with nothing queued.
  if (!fl.bp) {
    size_t q = sched_->stream_queued(ev.sid);
    if (q > cfg_.stream_budget || (q > FrameScheduler::kInteractive && sched_->over_high())) {
      fl.bp = true;
      paused_.insert(ev.sid);
      metrics::counter_add("tunnel_stream_pauses_total");
    }
  }
  set_paused(ev.sid, fl);
}

// Tells the call's reactor when the stream's wanted state (paused for
// back-pressure or for lack of credit) differs from what it was last told.
void ServeSession::set_paused(uint32_t sid, Inflight& fl) {
  bool want = fl.bp || fl.fc;
  if (want == fl.paused) return;
  fl.paused = want;
  command(fl.thread, Cmd{want ? Cmd::Pause : Cmd::Resume, sid});
}

void ServeSession::check_paused() {
  if (paused_.empty() || stopped_ || sched_->over_high()) return;
  for (auto p = paused_.begin(); p != paused_.end();) {
    uint32_t sid = *p;
    auto it = inflight_.find(sid);
    if (it == inflight_.end()) {
      p = paused_.erase(p);
      continue;
    }
    if (sched_->stream_queued(sid) <= cfg_.stream_budget / 4) {
      it->second.bp = false;
      p = paused_.erase(p);
      set_paused(sid, it->second);
      continue;
    }
    ++p;
  }
}

}  // namespace p2pt
