#include "http/client.h"

#include "core/log.h"

#include <deque>

namespace p2pt::http {

// Keep-alive pool plus "warm" connections: fresh, already-established
// sockets to the upstream origin opened ahead of demand. HTTP/1.0 upstreams
// (the reference's mock, many simple servers) close after every response, so
// keep-alive never helps them; a warm socket takes the TCP (and TLS)
// handshake off every request's time-to-first-token. The warm target follows
// the recent peak of concurrent requests (>= the configured minimum) and is
// topped up only when requests arrive. An unused warm socket is closed after
// an idle TTL: a single-threaded upstream serves one connection at a time and
// would otherwise sit blocked on our idle socket, starving its other clients.
using WarmWaiter = std::function<bool(std::shared_ptr<TcpConn>, const std::string&)>;

class ClientConnPool : public std::enable_shared_from_this<ClientConnPool> {
 public:
  explicit ClientConnPool(Reactor& r) : r_(r) {}
  std::shared_ptr<TcpConn> take(const std::string& key) {
    auto it = idle_.find(key);
    while (it != idle_.end() && !it->second.empty()) {
      auto c = it->second.back();
      it->second.pop_back();
      if (!c->closed()) return c;
    }
    return nullptr;
  }

  struct Warm {
    std::string host;
    uint16_t port = 0;
    bool tls = false;
    size_t min = 0, max = 512;  // warm-socket cap: follows peaks of up to 512 concurrent requests
    size_t peak = 0;          // recent peak of in-flight requests
    uint64_t peak_at_ms = 0;
    size_t inflight = 0;
    size_t connecting = 0;
    int failures = 0;
    uint64_t retry_timer = 0;
    uint64_t ttl_ms = 1000;
    uint64_t expiry_timer = 0;
    uint64_t topup_timer = 0;
    std::vector<std::shared_ptr<TcpConn>> ready;
    std::vector<uint64_t> ready_at;  // parallel to ready
    std::deque<WarmWaiter> waiters;  // calls waiting for the next warm socket
  };

  void configure_warm(const std::string& key, const std::string& host, uint16_t port, bool tls, size_t min,
                      uint64_t ttl_ms) {
    Warm& w = warm_[key];
    w.host = host;
    w.port = port;
    w.tls = tls;
    w.min = min;
    w.ttl_ms = ttl_ms ? ttl_ms : 1;
    replenish(key);
  }

  void erase_ready(Warm& w, size_t i) {
    w.ready.erase(w.ready.begin() + long(i));
    w.ready_at.erase(w.ready_at.begin() + long(i));
  }

  // Close warm sockets idle for longer than the TTL (oldest first; ready is in
  // connect order, so expired ones sit at the front).
  void schedule_expiry(const std::string& key) {
    auto it = warm_.find(key);
    if (it == warm_.end()) return;
    Warm& w = it->second;
    if (w.expiry_timer || w.ready.empty()) return;
    uint64_t now = Reactor::now_ms();
    uint64_t due = w.ready_at.front() + w.ttl_ms;
    std::weak_ptr<ClientConnPool> self = shared_from_this();
    w.expiry_timer = r_.call_later_ms(due > now ? due - now : 0, [self, key] {
      auto p = self.lock();
      if (!p) return;
      auto it2 = p->warm_.find(key);
      if (it2 == p->warm_.end()) return;
      Warm& w2 = it2->second;
      w2.expiry_timer = 0;
      uint64_t t = Reactor::now_ms();
      while (!w2.ready.empty() && w2.ready_at.front() + w2.ttl_ms <= t) {
        auto c = w2.ready.front();
        p->erase_ready(w2, 0);
        c->on_data(nullptr);
        c->on_close(nullptr);
        c->close();
      }
      p->schedule_expiry(key);
    });
  }
  bool has_warm(const std::string& key) const { return warm_.count(key) != 0; }

  // With no warm socket ready, a call queues for the next one to finish
  // connecting instead of opening its own: every upstream connection then
  // comes from one FIFO, so use order follows connect (= accept) order even
  // for a single-threaded upstream. False while backing off after connect
  // failures (the caller connects directly and reports its own error).
  bool wait_warm(const std::string& key, WarmWaiter fn) {
    auto it = warm_.find(key);
    if (it == warm_.end() || it->second.retry_timer) return false;
    it->second.waiters.push_back(std::move(fn));
    replenish(key);
    return true;
  }

  std::shared_ptr<TcpConn> take_warm(const std::string& key) {
    auto it = warm_.find(key);
    if (it == warm_.end()) return nullptr;
    // Oldest first: a single-threaded upstream (the reference's own mock)
    // accepts connections in connect order and blocks reading the first one,
    // so handing out a newer warm socket would wait behind an idle one forever.
    Warm& w = it->second;
    std::shared_ptr<TcpConn> c;
    while (!w.ready.empty()) {
      c = w.ready.front();
      erase_ready(w, 0);
      if (!c->closed()) break;
      c.reset();
    }
    if (c) {
      c->on_data(nullptr);
      c->on_close(nullptr);
    }
    return c;
  }

  void call_started(const std::string& key) {
    auto it = warm_.find(key);
    if (it == warm_.end()) return;
    Warm& w = it->second;
    w.inflight++;
    uint64_t now = Reactor::now_ms();
    if (w.inflight >= w.peak || now - w.peak_at_ms > 30000) {
      w.peak = w.inflight;
      w.peak_at_ms = now;
    }
    schedule_topup(key, w);
  }
  void call_finished(const std::string& key) {
    auto it = warm_.find(key);
    if (it == warm_.end()) return;
    if (it->second.inflight) it->second.inflight--;
    // Refill toward the recent peak between bursts, so the next burst of
    // requests finds connected sockets instead of queueing for connects.
    schedule_topup(key, it->second);
  }
  // Top up a little later, not inside the burst that is taking the sockets:
  // connect() calls would sit on the critical path of the requests still being
  // parsed in this and the next reactor iterations.
  void schedule_topup(const std::string& key, Warm& w) {
    if (w.topup_timer) return;
    std::weak_ptr<ClientConnPool> self = shared_from_this();
    w.topup_timer = r_.call_later_ms(2, [self, key] {
      auto p = self.lock();
      if (!p) return;
      auto it2 = p->warm_.find(key);
      if (it2 == p->warm_.end()) return;
      it2->second.topup_timer = 0;
      p->replenish(key);
    });
  }

  void replenish(const std::string& key) {
    auto it = warm_.find(key);
    if (it == warm_.end()) return;
    Warm& w = it->second;
    if (w.retry_timer) return;  // backing off after connect failures
    size_t target = std::min(w.max, std::max(w.min, w.peak)) + w.waiters.size();
    std::weak_ptr<ClientConnPool> self = shared_from_this();
    while (w.ready.size() + w.connecting < target) {
      w.connecting++;
      TcpConn::connect(r_, w.host, w.port, w.tls, [self, key](std::shared_ptr<TcpConn> c, std::string err) {
        auto p = self.lock();
        if (!p) {
          if (c) c->close();
          return;
        }
        auto it2 = p->warm_.find(key);
        if (it2 == p->warm_.end()) {
          if (c) c->close();
          return;
        }
        Warm& w2 = it2->second;
        w2.connecting--;
        if (!c) {
          // Upstream down: fail the waiting calls (each becomes a 502) and back off.
          auto waiters = std::move(w2.waiters);
          w2.waiters.clear();
          for (auto& fn : waiters) fn(nullptr, err);
          it2 = p->warm_.find(key);
          if (it2 == p->warm_.end()) return;
          Warm& w3 = it2->second;
          if (w3.retry_timer) return;
          w3.failures++;
          uint64_t delay = std::min<uint64_t>(100ull << std::min(w3.failures, 6), 5000);
          w3.retry_timer = p->r_.call_later_ms(delay, [self, key] {
            auto p2 = self.lock();
            if (!p2) return;
            auto it3 = p2->warm_.find(key);
            if (it3 == p2->warm_.end()) return;
            it3->second.retry_timer = 0;
            p2->replenish(key);
          });
          return;
        }
        w2.failures = 0;
        while (!w2.waiters.empty()) {
          WarmWaiter fn = std::move(w2.waiters.front());
          w2.waiters.pop_front();
          if (fn(c, "")) return;  // the call took it; a declined one (cancelled) tries the next
        }
        std::weak_ptr<TcpConn> wc = c;
        // A warm socket that turns readable/closed was dropped by the server
        // (its idle timeout): discard it; the next request tops the pool up.
        auto drop = [self, key, wc] {
          auto p2 = self.lock();
          auto conn = wc.lock();
          if (!p2 || !conn) return;
          auto it3 = p2->warm_.find(key);
          if (it3 == p2->warm_.end()) return;
          auto& v = it3->second.ready;
          for (size_t i = 0; i < v.size(); i++)
            if (v[i] == conn) {
              p2->erase_ready(it3->second, i);
              break;
            }
          conn->on_close(nullptr);
          conn->close();
        };
        c->on_data([drop](const uint8_t*, size_t) { drop(); });
        c->on_close([drop](const std::string&) { drop(); });
        w2.ready.push_back(std::move(c));
        w2.ready_at.push_back(Reactor::now_ms());
        p->schedule_expiry(key);
      });
    }
  }
  void put(const std::string& key, std::shared_ptr<TcpConn> c) {
    if (c->closed()) return;
    auto& v = idle_[key];
    if (v.size() >= 64) {
      c->close();
      return;
    }
    std::weak_ptr<TcpConn> w = c;
    // An idle connection that becomes readable is either closing or broken.
    c->on_data([w](const uint8_t*, size_t) {
      if (auto s = w.lock()) s->close("unexpected data on idle connection");
    });
    std::weak_ptr<ClientConnPool> wp;  // pool outlives conns via HttpClient
    c->on_close([this, key, w](const std::string&) { remove(key, w); });
    v.push_back(std::move(c));
  }
  void remove(const std::string& key, const std::weak_ptr<TcpConn>& w) {
    auto it = idle_.find(key);
    if (it == idle_.end()) return;
    auto s = w.lock();
    auto& v = it->second;
    for (size_t i = 0; i < v.size(); i++)
      if (v[i] == s) {
        v.erase(v.begin() + long(i));
        break;
      }
  }
  size_t idle() const {
    size_t n = 0;
    for (auto& kv : idle_) n += kv.second.size();
    return n;
  }
  void clear() {
    auto all = std::move(idle_);
    idle_.clear();
    for (auto& kv : all)
      for (auto& c : kv.second) {
        c->on_close(nullptr);
        c->close();
      }
    auto warm = std::move(warm_);
    warm_.clear();
    for (auto& kv : warm) {
      if (kv.second.retry_timer) r_.cancel(kv.second.retry_timer);
      if (kv.second.expiry_timer) r_.cancel(kv.second.expiry_timer);
      if (kv.second.topup_timer) r_.cancel(kv.second.topup_timer);
      if (!kv.second.waiters.empty())
        r_.post([ws = std::move(kv.second.waiters)]() mutable {
          for (auto& fn : ws) fn(nullptr, "client shut down");
        });
      for (auto& c : kv.second.ready) {
        c->on_close(nullptr);
        c->close();
      }
    }
  }
  size_t warm_ready(const std::string& key) const {
    auto it = warm_.find(key);
    return it == warm_.end() ? 0 : it->second.ready.size();
  }
  Reactor& r_;

 private:
  std::map<std::string, std::vector<std::shared_ptr<TcpConn>>> idle_;
  std::map<std::string, Warm> warm_;
};

HttpClient::HttpClient(Reactor& r) : r_(r), pool_(std::make_shared<ClientConnPool>(r)) {}
HttpClient::~HttpClient() { pool_->clear(); }
size_t HttpClient::idle_connections() const { return pool_->idle(); }

bool HttpClient::prewarm(const std::string& url, size_t min_ready, uint64_t idle_ttl_ms, std::string* err) {
  Url u;
  if (!parse_url(url, u, err)) return false;
  if (u.scheme != "http" && u.scheme != "https") {
    if (err) *err = "unsupported scheme";
    return false;
  }
  pool_->configure_warm(u.scheme + "://" + u.host + ":" + std::to_string(u.port), u.host, u.port, u.tls(), min_ready,
                        idle_ttl_ms);
  return true;
}

size_t HttpClient::warm_connections(const std::string& url) const {
  Url u;
  if (!parse_url(url, u, nullptr)) return 0;
  return pool_->warm_ready(u.scheme + "://" + u.host + ":" + std::to_string(u.port));
}

std::shared_ptr<ClientCall> HttpClient::request(ClientRequest req, ClientCallbacks cb) {
  auto call = std::shared_ptr<ClientCall>(new ClientCall());
  call->r_ = &r_;
  call->pool_ = pool_;
  call->req_ = std::move(req);
  call->cb_ = std::move(cb);
  call->start();
  return call;
}

ClientCall::~ClientCall() {
  if (conn_) {
    conn_->on_close(nullptr);
    conn_->close();
  }
}

namespace {
// Calls keep themselves alive until finished (fire-and-forget semantics like tokio::spawn).
std::map<ClientCall*, std::shared_ptr<ClientCall>>& live_calls() {
  thread_local std::map<ClientCall*, std::shared_ptr<ClientCall>> m;  // per reactor thread
  return m;
}
}  // namespace

void ClientCall::start() {
  std::string err;
  if (!parse_url(req_.url, url_, &err) || (url_.scheme != "http" && url_.scheme != "https")) {
    if (err.empty()) err = "unsupported scheme: " + url_.scheme;
    auto self = shared_from_this();
    live_calls()[this] = self;
    r_->post([self, err] { self->finish("builder error for url (" + self->req_.url + "): " + err); });
    return;
  }
  live_calls()[this] = shared_from_this();
  pool_key_ = url_.scheme + "://" + url_.host + ":" + std::to_string(url_.port);
  pool_->call_started(pool_key_);
  counted_ = true;
  chunked_body_ = req_.stream_body && req_.content_length < 0;
  if (req_.stream_body) {
    for (auto& b : req_.body) queued_body_ += b.size();
    std::weak_ptr<ClientCall> w = shared_from_this();
    TcpConn::connect(*r_, url_.host, url_.port, url_.tls(), [w](std::shared_ptr<TcpConn> c, std::string e) {
      auto self = w.lock();
      if (!self || self->finished_) {
        if (c) c->close();
        return;
      }
      if (!c) {
        if (self->cb_.on_connect_failed) self->cb_.on_connect_failed();
        self->finish("error sending request for url (" + self->req_.url + "): " + e);
        return;
      }
      self->attach(c, false);
    });
    return;
  }
  if (auto c = pool_->take(pool_key_)) {
    attach(c, true);
    return;
  }
  // A warm socket may have been closed by the server an instant ago; it is
  // treated like a reused keep-alive socket (one transparent retry).
  if (auto c = pool_->take_warm(pool_key_)) {
    attach(c, true);
    return;
  }
  std::weak_ptr<ClientCall> w = shared_from_this();
  auto deliver = [w](std::shared_ptr<TcpConn> c, const std::string& e) -> bool {
    auto self = w.lock();
    if (!self || self->finished_) return false;
    if (!c) {
      if (self->cb_.on_connect_failed) self->cb_.on_connect_failed();
      self->finish("error sending request for url (" + self->req_.url + "): " + e);
      return true;
    }
    self->attach(c, false);
    return true;
  };
  if (pool_->wait_warm(pool_key_, deliver)) return;
  TcpConn::connect(*r_, url_.host, url_.port, url_.tls(), [deliver](std::shared_ptr<TcpConn> c, std::string e) {
    if (!deliver(c, e) && c) c->close();
  });
}

void ClientCall::attach(std::shared_ptr<TcpConn> c, bool reused) {
  conn_ = std::move(c);
  reused_ = reused;
  std::weak_ptr<ClientCall> w = shared_from_this();
  conn_->on_data([w](const uint8_t* p, size_t n) {
    if (auto s = w.lock()) s->on_data(p, n);
  });
  conn_->on_close([w](const std::string& err) {
    if (auto s = w.lock()) s->on_close(err);
  });
  std::string head;
  head.reserve(256);
  head += req_.method;
  head += ' ';
  head += url_.path;
  head += " HTTP/1.1\r\nhost: ";
  head += url_.host_header();
  head += "\r\n";
  bool has_accept = false;
  for (auto& h : req_.headers) {
    if (iequals(h.name, "accept")) has_accept = true;
    head += h.name;
    head += ": ";
    head += h.value;
    head += "\r\n";
  }
  if (!has_accept) head += "accept: */*\r\n";
  if (req_.stream_body) {
    if (chunked_body_) head += "transfer-encoding: chunked\r\n";
    else head += "content-length: " + std::to_string(req_.content_length) + "\r\n";
    head += "\r\n";
    conn_->write(std::move(head));
    std::weak_ptr<ClientCall> wd = shared_from_this();
    conn_->on_drain(
        [wd] {
          auto s = wd.lock();
          if (s && !s->finished_ && s->cb_.on_body_drain) s->cb_.on_body_drain();
        },
        cb_.body_low_water);
    auto pieces = std::move(req_.body);
    req_.body.clear();
    queued_body_ = 0;
    for (auto& b : pieces) write_piece(b);
    if (body_ended_ && chunked_body_) conn_->write(std::string("0\r\n\r\n"));
    if (paused_) conn_->pause_reading();
    if (cb_.on_sent) cb_.on_sent(reused);
    if (cb_.on_body_drain && conn_->pending_out() <= cb_.body_low_water) cb_.on_body_drain();
    return;
  }
  if (req_.body_len > 0 || req_.force_content_length) head += "content-length: " + std::to_string(req_.body_len) + "\r\n";
  head += "\r\n";
  // Small bodies ride in the same segment as the head.
  if (req_.body_len <= 16384) {
    for (auto& b : req_.body) head.append(reinterpret_cast<const char*>(b.data()), b.size());
    conn_->write(std::move(head));
  } else {
    conn_->write(std::move(head));
    for (auto& b : req_.body) conn_->write(b);
  }
  if (paused_) conn_->pause_reading();
  if (cb_.on_sent) cb_.on_sent(reused);
}

void ClientCall::on_data(const uint8_t* p, size_t n) {
  got_any_ = true;
  if (head_done_ && buf_.empty() && !finished_ && !paused_ && !body_.done()) {
    // Body bytes straight from the socket buffer (no staging copy).
    auto self = shared_from_this();
    size_t used = body_.feed(p, n, [this](const uint8_t* d, size_t k) {
      if (cb_.on_data && !finished_) cb_.on_data(conn_ ? conn_->rx_view(d, k) : Bytes::copy(d, k));
    });
    if (used == SIZE_MAX) {
      finish("error decoding response body: " + body_.error());
      return;
    }
    if (finished_) return;
    if (used < n) buf_.append(reinterpret_cast<const char*>(p + used), n - used);
    if (body_.done() && buf_.empty()) {
      finish("");
      return;
    }
    process();
    return;
  }
  buf_.append(reinterpret_cast<const char*>(p), n);
  process();
}

void ClientCall::process() {
  auto self = shared_from_this();
  while (!finished_ && !paused_) {
    if (!head_done_) {
      size_t used = 0;
      std::string err;
      Head h;
      auto res = parse_response_head(buf_, h, used, &err);
      if (res == ParseResult::Incomplete) return;
      if (res == ParseResult::Error) {
        finish("error sending request for url (" + req_.url + "): invalid HTTP response: " + err);
        return;
      }
      buf_.erase(0, used);
      if (h.status >= 100 && h.status < 200 && h.status != 101) continue;  // interim
      head_ = std::move(h);
      head_done_ = true;
      uint64_t len = 0;
      auto mode = response_body_mode(head_, req_.method, len);
      body_.reset(mode, len);
      bool close_tok = head_.has_token("connection", "close");
      keep_alive_ = mode != BodyDecoder::Mode::UntilClose &&
                    (head_.version_minor >= 1 ? !close_tok : head_.has_token("connection", "keep-alive"));
      if (cb_.on_head) cb_.on_head(head_);
      if (finished_ || paused_) return;
    }
    if (body_.done()) {
      finish("");
      return;
    }
    if (buf_.empty()) return;
    size_t used = body_.feed(reinterpret_cast<const uint8_t*>(buf_.data()), buf_.size(),
                             [this](const uint8_t* d, size_t k) {
                               if (cb_.on_data && !finished_) cb_.on_data(Bytes::copy(d, k));
                             });
    if (used == SIZE_MAX) {
      finish("error decoding response body: " + body_.error());
      return;
    }
    buf_.erase(0, used);
    if (body_.done()) {
      if (!buf_.empty()) keep_alive_ = false;  // trailing garbage
      finish("");
      return;
    }
    if (used == 0) return;
  }
}

void ClientCall::on_close(const std::string& err) {
  auto self = shared_from_this();
  conn_.reset();
  if (finished_) return;
  if (!got_any_ && reused_) {
    // Stale pooled connection: retry once on a fresh one.
    reused_ = false;
    std::weak_ptr<ClientCall> w = self;
    TcpConn::connect(*r_, url_.host, url_.port, url_.tls(), [w](std::shared_ptr<TcpConn> c, std::string e) {
      auto s = w.lock();
      if (!s || s->finished_) {
        if (c) c->close();
        return;
      }
      if (!c) {
        if (s->cb_.on_connect_failed) s->cb_.on_connect_failed();
        s->finish("error sending request for url (" + s->req_.url + "): " + e);
        return;
      }
      s->attach(c, false);
    });
    return;
  }
  keep_alive_ = false;
  if (!head_done_) {
    // The peer may have sent a complete head without body framing then closed.
    process();
    if (finished_) return;
    finish("error sending request for url (" + req_.url + "): " +
           (err.empty() ? std::string("connection closed before message completed") : err));
    return;
  }
  // Deliver anything buffered (paused) before judging EOF.
  paused_ = false;
  process();
  if (finished_) return;
  if (body_.on_eof()) finish("");
  else finish("error decoding response body: " + (err.empty() ? body_.error() : err));
}

void ClientCall::finish(const std::string& err) {
  if (finished_) return;
  finished_ = true;
  auto self = shared_from_this();
  if (counted_) {
    counted_ = false;
    pool_->call_finished(pool_key_);
  }
  if (conn_) {
    auto c = std::move(conn_);
    conn_.reset();
    if (err.empty() && keep_alive_ && buf_.empty() && !c->closed()) {
      c->resume_reading();
      pool_->put(pool_key_, c);
    } else {
      c->on_close(nullptr);
      c->close();
    }
  }
  bool before_head = !head_done_;
  auto cb = std::move(cb_.on_done);
  cb_ = ClientCallbacks{};
  if (cb) cb(err, before_head);
  live_calls().erase(this);
}

void ClientCall::write_piece(const Bytes& b) {
  if (b.empty() || !conn_) return;
  if (chunked_body_) {
    char h[24];
    int n = snprintf(h, sizeof h, "%zx\r\n", b.size());
    conn_->write(slab_copy(h, size_t(n)));
    conn_->write(b);
    conn_->write(slab_copy("\r\n", 2));
  } else {
    conn_->write(b);
  }
}

void ClientCall::write_body(Bytes b) {
  if (finished_ || body_ended_ || b.empty()) return;
  if (!conn_) {  // still connecting: queued, written right after the head
    queued_body_ += b.size();
    req_.body.push_back(std::move(b));
    return;
  }
  write_piece(b);
}

void ClientCall::end_body() {
  if (finished_ || body_ended_) return;
  body_ended_ = true;
  if (conn_ && chunked_body_) conn_->write(std::string("0\r\n\r\n"));
}

size_t ClientCall::body_backlog() const { return conn_ ? conn_->pending_out() : size_t(queued_body_); }

void ClientCall::pause() {
  if (paused_ || finished_) return;
  paused_ = true;
  if (conn_) conn_->pause_reading();
}

void ClientCall::resume() {
  if (!paused_ || finished_) return;
  paused_ = false;
  if (conn_) conn_->resume_reading();
  std::weak_ptr<ClientCall> w = shared_from_this();
  r_->post([w] {
    if (auto s = w.lock()) {
      if (!s->buf_.empty()) s->process();
    }
  });
}

void ClientCall::cancel() {
  if (finished_) return;
  keep_alive_ = false;
  auto cb = std::move(cb_.on_done);
  cb_ = ClientCallbacks{};
  finish("cancelled");
  (void)cb;
}

}  // namespace p2pt::http
