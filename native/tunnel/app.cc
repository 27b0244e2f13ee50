#include "tunnel/app.h"

#include <signal.h>
#include <unistd.h>

#include "core/log.h"
#include "core/net.h"
#include "tunnel/metrics.h"
#include "tunnel/session.h"

namespace p2pt {

static const char* kT = "tunnel";

uint64_t backoff_secs(uint64_t attempt) {
  const uint64_t initial = 2, cap = 60;
  uint64_t e = attempt < 10 ? attempt : 10;
  if (e == 0) e = 1;
  uint64_t b = initial << (e - 1);
  return b < cap ? b : cap;
}

namespace {

// --transport tcp-listen:ADDR / tcp-connect:ADDR (debug + benchmark link).
struct TcpLink {
  std::unique_ptr<TcpListener> listener;
  std::shared_ptr<TcpMessageChannel> ch;
  uint64_t retry_timer = 0;
  Reactor* r = nullptr;
  bool done = false;
  std::shared_ptr<std::function<void()>> attempt;  // tcp-connect retry loop (owned here, weakly self-referenced)
  ~TcpLink() {
    if (retry_timer && r) r->cancel(retry_timer);
    if (ch) ch->close();
  }
};

std::shared_ptr<void> connect_tcp(Reactor& r, const std::string& spec, ConnectCb cb) {
  auto link = std::make_shared<TcpLink>();
  link->r = &r;
  std::weak_ptr<TcpLink> w = link;
  auto deliver = std::make_shared<ConnectCb>(std::move(cb));
  if (spec.rfind("tcp-listen:", 0) == 0) {
    std::string addr = spec.substr(11);
    std::string err;
    Reactor* rp = &r;
    link->listener = TcpListener::bind(
        r, addr,
        [w, rp, deliver](int fd, SockAddr peer) {
          auto l = w.lock();
          if (!l || l->done) {
            ::close(fd);
            return;
          }
          l->done = true;
          LOG_INFO("tunnel::transport", "tcp transport: accepted peer %s", peer.str().c_str());
          l->ch = TcpMessageChannel::wrap(TcpConn::adopt(*rp, fd));
          // One peer per session, like a WebRTC room of two.
          rp->post([w] {
            if (auto l2 = w.lock()) l2->listener.reset();
          });
          (*deliver)(l->ch, "");
        },
        &err);
    if (!link->listener) {
      r.post([deliver, err] { (*deliver)(nullptr, err); });
      return link;
    }
    LOG_INFO("tunnel::transport", "tcp transport: listening on %s", link->listener->local_addr().str().c_str());
    return link;
  }
  if (spec.rfind("tcp-connect:", 0) == 0) {
    std::string addr = spec.substr(12);
    size_t colon = addr.rfind(':');
    std::string host = colon == std::string::npos ? addr : addr.substr(0, colon);
    uint16_t port = colon == std::string::npos ? 0 : uint16_t(atoi(addr.c_str() + colon + 1));
    if (host.size() > 1 && host.front() == '[') host = host.substr(1, host.size() - 2);
    auto deadline = Reactor::now_ms() + 30000;
    auto attempt = std::make_shared<std::function<void()>>();
    link->attempt = attempt;
    std::weak_ptr<std::function<void()>> wa = attempt;
    Reactor* rp = &r;
    *attempt = [w, rp, host, port, deliver, deadline, wa] {
      TcpConn::connect(*rp, host, port, false, [w, rp, deliver, deadline, wa](std::shared_ptr<TcpConn> c, std::string e) {
        auto l = w.lock();
        if (!l || l->done) return;
        if (!c) {
          if (Reactor::now_ms() < deadline) {
            l->retry_timer = rp->call_later_ms(100, [w, wa] {
              auto l2 = w.lock();
              auto a = wa.lock();
              if (l2 && a) {
                l2->retry_timer = 0;
                (*a)();
              }
            });
            return;
          }
          l->done = true;
          (*deliver)(nullptr, "tcp transport: " + e);
          return;
        }
        l->done = true;
        l->ch = TcpMessageChannel::wrap(c);
        LOG_INFO("tunnel::transport", "tcp transport: connected to %s", c->peer().str().c_str());
        (*deliver)(l->ch, "");
      });
    };
    (*attempt)();
    return link;
  }
  r.post([deliver, spec] { (*deliver)(nullptr, "unknown transport: " + spec); });
  return link;
}

// --listen-early: bound before the first handshake, survives reconnects, and
// answers 503 "Tunnel not ready" while no session is ready (Q8 option).
struct EarlyListener {
  std::unique_ptr<TcpListener> listener;
  std::weak_ptr<ProxySession> session;
};

void reply_not_ready(Reactor& r, int fd) {
  auto c = TcpConn::adopt(r, fd);
  auto buf = std::make_shared<std::string>();
  std::weak_ptr<TcpConn> w = c;
  auto hold = std::make_shared<std::shared_ptr<TcpConn>>(c);
  c->on_data([w, buf](const uint8_t* p, size_t n) {
    buf->append(reinterpret_cast<const char*>(p), n);
    if (buf->find("\r\n\r\n") == std::string::npos && buf->size() < 65536) return;
    if (auto s = w.lock()) {
      s->write(std::string(
          "HTTP/1.1 503 Service Unavailable\r\ncontent-type: text/plain\r\ncontent-length: 16\r\n"
          "connection: close\r\n\r\nTunnel not ready"));
      s->close_after_flush();
    }
  });
  c->on_close([hold](const std::string&) { hold->reset(); });
}

}  // namespace

std::shared_ptr<void> connect_transport(Reactor& r, const AppConfig& cfg, ConnectCb cb) {
  if (cfg.transport == "webrtc" || cfg.transport.empty()) return connect_webrtc(r, cfg, std::move(cb));
  return connect_tcp(r, cfg.transport, std::move(cb));
}

int run_app(const AppConfig& cfg) {
  Reactor r;
  r.set_busy_poll_us(cfg.busy_poll_us);
  // Worker threads for per-stream HTTP work (tunnel/workers.h); they outlive
  // sessions, so reconnects reuse them.
  WorkerPool pool(cfg.workers, cfg.busy_poll_us);
  if (pool.size()) LOG_INFO(kT, "%zu worker threads (streams beyond %zu per session spill onto them)", pool.size(),
                            cfg.inline_streams);
  struct State {
    uint64_t attempt = 0;
    std::shared_ptr<void> transport;
    std::shared_ptr<ServeSession> serve;
    std::shared_ptr<ProxySession> proxy;
    uint64_t backoff_timer = 0;
    uint64_t session_start_ms = 0;
    int exit_code = 0;
    bool interrupted = false;  // Ctrl-C / SIGTERM, as opposed to giving up after --max-retries
    bool in_attempt = false;
    EarlyListener early;
  } st;
  std::shared_ptr<void> metrics_srv;
  if (!cfg.metrics_listen.empty()) {
    std::string err;
    metrics_srv = metrics::serve(r, cfg.metrics_listen, &err);
    if (!metrics_srv) LOG_WARN(kT, "metrics endpoint disabled: %s", err.c_str());
    else LOG_INFO(kT, "metrics on http://%s/metrics", cfg.metrics_listen.c_str());
  }
  if (cfg.mode == "proxy" && cfg.listen_early) {
    std::string err;
    Reactor* rp = &r;
    st.early.listener = TcpListener::bind(
        r, cfg.listen,
        [&st, rp](int fd, SockAddr) {
          auto s = st.early.session.lock();
          if (s && s->ready()) s->accept(fd);
          else reply_not_ready(*rp, fd);
        },
        &err);
    if (!st.early.listener) {
      LOG_ERROR(kT, "%s", err.c_str());
      return 1;
    }
    LOG_INFO("tunnel::proxy", "proxy listening on http://%s (early; 503 until the tunnel is ready)",
             st.early.listener->local_addr().str().c_str());
  }

  std::function<void()> start_attempt;
  std::function<void(const std::string&)> on_fail;

  on_fail = [&](const std::string& err) {
    if (!st.in_attempt) return;
    st.in_attempt = false;
    // Tear down on the next iteration: we may be inside a callback of the
    // objects being destroyed.
    auto t = std::move(st.transport);
    auto s1 = std::move(st.serve);
    auto s2 = std::move(st.proxy);
    r.post([t, s1, s2] {});
    if (cfg.reset_backoff_after_s && st.session_start_ms &&
        Reactor::now_ms() - st.session_start_ms >= cfg.reset_backoff_after_s * 1000)
      st.attempt = 0;
    st.session_start_ms = 0;
    st.attempt++;
    if (st.attempt > cfg.max_retries) {
      LOG_ERROR(kT, "%s failed after %llu attempts, giving up: %s", cfg.mode.c_str(),
                static_cast<unsigned long long>(cfg.max_retries), err.c_str());
      st.exit_code = 1;
      r.stop();
      return;
    }
    uint64_t b = backoff_secs(st.attempt);
    LOG_WARN(kT, "%s failed (attempt %llu): %s. Retrying in %llus...", cfg.mode.c_str(),
             static_cast<unsigned long long>(st.attempt), err.c_str(), static_cast<unsigned long long>(b));
    st.backoff_timer = r.call_later_ms(b * 1000, [&] {
      st.backoff_timer = 0;
      start_attempt();
    });
  };

  start_attempt = [&] {
    st.in_attempt = true;
    st.transport = connect_transport(r, cfg, [&](std::shared_ptr<MessageChannel> ch, std::string err) {
      if (!st.in_attempt) return;
      if (!ch) {
        on_fail(err);
        return;
      }
      st.session_start_ms = Reactor::now_ms();
      // Extra associations ("assoc") are WebRTC connections like the first.
      std::shared_ptr<const rtc::PcConfig> assoc_pc;
      if (cfg.assoc > 1 && (cfg.transport == "webrtc" || cfg.transport.empty()))
        assoc_pc = std::make_shared<rtc::PcConfig>(make_pc_config(cfg));
      if (cfg.mode == "serve") {
        LOG_INFO(kT, "WebRTC connected, starting serve...");
        ServeConfig sc;
        sc.upstream = cfg.upstream;
        sc.advertise = cfg.advertise;
        sc.handshake_timeout_ms = cfg.handshake_timeout_ms;
        sc.ping_interval_ms = cfg.ping_interval_ms;
        sc.pong_timeout_ms = cfg.pong_timeout_ms;
        sc.upstream_prewarm = cfg.upstream_prewarm;
        sc.upstream_prewarm_ttl_ms = cfg.upstream_prewarm_ttl_ms;
        sc.secret = cfg.secret;
        sc.inline_streams = cfg.inline_streams;
        sc.max_request_body = cfg.max_request_body;
        sc.stream_body_threshold = cfg.stream_body_threshold ? cfg.stream_body_threshold : UINT64_MAX;
        sc.assoc = cfg.assoc;
        sc.assoc_pc = assoc_pc;
        sc.busy_poll_us = cfg.busy_poll_us;
        st.serve = ServeSession::start(r, ch, sc, [&](const std::string& e) { on_fail(e); }, &pool);
      } else {
        LOG_INFO(kT, "WebRTC connected, starting proxy...");
        ProxyConfig pc;
        pc.listen = cfg.listen;
        pc.handshake_timeout_ms = cfg.handshake_timeout_ms;
        pc.header_timeout_ms = cfg.header_timeout_ms;
        pc.ping_interval_ms = cfg.ping_interval_ms;
        pc.pong_timeout_ms = cfg.pong_timeout_ms;
        pc.listen_early = cfg.listen_early;
        pc.secret = cfg.secret;
        pc.inline_streams = cfg.inline_streams;
        pc.assoc = cfg.assoc;
        pc.assoc_pc = assoc_pc;
        pc.busy_poll_us = cfg.busy_poll_us;
        st.proxy = ProxySession::start(r, ch, pc, [&](const std::string& e) { on_fail(e); }, &pool);
        st.early.session = st.proxy;
      }
    });
  };

  auto interrupt = [&] {
    if (st.backoff_timer) {
      LOG_INFO(kT, "received Ctrl+C during retry backoff, exiting");
      r.cancel(st.backoff_timer);
      st.backoff_timer = 0;
    } else {
      LOG_INFO(kT, "received Ctrl+C, exiting");
    }
    st.exit_code = 1;
    st.interrupted = true;
    st.in_attempt = false;
    r.stop();
  };
  r.on_signal(SIGINT, interrupt);
  r.on_signal(SIGTERM, interrupt);
  signal(SIGPIPE, SIG_IGN);

  start_attempt();
  r.run();
  // Orderly teardown: sessions first, then the transport (sends "bye").
  st.serve.reset();
  st.proxy.reset();
  st.transport.reset();
  // Let queued close/bye frames go out.
  r.run_until([] { return false; }, 50);
  if (st.interrupted) fprintf(stderr, "Error: interrupted by user\n");
  else if (st.exit_code) fprintf(stderr, "Error: %s failed after %llu attempts\n", cfg.mode.c_str(),
                                 static_cast<unsigned long long>(cfg.max_retries));
  return st.exit_code;
}

}  // namespace p2pt
