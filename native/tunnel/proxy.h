// Proxy (consumer) role: sends HELLO, waits for AGREE, then serves HTTP/1.1
// on the listen address and multiplexes each request onto the channel as a
// stream.
//
// Behavioural parity with reference tunnel/src/proxy.rs:
//   - HELLO -> AGREE (300 s), then PING every 10 s (first immediately)    (:65-103)
//   - the listener binds only after the handshake and logs
//     "proxy listening on http://ADDR" (scripts grep it)                  (:175-177)
//   - stream ids are monotone from 1                                       (:52, :265)
//   - REQ_HEADERS{stream_id,method,path_and_query,headers} (all visible-
//     ASCII request headers incl. host), REQ_BODY <= 65408 B, REQ_END      (:265-336)
//   - 60 s wait for RES_HEADERS -> 504 "Tunnel response timeout"; ERROR or
//     END before headers -> 502 "Tunnel error: ..."                       (:339-376)
//   - response minus transfer-encoding/connection, body streamed per frame (:379-419)
// Differences (local only, wire-compatible): request bodies are streamed
// instead of fully buffered; a mid-stream ERROR aborts the client connection
// instead of ending the body as if complete (Q10); a client disconnect sends
// CANCEL when the peer negotiated it (Q12); --listen-early binds before the
// handshake and answers 503 "Tunnel not ready" until it completes (Q8).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <unordered_map>

#include "proto/frame.h"
#include "tunnel/channel.h"
#include "tunnel/scheduler.h"

namespace p2pt {

struct ProxyConfig {
  std::string listen = "127.0.0.1:8000";
  uint64_t handshake_timeout_ms = 300000;
  uint64_t header_timeout_ms = 60000;
  uint64_t ping_interval_ms = 10000;
  uint64_t pong_timeout_ms = 0;
  bool listen_early = false;
  size_t high_water = 4 << 20;
  size_t low_water = 1 << 20;
  // Pre-shared secret ("psk" extension, --secret): HELLO carries a proof and
  // an AGREE without the serve side's proof ends the session.
  std::string secret;
  // Called with the bound address once listening (tests/bench use port 0).
  std::function<void(const std::string&)> on_listening;
};

class ProxyConn;
class TcpListener;

class ProxySession : public std::enable_shared_from_this<ProxySession> {
 public:
  static std::shared_ptr<ProxySession> start(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg,
                                             std::function<void(const std::string&)> done);
  ~ProxySession();
  // Hand an accepted client socket to this session (used by the early
  // listener, which outlives sessions; see tunnel/app.cc).
  void accept(int fd);
  void stop(const std::string& why);
  bool ready() const { return ready_; }

  // ---- used by ProxyConn
  uint32_t next_stream_id() { return next_sid_++; }
  void register_stream(uint32_t sid, std::weak_ptr<ProxyConn> c) { streams_[sid] = std::move(c); }
  void unregister_stream(uint32_t sid) { streams_.erase(sid); }
  void send(proto::Frame f) { sched_->send(std::move(f)); }
  bool congested() const { return sched_->over_high(); }
  size_t body_chunk() const { return sched_->body_chunk(); }
  void add_paused_reader(std::weak_ptr<ProxyConn> c) { paused_readers_.push_back(std::move(c)); }
  bool cancel_feature() const { return cancel_feature_; }
  const ProxyConfig& config() const { return cfg_; }
  Reactor& reactor() { return r_; }

 private:
  ProxySession(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg);
  void on_open();
  void on_message(Bytes raw);
  void on_agree(const proto::Frame& f);
  void route(const proto::Frame& f);
  void send_ping();
  bool bind_listener();
  void on_relief();

  Reactor& r_;
  std::shared_ptr<MessageChannel> ch_;
  std::unique_ptr<FrameScheduler> sched_;
  ProxyConfig cfg_;
  std::function<void(const std::string&)> done_;
  std::unique_ptr<TcpListener> listener_;
  std::unordered_map<uint32_t, std::weak_ptr<ProxyConn>> streams_;
  std::unordered_map<ProxyConn*, std::shared_ptr<ProxyConn>> conns_;
  std::vector<std::weak_ptr<ProxyConn>> paused_readers_;
  uint32_t next_sid_ = 1;
  bool hello_sent_ = false;
  bool ready_ = false;
  bool stopped_ = false;
  bool cancel_feature_ = false;
  std::string psk_nonce_;  // psk extension: the nonce our HELLO carried
  uint64_t agree_timer_ = 0;
  uint64_t ping_timer_ = 0;
  uint64_t last_pong_ms_ = 0;
  friend class ProxyConn;
};

}  // namespace p2pt
