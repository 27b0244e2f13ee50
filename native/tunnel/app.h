// Application layer: supervisor (retry with exponential backoff), transport
// establishment and role sessions.
//
// Mirrors reference tunnel/src/main.rs:
//   - run_with_retry: re-run connect -> serve/proxy forever; backoff
//     min(2 * 2^(min(attempt,10)-1), 60) s; attempt never reset (Q5, kept
//     by default; --reset-backoff-after opts into a reset)         (main.rs:111-159)
//   - Ctrl-C aborts a running attempt and a backoff sleep            (main.rs:119-125, :149-155)
//   - startup log lines and "TURN server configured: ..."           (main.rs:43-48, :79-84)
#pragma once

#include <functional>
#include <memory>
#include <string>

#include "core/reactor.h"
#include "tunnel/channel.h"
#include "tunnel/proxy.h"
#include "tunnel/serve.h"

namespace p2pt {

struct TurnConfig {
  std::string url;
  std::string username;
  std::string password;
  bool set() const { return !url.empty(); }
};

struct RtcOptions {
  std::vector<std::string> stun_servers{"stun:stun.l.google.com:19302"};
  TurnConfig turn;
  bool include_loopback = true;     // host candidates on lo (offline / same-host peers)
  bool include_ipv6 = false;
  bool ipv6_only = false;
  bool relay_only = false;            // iceTransportPolicy=relay
  uint64_t gather_timeout_ms = 5000;  // reference waits <= 5 s (rtc.rs:181-182)
  uint64_t ice_failed_timeout_ms = 30000;
  size_t sctp_mtu = 1200;             // interop-safe DTLS payload budget
  bool allow_jumbo_loopback = true;   // larger SCTP packets when both ends say so and path is loopback
};

struct AppConfig {
  std::string mode;  // "serve" | "proxy"
  std::string signal = "wss://signal-server.fly.dev";
  std::string room;
  std::string upstream;
  std::string advertise = "/";
  std::string listen = "127.0.0.1:8000";
  std::string transport = "webrtc";  // or tcp-listen:HOST:PORT / tcp-connect:HOST:PORT
  RtcOptions rtc;
  uint64_t max_retries = UINT32_MAX;
  uint64_t reset_backoff_after_s = 0;  // 0 = never reset (reference)
  uint64_t pong_timeout_ms = 0;
  uint64_t ping_interval_ms = 10000;
  uint64_t header_timeout_ms = 60000;
  uint64_t handshake_timeout_ms = 300000;
  bool listen_early = false;
  std::string metrics_listen;
  size_t upstream_prewarm = 4;
  uint64_t upstream_prewarm_ttl_ms = 1000;
  // Adaptive busy polling (Reactor::set_busy_poll_us) on the association
  // thread and the workers: after any I/O a loop polls epoll for this long
  // before it sleeps, so the next hop of a request or token (often tens of
  // microseconds later) finds it awake. A deep-idle CPU on the MI355X host
  // (C2, 100 us exit latency) took 10-20 us longer per hand-off
  // (tunnel-wakebench, profiles/r05/b01); the headline's added p50 TTFT went
  // 0.157 -> 0.115 ms over 12 interleaved runs of 0 vs 250 us (b02-b04) for
  // 0.4-1 % of a core per tunnel process.
  uint64_t busy_poll_us = 250;
  // HTTP worker threads next to the association thread (-1 = auto: one per
  // 4 CPUs, 1..4; 0 = everything on one reactor thread).
  int workers = -1;
  // Streams kept on the association thread before new ones go to workers.
  size_t inline_streams = 16;
  // "assoc" extension (tunnel/assoc.h): associations in total, <= 1 = off.
  // 3 by default: on the MI355X host the 64 x 1 MB echo went 0.61 -> 0.83 of
  // direct at 1200 MTU and the download next to SSE 0.21 -> 0.43, the
  // headline unchanged (profiles/r06/b02, b03).
  uint32_t assoc = 3;
  // serve: request bodies at least this big stream to the upstream as they
  // arrive; 413 above max_request_body (0 = unlimited).
  uint64_t stream_body_threshold = 8 << 20;
  uint64_t max_request_body = 0;
  std::string secret;  // "psk" extension; empty = reference behaviour
};

// Establishes one MessageChannel (signalling + WebRTC, or a TCP debug link).
// The callback fires exactly once. The returned handle keeps the transport
// machinery (peer connection, signalling socket) alive; dropping it tears
// everything down (the signalling client sends "bye").
using ConnectCb = std::function<void(std::shared_ptr<MessageChannel>, std::string err)>;
std::shared_ptr<void> connect_transport(Reactor& r, const AppConfig& cfg, ConnectCb cb);

// Runs the supervisor loop until Ctrl-C / SIGTERM or max_retries. Returns the
// process exit code.
int run_app(const AppConfig& cfg);

// Backoff in seconds for the n-th failed attempt (n >= 1).
uint64_t backoff_secs(uint64_t attempt);

}  // namespace p2pt
