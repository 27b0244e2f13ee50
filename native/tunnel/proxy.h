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
// instead of fully buffered, and a stream whose REQ_BODY frames pile up has
// just its own client read paused; a mid-stream ERROR aborts the client
// connection instead of ending the body as if complete (Q10); a client
// disconnect sends CANCEL when the peer negotiated it (Q12); --listen-early
// binds before the handshake and answers 503 "Tunnel not ready" until it
// completes (Q8).
//
// Threads (tunnel/workers.h): the session (handshake, keepalive, routing of
// RES_* frames by stream id) lives on the association thread; each client
// connection lives on one reactor — the association thread's own for the
// first `inline_streams` connections, a worker's beyond that (the reference's
// task per connection, proxy.rs:196-217).
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include <unordered_map>
#include <unordered_set>

#include "proto/frame.h"
#include "tunnel/channel.h"
#include "tunnel/scheduler.h"
#include "tunnel/workers.h"

namespace p2pt {

namespace rtc {
struct PcConfig;
}
class AssocGroup;
class ProxyRouter;

struct ProxyConfig {
  std::string listen = "127.0.0.1:8000";
  uint64_t handshake_timeout_ms = 300000;
  uint64_t header_timeout_ms = 60000;
  uint64_t ping_interval_ms = 10000;
  uint64_t pong_timeout_ms = 0;
  bool listen_early = false;
  size_t high_water = 4 << 20;
  size_t low_water = 1 << 20;
  size_t stream_budget = 256 << 10;  // one upload's queued bytes before its client read pauses
  // Pre-shared secret ("psk" extension, --secret): HELLO carries a proof and
  // an AGREE without the serve side's proof ends the session.
  std::string secret;
  // Client connections kept on the association thread before new ones go to
  // worker threads (see tunnel/workers.h).
  size_t inline_streams = 16;
  // Called with the bound address once listening (tests/bench use port 0).
  std::function<void(const std::string&)> on_listening;
  // "assoc" extension (tunnel/assoc.h): associations wanted in total, the
  // first included (<= 1: off); `assoc_pc` builds the extra PeerConnections
  // (null: the transport has none); their threads busy-poll `busy_poll_us`.
  uint32_t assoc = 1;
  std::shared_ptr<const rtc::PcConfig> assoc_pc;
  uint64_t busy_poll_us = 0;
  // This session's association: 0 = the first (the listener; negotiates the
  // others), k > 0 = an extra one, which takes client connections from the
  // first session's `router` only.
  size_t assoc_index = 0;
  std::shared_ptr<ProxyRouter> router;
};

class ProxySession;

// Which association a client connection's request runs on (the "assoc"
// extension; thread-safe, shared by the first session and the extra ones).
// Requests known to be bulk — a request body of at least Placement::kBulkBytes,
// or a route whose last response was that large and not streamed — move their
// connection to the ready extra association with the fewest such
// connections; every other request runs on the first association, so SSE
// tokens never wait behind bulk data in one association's queues. The route
// table is shared too: what one thread learns, every thread places by.
class ProxyRouter : public std::enable_shared_from_this<ProxyRouter> {
 public:
  void attach(size_t k, Reactor* r, std::weak_ptr<ProxySession> s);
  // Association k's session is going away: nothing is handed to it any more
  // (its connections go to the first association), and its reactor is not
  // touched after this returns.
  void detach(size_t k);
  void set_ready(size_t k, bool ready);
  // The association for a bulk request: the ready one with the fewest bulk
  // connections — the first association only while no interactive request
  // has run on it for quiet_us (a download placed there in a lull stays until
  // it ends: SSE TTFT p99 next to downloads 0.53-1.26 ms with the first
  // association taking bulk while idle, profiles/r06/b11) — or -1 when no
  // extra association is ready.
  // `counted_on_first`: the asking connection is counted on the first one.
  int pick_bulk(bool counted_on_first = false);
  void count(size_t k);
  // Interactive requests in flight on association k (+1 / -1).
  void interactive(size_t k, int delta);
  // The association for an interactive request of a connection on `own`:
  // the first one, unless it already carries kSpill interactive requests —
  // node-scale load (one association thread per side ~90 % busy at 1024
  // streams, profiles/r05/b11/nodeprof) — then the extra one with the fewest.
  // With the load gate (the default), only while the first one's thread is
  // at least kSpillLoad busy, and only to threads below it. Two boxes, 3
  // interleaved reps each (profiles/r06/b13, b20): at 1024 streams the gate
  // is ahead on both (events 0.855 / 0.851 of direct vs 0.841 / 0.838 on the
  // count alone, added p50 TTFT 3.7 / 3.9 vs 4.5 / 4.5 ms); at 256 streams the
  // two are within the spread (added p50 0.356 / 0.342 vs 0.293 / 0.338 ms).
  // -1: no ready association.
  int pick_interactive(size_t own);
  static constexpr size_t kSpill = 32;
  static constexpr uint64_t kQuietUs = 30000000;
  void set_quiet_us(uint64_t us) {  // tests
    std::lock_guard<std::mutex> lk(mu_);
    quiet_us_ = us;
  }
  static constexpr double kSpillLoad = 0.5;  // Reactor::load() of a busy association thread
  void set_load_gate(bool on) {
    std::lock_guard<std::mutex> lk(mu_);
    load_gate_ = on;
  }
  // Moves a client connection (its socket and the bytes read but not parsed)
  // to association k's session; k > 0 counts it there until release(k).
  void hand(size_t k, int fd, Bytes unparsed);
  void release(size_t k);
  // Tests: where association k's thread load comes from (default: its reactor).
  void set_load_fn(std::function<double(size_t)> f) { load_fn_ = std::move(f); }
  bool bulk_route(const std::string& key);
  void note_route(const std::string& key, uint64_t bytes, bool streaming);
  size_t connections(size_t k);

 private:
  struct Target {
    Reactor* r = nullptr;
    std::weak_ptr<ProxySession> s;
    bool ready = false;
    size_t conns = 0;
    size_t interactive = 0;  // interactive requests in flight
  };
  double load(size_t k) const;  // mu_ held
  std::mutex mu_;
  std::vector<Target> t_;
  BulkRoutes routes_;
  uint64_t quiet_us_ = kQuietUs;
  bool load_gate_ = true;
  uint64_t last_interactive_us_ = 0;  // the last interactive request start / end on the first association (0: never)
  std::function<double(size_t)> load_fn_;
};

class ProxyConn;
class ProxyWorker;
class TcpListener;

class ProxySession : public std::enable_shared_from_this<ProxySession> {
 public:
  static std::shared_ptr<ProxySession> start(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg,
                                             std::function<void(const std::string&)> done,
                                             WorkerPool* pool = nullptr);
  ~ProxySession();
  // Hand an accepted client socket to this session (also used by the early
  // listener, which outlives sessions; see tunnel/app.cc).
  void accept(int fd);
  // A client connection handed over by another association's session
  // (ProxyRouter::hand): `counted` when the router counts it on this one.
  void adopt_handed(int fd, Bytes unparsed, bool counted);
  void stop(const std::string& why);
  bool ready() const { return ready_; }

  // State the connection threads read.
  struct Shared {
    ProxyConfig cfg;
    std::atomic<uint32_t> next_sid{1};
    std::atomic<bool> ready{false};
    std::atomic<bool> cancel_feature{false};
    std::atomic<bool> flow{false};  // "flow" negotiated: per-stream credit both ways
    std::atomic<uint64_t> rtt_us{0};  // transport SRTT, refreshed as body frames arrive ("flow" windows)
    size_t body_chunk = proto::kMaxBodyChunk;
    size_t workers = 0;  // worker threads beside the association thread
    size_t assoc_index = 0;                // this session's association ("assoc")
    std::shared_ptr<ProxyRouter> router;   // shared by all associations' sessions
  };
  // Association thread -> a connection thread.
  struct Cmd {
    enum Kind : uint8_t { Adopt, Headers, Body, End, Error, Pause, Resume, Credit } kind;
    explicit Cmd(Kind k, uint32_t s = 0) : kind(k), sid(s) {}
    uint32_t sid = 0;
    int fd = -1;                                  // Adopt
    uint64_t t_us = 0;                            // Adopt: accept time (TUNNEL_TRACE)
    Bytes data;                                   // Body / Error message; Adopt: bytes already read
    std::vector<Bytes> more;                      // Body: the rest of a frame that arrived in fragments
    std::shared_ptr<proto::ResponseHeaders> rh;   // Headers
    uint32_t bytes = 0;                           // Credit: REQ_BODY bytes granted by serve
    bool urgent = false;                          // the start of a response: handed over at once (Pipe::push)
    bool counted = false;                         // Adopt: counted on this association by the router
  };
  // A connection thread -> association thread.
  struct Ev {
    // Migrate: an inline connection whose request turned out bulk hands its
    // socket (fd) and unparsed bytes (frame.payload) to a worker.
    enum Kind : uint8_t { Route, Unroute, Frame, ConnClosed, Migrate } kind;
    explicit Ev(Kind k, uint32_t s = 0) : kind(k), sid(s) {}
    uint32_t sid = 0;
    int fd = -1;
    proto::Frame frame{proto::MsgType::Ping, 0, Bytes()};
  };

 private:
  struct Link {
    Reactor* r = nullptr;
    std::unique_ptr<Pipe<Cmd>> to;
    std::shared_ptr<ProxyWorker> worker;  // owned here; released on its own thread
  };
  struct Route {
    size_t thread = 0;
    bool paused = false;
    bool body_seen = false;  // trace: first RES_BODY frame out of the channel
  };
  ProxySession(Reactor& r, std::shared_ptr<MessageChannel> ch, ProxyConfig cfg);
  void init_links(WorkerPool* pool);
  void release_links(const std::string& fail_why);
  void on_open();
  void on_message(Bytes raw, std::vector<Bytes>* more = nullptr);
  void on_agree(const proto::Frame& f);
  void route(const proto::Frame& f);
  void send_ping();
  void watchdog();  // send-path stall watchdog (1 s)
  bool bind_listener();
  void on_event(size_t thread, Ev& ev);
  void check_paused();
  void start_assoc(uint32_t count);
  // "assoc": extra associations only on paths with a base RTT up to this
  // (same host, LAN, metro). Early samples of a loopback path read 2-5 ms in
  // a loaded build container (startup work on both loops), a WAN path tens.
  static constexpr uint64_t kAssocMaxRttUs = 10000;
  void command(size_t thread, Cmd c) {
    const bool urgent = c.urgent;
    links_[thread].to->push(std::move(c), urgent);
  }

  Reactor& r_;
  std::shared_ptr<MessageChannel> ch_;
  std::unique_ptr<FrameScheduler> sched_;
  ProxyConfig cfg_;
  std::shared_ptr<Shared> shared_;
  std::function<void(const std::string&)> done_;
  std::unique_ptr<TcpListener> listener_;
  WorkerPool* pool_ = nullptr;
  std::shared_ptr<AssocGroup> assoc_;  // extra associations ("assoc"), first association only
  std::unordered_map<uint32_t, Route> routes_;
  std::unordered_set<uint32_t> paused_;
  std::vector<Link> links_;
  std::unique_ptr<Placement> place_;
  bool hello_sent_ = false;
  bool ready_ = false;
  bool stopped_ = false;
  std::string psk_nonce_;  // psk extension: the nonce our HELLO carried
  uint64_t agree_timer_ = 0;
  uint64_t ping_timer_ = 0;
  uint64_t wd_timer_ = 0;
  int wd_stalled_s_ = 0;
  uint64_t last_pong_ms_ = 0;
  friend class ProxyWorker;
};

}  // namespace p2pt
