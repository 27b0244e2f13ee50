// Serve (provider) role: answers HELLO with AGREE, then turns REQ_* frames
// into upstream HTTP requests and streams RES_* frames back.
//
// Behavioural parity with reference tunnel/src/serve.rs:
//   - wait for HELLO (300 s), reply AGREE, log "sent AGREE, tunnel ready"  (:37-59)
//   - PING every 10 s, first one immediately; PING -> PONG              (:68-80, :140-148)
//   - REQ_HEADERS keyed by the JSON stream_id; REQ_BODY appended; REQ_END
//     starts the upstream request                                        (:112-139)
//   - upstream connect failure -> 502 text/plain "Bad Gateway: ..." + END (:219-242)
//   - RES_BODY per upstream read, sub-chunked at 65408 B                 (:263-276)
//   - mid-stream upstream failure -> ERROR "upstream error: ..." + END    (:278-290)
// Local robustness fixes (wire-compatible): malformed
// REQ_HEADERS (Q3) and unparseable methods (Q4) answer 400 instead of killing
// the session / hanging the client; a stream whose frames queue up beyond its
// budget has just its own upstream read paused (Q11); a negotiated CANCEL
// aborts the upstream request (Q12).
//
// Threads (tunnel/workers.h): the session, frame scheduler and stream table
// live on the association thread; each upstream call runs on one reactor —
// the association thread's own for the first `inline_streams` concurrent
// requests, a worker's beyond that (the reference's task per request,
// serve.rs:131-137).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "http/client.h"
#include "proto/frame.h"
#include "tunnel/channel.h"
#include "tunnel/scheduler.h"
#include "tunnel/workers.h"

namespace p2pt {

namespace rtc {
struct PcConfig;
}
class AssocGroup;

struct ServeConfig {
  // One upstream base URL, or several separated by commas (extension: e.g. one
  // inference endpoint per GPU of the node); each request goes to the one
  // with the fewest requests in flight, ties round-robin.
  std::string upstream;
  std::string advertise = "/";
  uint64_t handshake_timeout_ms = 300000;
  uint64_t ping_interval_ms = 10000;
  uint64_t pong_timeout_ms = 0;  // 0 = reference behaviour (PONG only logged)
  size_t high_water = 4 << 20;   // all streams: above this, backlogged streams pause
  size_t low_water = 1 << 20;
  size_t stream_budget = 256 << 10;  // one stream's queued bytes before its upstream read pauses
  // Spare pre-connected upstream sockets (0 = connect per request like reqwest).
  size_t upstream_prewarm = 4;
  uint64_t upstream_prewarm_ttl_ms = 1000;  // close unused warm sockets after this idle time
  // Pre-shared secret ("psk" extension, --secret): when set, a HELLO without a
  // valid proof ends the session; empty = room name only (reference).
  std::string secret;
  // Concurrent upstream calls kept on the association thread before new ones
  // go to worker threads (see tunnel/workers.h).
  size_t inline_streams = 16;
  // Request bodies are buffered to REQ_END like the reference (serve.rs:120-
  // 139) while below this size (declared or received); larger ones stream to
  // the upstream as they arrive, so serve memory stays bounded.
  uint64_t stream_body_threshold = 8 << 20;
  // 413 above this many request-body bytes (0 = unlimited, the reference).
  uint64_t max_request_body = 0;
  // "assoc" extension (tunnel/assoc.h): associations this side accepts in
  // total, the first included (<= 1: off); `assoc_pc` builds the extra
  // PeerConnections (null: the transport has none, e.g. TCP); their threads
  // busy-poll like the rest (`busy_poll_us`).
  uint32_t assoc = 1;
  std::shared_ptr<const rtc::PcConfig> assoc_pc;
  uint64_t busy_poll_us = 0;
  // This session's association: 0 = the first (negotiates the others), k > 0
  // = an extra one (its HELLO has no "assoc"; it registers no gauges).
  size_t assoc_index = 0;
};

class ServeWorker;

class ServeSession : public std::enable_shared_from_this<ServeSession> {
 public:
  // `done` fires once with the reason the session ended (always an error:
  // like the reference, a session only ends on failure). `pool` (may be null)
  // supplies the worker threads.
  static std::shared_ptr<ServeSession> start(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg,
                                             std::function<void(const std::string&)> done,
                                             WorkerPool* pool = nullptr);
  ~ServeSession();
  void stop(const std::string& why);
  size_t active_streams() const { return streams_.size() + inflight_.size(); }

  // Association thread -> the reactor running a call.
  struct Cmd {
    enum Kind : uint8_t { Start, Cancel, Pause, Resume, Prewarm, Body, BodyEnd } kind;
    explicit Cmd(Kind k, uint32_t s = 0) : kind(k), sid(s) {}
    uint32_t sid = 0;
    http::ClientRequest req;  // Start
    size_t body_chunk = 0;    // Start: RES_BODY payload size for this channel
    bool retryable = false;   // Start: hand the request back if the upstream is unreachable
    bool grant = false;       // Start: report consumed streamed-body bytes (Ev::Credit)
    Bytes data;               // Body
    std::vector<Bytes> more;  // Body: the rest of a frame that arrived in fragments
  };
  // An upstream call that never connected, handed back for another upstream.
  struct Unreachable {
    http::ClientRequest req;
    std::string err;
  };
  // A call's reactor -> association thread.
  struct Ev {
    enum Kind : uint8_t { Frame, Done, Credit } kind;
    explicit Ev(Kind k, uint32_t s = 0) : kind(k), sid(s) {}
    uint32_t sid = 0;
    proto::Frame frame{proto::MsgType::Ping, 0, Bytes()};
    bool responded = false;                    // Done: the upstream answered (any status)
    std::shared_ptr<Unreachable> unreachable;  // Done: no connection, nothing sent yet
    uint32_t bytes = 0;                        // Credit: streamed-body bytes the upstream took
  };

 private:
  struct Pending {
    proto::RequestHeaders headers;
    std::vector<Bytes> body;
    uint64_t body_len = 0;
    int64_t declared = -1;  // content-length of the request, if given
    bool rejected = false;  // 413 sent: drop the rest of the body
    uint64_t owed = 0;      // "flow": received body bytes not yet granted back
  };
  struct Inflight {
    size_t up = 0;      // index into ups_
    size_t thread = 0;  // index into links_
    bool paused = false;  // what the call's reactor was last told
    uint8_t tries = 0;  // upstreams tried after connect failures
    std::string path;   // request path (the URL is rebuilt for another upstream)
    bool bp = false;    // paused because its frames pile up here (back-pressure)
    bool fc = false;    // paused because the peer's credit ran out ("flow")
    bool uploading = false;   // request body still streaming to the upstream
    uint64_t uploaded = 0;    // request-body bytes received
    int64_t credit = proto::flow_window();  // "flow": RES_BODY bytes we may still send
    proto::FlowWindow upwin;              // "flow": streamed REQ_BODY window autotuning
    std::string route;                    // BulkRoutes key
    uint64_t res_bytes = 0;               // response body bytes so far
    bool res_streaming = false;           // SSE / NDJSON response
  };
  // One upstream origin (one inference endpoint, e.g. one per GPU) and its
  // passive health: an origin that refuses connections is ejected for an
  // exponentially growing time (1 s .. 30 s) and requests go to the others.
  struct Upstream {
    std::string base;
    size_t outstanding = 0;
    uint64_t down_until_ms = 0;
    uint32_t fails = 0;
  };
  struct Link {
    Reactor* r = nullptr;
    std::unique_ptr<Pipe<Cmd>> to;
    std::shared_ptr<ServeWorker> worker;  // owned here; released on its own thread
  };
  size_t pick_upstream(size_t avoid = SIZE_MAX);
  void release_upstream(const Inflight& f) {
    if (f.up < ups_.size() && ups_[f.up].outstanding) ups_[f.up].outstanding--;
  }
  void send_start(uint32_t sid, Inflight& fl, http::ClientRequest req);
  bool any_healthy(size_t except) const;

  ServeSession(Reactor& r, std::shared_ptr<MessageChannel> ch, ServeConfig cfg);
  void init_links(WorkerPool* pool);
  void release_links();
  void on_open();
  void on_message(Bytes raw, std::vector<Bytes>* more = nullptr);
  void on_hello(const proto::Frame& f);
  void handle_frame(const proto::Frame& f);
  void start_request(uint32_t sid, Pending p, bool streaming);
  void send_simple_response(uint32_t sid, uint16_t status, const std::string& body);
  void send_ping();
  void watchdog();  // send-path stall watchdog (1 s)
  void on_event(Ev& ev);
  void check_paused();
  void set_paused(uint32_t sid, Inflight& fl);
  void grant(uint32_t sid, uint64_t& owed, uint64_t n, bool force = false);
  void reject_too_large(uint32_t sid);
  void command(size_t thread, Cmd c) {
    const bool urgent = c.kind == Cmd::Start;  // a new request: handed over at once (Pipe::push)
    links_[thread].to->push(std::move(c), urgent);
  }

  void start_assoc(uint32_t count);

  Reactor& r_;
  std::shared_ptr<MessageChannel> ch_;
  std::unique_ptr<FrameScheduler> sched_;
  ServeConfig cfg_;
  std::function<void(const std::string&)> done_;
  WorkerPool* pool_ = nullptr;
  std::shared_ptr<AssocGroup> assoc_;  // extra associations ("assoc"), first association only
  bool handshaken_ = false;
  bool stopped_ = false;
  bool cancel_feature_ = false;
  bool flow_ = false;  // "flow" negotiated: per-stream credit both ways
  uint64_t hello_timer_ = 0;
  uint64_t ping_timer_ = 0;
  uint64_t wd_timer_ = 0;
  int wd_stalled_s_ = 0;
  uint64_t last_pong_ms_ = 0;
  std::unordered_map<uint32_t, Pending> streams_;
  std::unordered_map<uint32_t, Inflight> inflight_;
  std::unordered_set<uint32_t> paused_;
  std::vector<Upstream> ups_;
  size_t rr_ = 0;
  std::vector<Link> links_;
  std::unique_ptr<Placement> place_;
  BulkRoutes bulk_routes_;
  friend class ServeWorker;
};

}  // namespace p2pt
