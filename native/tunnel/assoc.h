// Parallel associations (extension "assoc"): N - 1 extra PeerConnections
// beside the one the rendezvous established, each with its own SCTP
// association on its own thread, so bulk transfers are not capped by one
// association thread per side.
//
// Why: with the socket reader's records opened on lanes, the association
// thread is the saturated stage of a 1200-MTU bulk transfer (>= 90 % busy;
// 44 % of it copying fragments into messages, 9 % SACKs; docs/ROUND5.md),
// and three single-thread remedies did not move it. The reference has one
// PeerConnection and one data channel "tunnel" (rtc.rs:126-273, :133); so
// does this tunnel whenever a peer does not list "assoc".
//
// Protocol (both sides list "assoc"; HELLO carries the proxy's count, AGREE
// the agreed min(proxy, serve), proto/frame.h):
//   - the extra connections are signalled in-band on the first data channel
//     (ASSOC frames, stream_id = index 1..N-1), never through the signal
//     server: the proxy offers, serve answers, candidates trickle both ways;
//   - each extra connection carries one data channel "tunnel" with its own
//     HELLO/AGREE (without "assoc") and a serve / proxy session of its own;
//   - stream ids are per channel, as every frame of a request and its
//     response stays on the channel the request came in on.
// Placement (proxy side, tunnel/proxy.h ProxyRouter): requests known to be
// bulk (a large upload, or a route whose last response was a large
// non-streaming body) move their client connection to the least-loaded ready
// extra association; every other request runs on the first, so SSE tokens
// never queue behind bulk data in one association. An extra association that
// fails is dropped from placement (its requests fail like any tunnel error);
// the first one's failure ends the whole tunnel as before.
//
// Threads: AssocGroup lives on the first association's thread (the session
// that negotiated it); link k's PeerConnection, data channel and session live
// on its own reactor thread (WorkerThread) and talk to the group only through
// post_threadsafe.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/reactor.h"
#include "proto/frame.h"
#include "tunnel/channel.h"
#include "tunnel/workers.h"

namespace p2pt {

namespace rtc {
struct PcConfig;
}

class AssocLink;

class AssocGroup : public std::enable_shared_from_this<AssocGroup> {
 public:
  // Starts the session of extra association `index` on its thread `r` once
  // its data channel is open; `done` reports the session's end. Returns what
  // keeps the session alive (dropped on that thread).
  using SessionFactory = std::function<std::shared_ptr<void>(
      Reactor& r, std::shared_ptr<MessageChannel> ch, size_t index, std::function<void(const std::string&)> done)>;
  // Sends one ASSOC frame on the first data channel (primary thread).
  using SendFn = std::function<void(proto::Frame)>;
  // Link state changes (primary thread): index, up (session started) / down.
  using StateFn = std::function<void(size_t index, bool up, const std::string& why)>;

  // `offerer`: the proxy side creates and offers the extra connections; the
  // serve side answers them as their offers arrive. `count`: associations in
  // total (the first included).
  static std::shared_ptr<AssocGroup> create(Reactor& primary, bool offerer, uint32_t count, const rtc::PcConfig& pc,
                                            uint64_t busy_poll_us, SessionFactory factory, SendFn send,
                                            StateFn state = nullptr);
  ~AssocGroup();
  // An ASSOC frame from the peer (primary thread).
  void on_frame(const proto::Frame& f);
  size_t extra() const { return threads_.size(); }
  Reactor& reactor(size_t index) { return threads_[index - 1]->reactor(); }

 private:
  friend class AssocLink;
  AssocGroup(Reactor& primary, bool offerer, uint32_t count, const rtc::PcConfig& pc, uint64_t busy_poll_us,
             SessionFactory factory, SendFn send, StateFn state);
  void start();
  // From link threads (via post_threadsafe onto the primary thread).
  void send_signal(size_t index, const std::string& kind, const std::string& key, const std::string& value);
  void link_state(size_t index, bool up, const std::string& why);

  Reactor& primary_;
  bool offerer_;
  std::unique_ptr<rtc::PcConfig> pc_;
  SessionFactory factory_;
  SendFn send_;
  StateFn state_;
  std::vector<std::unique_ptr<WorkerThread>> threads_;
  std::vector<std::shared_ptr<AssocLink>> links_;  // each used on its own thread only
};

// The associations a HELLO asks for / an AGREE grants, and the JSON of one
// ASSOC frame (exposed for tests).
uint32_t assoc_agree(uint32_t proxy_count, uint32_t serve_count);
proto::Frame make_assoc_frame(uint32_t index, const std::string& kind, const std::string& key,
                              const std::string& value);

}  // namespace p2pt
