// SCTP association over DTLS (RFC 9260 subset + RFC 8261 encapsulation),
// as used by WebRTC data channels.
//
// Replaces webrtc-sctp 0.10 in the reference stack. Implemented:
//   INIT/INIT-ACK/COOKIE-ECHO/COOKIE-ACK incl. simultaneous open (both WebRTC
//   peers send INIT), HMAC-signed stateless cookies; DATA fragmentation and
//   reassembly (B/E flags, ordered/unordered); SACK with gap blocks and
//   duplicate TSNs; RTO per RFC 6298; T3-rtx; fast retransmit on 3 miss
//   indications with fast recovery; cwnd/ssthresh slow start + congestion
//   avoidance; peer rwnd; zero-window probing; HEARTBEAT reply; SHUTDOWN /
//   ABORT; FORWARD-TSN receive; RE-CONFIG outgoing-stream-reset handling.
//
// Tuned for the tunnel's two traffic classes:
//   - small SSE tokens: no Nagle, no delayed SACK — everything produced during
//     one reactor batch is bundled and a SACK goes out per received batch;
//   - bulk bodies: large rwnd (8 MiB), RTO.min 100 ms, optional large packets
//     and initial cwnd on same-host paths.
#pragma once

#include <sys/uio.h>

#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_set>
#include <vector>

#include "core/buf.h"
#include "core/reactor.h"

namespace p2pt::rtc {

struct SctpConfig {
  uint16_t local_port = 5000;
  uint16_t remote_port = 5000;
  size_t mtu = 1200;                // max SCTP packet (DTLS record payload)
  size_t initial_cwnd = 0;          // 0 = RFC: min(4*MTU, max(2*MTU, 4380))
  uint32_t rwnd = 8u << 20;         // advertised receive window
  uint64_t rto_initial_ms = 1000;
  uint64_t rto_min_ms = 100;
  uint64_t rto_max_ms = 10000;
  int max_init_retrans = 8;
  int max_assoc_retrans = 20;
  uint64_t sack_delay_us = 5000;    // delayed SACK for lone packets (0 = always immediate)
  // RFC 9653 zero checksum with Error Detection Method 1 (the lower layer is
  // DTLS, which already authenticates every packet): advertised in INIT /
  // INIT-ACK; once both sides did, packets after setup carry checksum 0 and a
  // received checksum of 0 is not verified.
  bool zero_checksum = false;
  // Redundant copies of small whole messages: 1 always, 0 never, -1 once
  // the path has shown random loss.
  int dup_small = -1;
  // cwnd kept after a random loss, in % (50..100); -1: cc_policy() (tests
  // compare policies on one link with it).
  int random_beta_pct = -1;
};

// Congestion response (TUNNEL_SCTP_CC, read once; see sctp.cc).
struct CcPolicy {
  int random_beta_pct = 80;  // cwnd kept after a random (no standing queue) loss, in %
  bool queue_bound = true;   // the short-path queue bound
};
const CcPolicy& cc_policy();

struct SctpStats {
  uint64_t packets_sent = 0, packets_received = 0;
  uint64_t data_chunks_sent = 0, data_chunks_received = 0;
  uint64_t late_tsns = 0;  // new TSNs that arrived below the highest one seen (holes filled, reordering)
  uint64_t retransmits = 0, fast_retransmits = 0, t3_expirations = 0;
  uint64_t tlp_probes = 0, rack_marks = 0, random_loss_events = 0;
  uint64_t random_loss_cuts = 0;  // random-loss episodes that cut cwnd
  uint64_t congestion_cuts = 0;   // loss episodes read as congestion (0.7 cut)
  uint64_t queue_cuts = 0;        // short-path queue bound: cwnd cuts for a standing queue
  uint64_t over_bdp_losses = 0;   // ... of them because cwnd was past the delivery-rate BDP
  uint64_t hystart_exits = 0;     // initial slow starts ended by HyStart++ (rising delay)
  uint64_t dup_copies_sent = 0;  // redundant copies of small messages (lossy paths)
  uint64_t early_deliveries = 0;  // messages handed up ahead of a TSN gap (another stream's loss)
  uint64_t rwnd_drops = 0;        // out-of-order chunks dropped past the receive window
  uint64_t probe_ambiguous = 0;   // probe acks not taken as loss evidence (originals arrived with them)
  uint64_t spurious_undos = 0;    // loss episodes found spurious afterwards: cwnd cut undone
  uint64_t dup_tsns = 0;          // DATA chunks received again (spurious retransmissions, or lost SACKs)
  uint64_t sacks_sent = 0, sacks_received = 0;
  uint64_t bytes_sent = 0, bytes_received = 0;
};

class SctpAssociation : public std::enable_shared_from_this<SctpAssociation> {
 public:
  enum class State { Closed, CookieWait, CookieEchoed, Established, ShutdownPending, ShutdownSent, ShutdownReceived,
                     ShutdownAckSent };
  // One outbound SCTP packet as a gather list: common/chunk headers and small
  // payloads live in an internal assembly buffer, large payload slices are
  // referenced in place (the DTLS layer encrypts straight from them).
  // owners[i] is the Bytes that iov[i] is a view of (null for the assembly
  // buffer, which is reused after the call; `owners` itself may be null).
  using PacketOut = std::function<void(const iovec*, const Bytes* const* owners, int)>;

  static std::shared_ptr<SctpAssociation> create(Reactor& r, SctpConfig cfg, PacketOut out);
  // Contiguous view of a gathered packet (tests, fallbacks).
  static std::vector<uint8_t> flatten(const iovec* iov, int cnt) {
    std::vector<uint8_t> v;
    for (int i = 0; i < cnt; i++)
      v.insert(v.end(), static_cast<const uint8_t*>(iov[i].iov_base),
               static_cast<const uint8_t*>(iov[i].iov_base) + iov[i].iov_len);
    return v;
  }
  ~SctpAssociation();

  // Active open (send INIT). Safe to call on both peers (simultaneous open).
  void connect();
  // Feed one decrypted SCTP packet. Large single-chunk messages are delivered
  // as views into `pkt` (no copy); small ones are copied so a tiny message
  // never pins a whole receive buffer.
  void on_packet(const Bytes& pkt);
  void on_packet(const uint8_t* p, size_t n) { on_packet(Bytes::copy(p, n)); }
  void on_packets(const Bytes* pkts, size_t n);  // a receive burst
  // Queue a message made of gathered pieces (a single piece is never copied).
  bool send(uint16_t stream, uint32_t ppid, const std::vector<Bytes>& pieces, bool unordered = false);
  // Queue a message = a short header (copied, <= kMsgHdrMax bytes) followed by
  // a payload view (never copied): the tunnel's frame header + body.
  static constexpr size_t kMsgHdrMax = 16;
  // priority: a latency-sensitive message that fits one DATA chunk (an SSE
  // token frame, a control or credit frame) — sent ahead of queued bulk
  // messages that have not started, and up to kPriorityAllowance bytes past
  // cwnd, so it does not wait for a bulk transfer's window to drain.
  bool send_framed(uint16_t stream, uint32_t ppid, const uint8_t* hdr, size_t hlen, const Bytes& payload,
                   bool unordered = false, bool priority = false);
  // Build and emit packets (bundled). Called once per reactor batch.
  void flush();
  void shutdown();
  void abort(const std::string& reason);

  // Bytes accepted by send() that have not been transmitted yet.
  size_t buffered_amount() const { return unsent_bytes_; }
  // A SACK the next flush sends right away (>= 2 data packets unacknowledged,
  // a gap or duplicate to report, or the delayed-SACK timer fired).
  // Retransmissions or control chunks (stream reset, FORWARD-TSN, ...) are
  // waiting: a flush must not be held back for coalescing.
  bool urgent_pending() const { return !rtx_.empty() || !ctrl_.empty(); }
  bool ack_due() const {
    return sack_needed_ && (sack_urgent_ || data_pkts_unacked_ >= 2 || !ooo_.empty() || !dups_.empty());
  }
  size_t bytes_in_flight() const { return flight_size_; }
  State state() const { return state_; }
  bool established() const { return state_ == State::Established; }
  const SctpStats& stats() const { return stats_; }
  void set_dup_small(int mode) { cfg_.dup_small = mode; }  // tests: SctpConfig::dup_small after creation
  size_t cwnd() const { return cwnd_; }
  uint64_t srtt_us() const { return srtt_us_; }
  uint64_t min_rtt_us() const { return min_rtt_us_; }  // smallest RTT sample: the path's base RTT
  uint64_t last_round_min_rtt_us() const { return qb_last_; }  // smallest RTT of the last full round
  // One-line sender/receiver state for the send-path stall watchdog.
  std::string debug_state() const;
  uint64_t rto_us() const { return rto_us_; }
  void set_mtu(size_t mtu);
  void set_initial_cwnd(size_t c) { if (c > cwnd_) cwnd_ = c; }
  // Interactive traffic is flowing (see queue_bound()): the tighter queue
  // bound applies for the next 200 ms.
  void note_interactive();
  void request_stream_reset(uint16_t stream);

  std::function<void()> on_established;
  std::function<void(uint16_t stream, uint32_t ppid, Bytes msg)> on_message;
  // Optional: a fragmented message as the views of its fragments (the first
  // in `msg`, the rest in `more`, all zero-copy slices of the received
  // packets) instead of one reassembled copy. Unset: on_message gets a copy.
  std::function<void(uint16_t stream, uint32_t ppid, Bytes msg, std::vector<Bytes>& more)> on_message_chain;
  std::function<void(uint16_t stream)> on_stream_reset;  // peer reset its outgoing stream
  std::function<void(const std::string&)> on_closed;
  std::function<void()> on_sent;  // unsent_bytes_ decreased (back-pressure relief)

 private:
  struct Chunk;     // outbound DATA fragment
  struct BodyRef;   // a message body shared by its fragments
  struct InChunk;   // inbound DATA fragment awaiting cum-ack
  SctpAssociation(Reactor& r, SctpConfig cfg, PacketOut out);

  void packet_in(const Bytes& pkt);
  void handle_init(const uint8_t* c, size_t len, uint32_t vtag);
  void handle_init_ack(const uint8_t* c, size_t len);
  void handle_cookie_echo(const uint8_t* c, size_t len);
  void handle_data(uint8_t flags, const uint8_t* c, size_t len, const Bytes& pkt);
  void handle_sack(const uint8_t* c, size_t len);
  void handle_forward_tsn(const uint8_t* c, size_t len);
  void handle_reconfig(const uint8_t* c, size_t len);
  void handle_heartbeat(const uint8_t* c, size_t len);
  void handle_shutdown(const uint8_t* c, size_t len);
  void enter_established();
  void closed(const std::string& why);

  std::string make_cookie(uint32_t peer_tag, uint32_t peer_tsn, uint32_t peer_rwnd, uint16_t peer_os, uint16_t peer_mis,
                          uint32_t peer_flags);
  bool peer_offers_zero_checksum(const uint8_t* params, size_t len) const;
  void append_init_params(std::vector<uint8_t>& v);
  void send_init();
  void on_init_timer();
  void send_control(uint8_t type, uint8_t flags, const std::vector<uint8_t>& body, uint32_t vtag);
  void queue_control(uint8_t type, uint8_t flags, std::vector<uint8_t> body);
  void build_sack(std::vector<uint8_t>& body);
  void deliver_ready();
  void deliver_chunk(uint8_t fl, uint16_t st, uint16_t ssn, uint32_t pp, const Bytes& d);
  void deliver_message(uint16_t st, uint16_t ssn, bool unordered, uint32_t pp, Bytes msg,
                       std::vector<Bytes> more = {});
  void hand_up(uint16_t st, uint32_t pp, Bytes msg, std::vector<Bytes>& more);
  void release_ready(uint16_t st);
  void drain_in_order();
  void reset_inbound_stream(uint16_t st);
  static uint32_t stream_ssn(uint16_t st, uint16_t ssn) { return uint32_t(st) << 16 | ssn; }
  void update_rto(uint64_t rtt_us);
  void start_t3();
  void stop_t3();
  void on_t3();
  void arm_tlp();
  void on_tlp();
  void emit_packet(std::vector<uint8_t>& pkt);
  void begin_gather();
  void close_run();
  void emit_gather();
  void maybe_finish_shutdown();

  Reactor& r_;
  SctpConfig cfg_;
  PacketOut out_;
  State state_ = State::Closed;
  uint32_t my_vtag_, peer_vtag_ = 0;
  uint32_t my_init_tsn_, next_tsn_;
  uint8_t cookie_key_[32];
  std::vector<uint8_t> cookie_echo_;  // our COOKIE-ECHO while CookieEchoed
  int init_tries_ = 0;
  uint64_t init_timer_ = 0;

  // --- sender
  struct Msg {
    uint16_t stream;
    uint32_t ppid;
    bool unordered;
    uint16_t ssn;
    uint8_t hlen = 0;
    uint8_t hdr[kMsgHdrMax];
    Bytes body;      // message = hdr[0, hlen) ++ body (moved into `ref` at the first fragment)
    size_t len;
    size_t off = 0;  // bytes already fragmented
    BodyRef* ref = nullptr;
  };
  Chunk* new_chunk();
  void free_chunk(Chunk* c);
  BodyRef* new_ref(Bytes body);
  void unref(BodyRef* b);
  std::vector<Chunk*> chunk_free_;
  std::vector<BodyRef*> ref_free_;
  std::deque<Msg> sendq_;
  std::deque<Msg> sendq_pri_;  // single-chunk priority messages (send_framed(..., priority))
  std::map<uint16_t, uint16_t> next_ssn_;
  std::deque<Chunk*> inflight_;  // consecutive TSNs from cum_acked_ + 1
  // Loss bookkeeping kept incrementally (handle_sack is O(news), not O(window)):
  struct TsnLess {
    bool operator()(uint32_t a, uint32_t b) const { return int32_t(a - b) < 0; }
  };
  std::set<uint32_t, TsnLess> rtx_;  // TSNs marked for retransmission, in TSN order
  std::vector<std::pair<uint32_t, uint32_t>> gap_known_, blocks_;  // last SACK's gap blocks (absolute TSNs)
  struct SendRec {
    uint32_t tsn;
    int tx;            // transmission count this entry is for (stale once the chunk is sent again)
    uint64_t sent_us;
  };
  std::deque<SendRec> sendlog_;  // transmissions in send order (RACK)
  uint64_t rack_xmit_us_ = 0;    // latest send time of an acknowledged once-sent chunk (RACK.xmit_ts)
  std::vector<Chunk*> dup_;      // this flush's small whole messages to send twice
  static constexpr size_t kDupMaxChunk = 512;
  bool dup_small_enabled() const;
  size_t unsent_bytes_ = 0;
  size_t flight_size_ = 0;
  size_t cwnd_ = 0, ssthresh_ = 0, partial_acked_ = 0;
  size_t peer_rwnd_ = 0;
  uint32_t cum_acked_ = 0;  // peer's cumulative TSN ack
  bool fast_recovery_ = false;
  uint32_t fast_recovery_exit_ = 0;
  uint64_t t3_timer_ = 0;
  uint64_t tlp_timer_ = 0;  // tail-loss probe (fires before T3, no cwnd collapse)
  int tlp_count_ = 0;       // probes since the cumulative ack last advanced
  int cwnd_bypass_ = 0;     // chunks allowed out beyond cwnd (one per loss event)
  // HyStart++ state (hystart()).
  void hystart(uint32_t cum, uint64_t rtt_sample);
  static constexpr uint64_t kLongPathUs = 5000;  // base RTT from which a path counts as long (WAN)
  static constexpr int kHsSamples = 8, kCssRounds = 5, kHsLowWindow = 16;
  static constexpr size_t kCssDivisor = 4;
  // Delivery rate per round trip (bytes acknowledged between a round's first
  // SACK and the SACK covering the last TSN sent when it began), windowed max
  // over the last kDrRounds rounds in which the sender was cwnd-limited:
  // max rate x min RTT estimates the path's BDP (dr_bdp()).
  static constexpr int kDrRounds = 10;
  bool random_episode_ = false;  // a random-loss episode (no recovery period) is open until random_exit_
  uint32_t random_exit_ = 0;
  // Spurious-loss undo (after Linux's DSACK undo / RFC 3708): a loss
  // episode's cwnd cut is taken back if, once the window it covered is
  // acknowledged, none of its retransmissions was needed — every chunk it
  // marked was acknowledged before being resent, or its resend was reported
  // back as a duplicate TSN (the original had arrived).
  bool ep_active_ = false;
  uint32_t ep_exit_ = 0;
  size_t ep_undo_cwnd_ = 0, ep_undo_ssthresh_ = 0;
  int64_t ep_rtx_ = 0;  // TSNs retransmitted in the episode, less those reported back as duplicates
  std::unordered_set<uint32_t> ep_rtx_tsns_;  // this episode's retransmitted TSNs a duplicate report may undo
  bool dr_active_ = false, dr_limited_ = false;
  uint32_t dr_end_ = 0;
  uint64_t dr_start_us_ = 0, dr_bytes_ = 0;
  uint64_t dr_rates_[kDrRounds] = {};  // bytes per second
  int dr_next_ = 0;
  void dr_on_sack(uint32_t cum, size_t newly_acked, bool cwnd_limited, uint64_t now);
  void loss_response(bool random_loss, bool over_bdp, uint64_t now);
  size_t dr_bdp() const;
  // Short-path queue bound (queue_bound()): per round trip, the smallest RTT
  // sample minus the base RTT is the queue this association keeps standing
  // in front of itself (socket buffers, crypto lanes, the peer's reader).
  void queue_bound(uint32_t cum, uint64_t rtt_sample);
  uint32_t qb_end_ = 0;
  bool qb_active_ = false;
  uint64_t qb_min_ = UINT64_MAX, qb_last_ = 0;
  // The bound's base RTT: the smallest sample of the last 5-10 s (two 5 s
  // buckets), so a path whose base RTT rises (a route change, a peer that
  // moved) is not read as a standing queue forever.
  uint64_t qb_base_cur_ = UINT64_MAX, qb_base_prev_ = UINT64_MAX, qb_base_t0_ = 0;
  uint64_t interactive_until_us_ = 0;
  bool hs_done_ = false, hs_css_ = false, hs_round_ = false;
  int hs_samples_ = 0, hs_css_rounds_ = 0;
  uint32_t hs_window_end_ = 0;
  uint64_t hs_last_min_ = UINT64_MAX, hs_cur_min_ = UINT64_MAX, hs_css_base_ = 0;
  uint64_t last_loss_us_ = 0;
  uint64_t rto_us_;
  uint64_t srtt_us_ = 0, rttvar_us_ = 0;
  uint64_t min_rtt_us_ = 0;  // smallest RTT sample: the path's base RTT
  int assoc_errors_ = 0;
  bool retransmit_pending_ = false;

  // --- receiver
  bool peer_zero_checksum_ = false;  // peer advertised RFC 9653 EDMID 1
  bool have_peer_tsn_ = false;
  uint32_t peer_cum_tsn_ = 0;  // highest in-order TSN received
  uint32_t rx_high_tsn_ = 0;   // highest TSN received (stats: late arrivals)
  bool have_rx_high_ = false;
  std::map<uint32_t, InChunk*> ooo_;  // out-of-order (by TSN, serial order via custom cmp)
  size_t ooo_bytes_ = 0;
  std::vector<uint32_t> dups_;
  bool sack_needed_ = false;
  bool sack_urgent_ = false;
  int data_pkts_unacked_ = 0;
  uint64_t sack_timer_ = 0;
  struct Partial {
    uint32_t ppid = 0;
    RawBufPtr buf;  // pooled (reasm_pool_): a whole tunnel frame fits
    size_t len = 0;
    std::vector<uint8_t> big;  // only for messages beyond the pooled size
    std::vector<Bytes> frags;  // chained delivery: the fragments' views (no copy)
    size_t frag_bytes = 0;
    bool active = false;
    size_t size() const { return !frags.empty() ? frag_bytes : big.empty() ? len : big.size(); }
  };
  struct Held {  // a complete message waiting for its turn in its stream
    uint32_t ppid = 0;
    Bytes msg;
    std::vector<Bytes> more;
  };
  BufPool reasm_pool_{kReasmBuf, 256};
  static constexpr size_t kReasmBuf = 65536 + 1024;
  std::map<uint16_t, Partial> partial_;  // per-stream reassembly (ordered)
  std::map<uint16_t, Partial> partial_u_;  // unordered
  std::map<uint16_t, uint16_t> next_ssn_in_;      // per inbound stream: next SSN to deliver
  std::map<uint32_t, uint32_t> early_ready_;      // (stream, ssn) -> TSN of a complete message held out of order
  // Complete ordered messages that arrived in TSN order but ahead of their
  // stream's sequence (a peer may send a later small message of a stream
  // before an earlier large one: RFC 9260 orders by SSN, not TSN).
  std::map<uint32_t, Held> held_;  // (stream, ssn) -> message
  size_t held_bytes_ = 0;

  std::vector<std::vector<uint8_t>> ctrl_;  // control chunks to bundle at next flush
  bool shutdown_requested_ = false;
  bool closed_fired_ = false;
  uint32_t reconfig_seq_;
  SctpStats stats_;
  // gather assembly of the packet being built by flush()
  std::vector<uint8_t> pkt_;  // inline bytes; reserved so it never reallocates mid-packet
  std::vector<iovec> iov_;
  std::vector<const Bytes*> iov_own_;  // parallel to iov_
  size_t run_start_ = 0;      // start of the inline run not yet in iov_
  size_t pkt_len_ = 0;        // total packet bytes (inline + referenced)
};

}  // namespace p2pt::rtc
