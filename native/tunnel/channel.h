// MessageChannel: a reliable, ordered, message-oriented pipe between the two
// tunnel peers. This is the abstraction the roles (serve/proxy) run on; the
// reference hard-wires them to an Arc<RTCDataChannel> plus an unbounded mpsc
// of received messages (reference rtc.rs:23-28, :74-99).
//
// Implementations:
//   - rtc::DataChannel   (WebRTC SCTP/DTLS/ICE, the production transport)
//   - TcpMessageChannel  (length-prefixed frames over TCP; debug/bench
//                         transport selected by --transport tcp-listen:/tcp-connect:)
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/buf.h"
#include "core/net.h"
#include "core/reactor.h"
#include "proto/frame.h"

namespace p2pt {

class MessageChannel {
 public:
  virtual ~MessageChannel() = default;
  // Queue one message made of a small header and a payload view (gathered,
  // never concatenated by the caller). Returns false when the channel is closed.
  virtual bool send(const uint8_t* hdr, size_t hlen, const Bytes& payload) = 0;
  // The same for a latency-sensitive message (the frame scheduler's
  // interactive bypass: a token-sized frame of a stream with nothing queued):
  // a transport with a priority path may send it ahead of bulk messages it
  // holds unsent. Per-stream order is the transport's to keep.
  virtual bool send_urgent(const uint8_t* hdr, size_t hlen, const Bytes& payload) { return send(hdr, hlen, payload); }
  // Interactive traffic (a token-sized body frame) is flowing right now: a
  // transport may trade some bulk throughput for a shorter queue while it does.
  virtual void note_interactive() {}
  // Bytes accepted by send() but not yet handed to the network.
  virtual size_t buffered_amount() const = 0;
  virtual bool is_open() const = 0;
  virtual void close() = 0;
  virtual std::string describe() const = 0;
  // Largest REQ_BODY/RES_BODY payload per frame. The wire limit is 65408
  // (reference protocol.rs:10-12); a transport whose packets are smaller may
  // ask for frames that fit one packet so they are never fragmented/reassembled.
  virtual size_t body_chunk() const { return proto::kMaxBodyChunk; }
  // Identifies the secured channel for handshake proofs (psk extension): both
  // peers compute the same string. Empty when the transport has no such
  // identity (the TCP debug transport).
  virtual std::string channel_binding() const { return ""; }
  // How many bytes the transport can move per round trip right now (SCTP's
  // congestion window); 0 = unknown. The frame scheduler keeps only a
  // fraction of it queued in the channel, so on a slow path a token does
  // not wait behind a full 64 KiB of other streams' bodies.
  virtual size_t send_window_hint() const { return 0; }
  // The transport's base round-trip time (smallest sample) in microseconds;
  // 0 = unknown. "flow" receivers size their per-stream windows from it: the
  // path's bandwidth-delay product, not the queueing a bulk load adds.
  virtual uint64_t rtt_hint_us() const { return 0; }
  // The path's round-trip time as its connectivity checks measured it (no
  // transport ack delays in it); 0 = unknown. Falls back to rtt_hint_us().
  virtual uint64_t path_rtt_us() const { return rtt_hint_us(); }
  // Transport state for the send-path stall watchdog (empty: nothing to add).
  virtual std::string debug_state() const { return ""; }
  // "multistream" extension: spread the frames of tunnel stream ids over
  // `lanes` extra transport streams (SCTP streams delivered independently),
  // so a loss on one stream's packets does not hold back the others. Frames of
  // one tunnel stream always share a lane (their order is kept); stream 0
  // (control) stays on the channel's own stream. Transports without
  // independent streams ignore it.
  virtual void set_lanes(int lanes) { (void)lanes; }

  // Message arrived (whole message, zero-copy view where possible).
  std::function<void(Bytes)> on_message;
  // Optional: a message that arrived in fragments, as their views (first in
  // the Bytes, the rest in the vector, which the callee may take). Unset:
  // such a message reaches on_message as one copy.
  std::function<void(Bytes, std::vector<Bytes>&)> on_message_chain;
  // Hands a received message to the callbacks above.
  void deliver(Bytes msg, std::vector<Bytes>* more) {
    if (more && !more->empty()) {
      if (on_message_chain) {
        on_message_chain(std::move(msg), *more);
        return;
      }
      std::vector<uint8_t> v(msg.data(), msg.data() + msg.size());
      for (auto& b : *more) v.insert(v.end(), b.data(), b.data() + b.size());
      msg = Bytes::take(std::move(v));
    }
    if (on_message) on_message(std::move(msg));
  }
  // Channel became open (may already be open when handed out).
  std::function<void()> on_open;
  // Channel or the underlying connection failed / closed.
  std::function<void(const std::string&)> on_closed;
  // buffered_amount() fell to or below buffered_low_threshold.
  std::function<void()> on_buffered_low;
  size_t buffered_low_threshold = 64 * 1024;
};

// [u32 length][message] framing over a TcpConn.
class TcpMessageChannel : public MessageChannel, public std::enable_shared_from_this<TcpMessageChannel> {
 public:
  static std::shared_ptr<TcpMessageChannel> wrap(std::shared_ptr<TcpConn> c);
  bool send(const uint8_t* hdr, size_t hlen, const Bytes& payload) override;
  size_t buffered_amount() const override { return conn_ ? conn_->pending_out() : 0; }
  bool is_open() const override { return conn_ && !conn_->closed(); }
  void close() override;
  std::string describe() const override;

 private:
  void on_data(const uint8_t* p, size_t n);
  std::shared_ptr<TcpConn> conn_;
  uint8_t hdr_[4] = {};
  size_t hdr_len_ = 0;       // bytes of the length prefix read so far
  size_t need_ = 0;          // length of the message being assembled (0: none)
  std::vector<uint8_t> cur_;  // its bytes so far
};

}  // namespace p2pt
