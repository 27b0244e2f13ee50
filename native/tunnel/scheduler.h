// Fair frame scheduler in front of the single ordered message channel.
//
// The reference writes every frame straight into the data channel with no
// back-pressure (reference serve.rs:274, proxy.rs:324), so
// a 1 MB body queued ahead of an SSE token delays that token by the whole
// body. Here frames wait in per-stream FIFOs and are released into the channel
// only while its buffered amount is below a window, in this order:
//
//   1. control frames (stream 0: HELLO/AGREE/PING/PONG; CREDIT of any stream);
//   2. the "interactive" lane: streams with little queued (<= kInteractive
//      bytes, e.g. an SSE stream with its next token), one frame per turn;
//   3. the bulk lane: backlogged streams. A stream's first kFifoBytes go out
//      oldest stream first (lowest id; ids are handed out in arrival order):
//      with round-robin, 64 concurrent 1 MB uploads all finished together at
//      the very end, so the upstream of a store-and-forward hop idled until
//      then; served in order, each completes in turn and the next hop starts
//      on it while the rest are still in transit. Past kFifoBytes a stream
//      goes round-robin, one frame per turn, so a long transfer never holds
//      the others back for longer than that. The round-robin lane is never
//      starved by a steady arrival of new streams: after kBulkShareBytes of
//      oldest-first frames it gets one frame (about a fifth of the bytes while
//      both lanes are backlogged).
//
// So a token waits for at most the channel window plus one frame, never for
// other streams' queued bodies. Per-stream FIFO order is preserved (the wire
// format is unchanged: frames of one stream never reorder). Per-stream queue
// sizes are exposed so producers can pause just the streams that are over
// their budget instead of everyone.
#pragma once

#include <cstdlib>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <unordered_map>
#include <unordered_set>

#include "proto/frame.h"
#include "tunnel/channel.h"

namespace p2pt {

class FrameScheduler {
 public:
  static constexpr size_t kInteractive = 4096;
  static constexpr uint64_t kBulkSent = 256 * 1024;  // a stream past this is bulk, not interactive
  static constexpr uint64_t kFifoBytes = 2u << 20;
  static constexpr uint64_t kBulkShareBytes = 256 * 1024;  // oldest-first bytes per guaranteed round-robin frame

  explicit FrameScheduler(std::shared_ptr<MessageChannel> ch, size_t window = 64 * 1024);
  ~FrameScheduler();

  void send(proto::Frame f);
  // Bytes held here plus bytes buffered in the channel.
  size_t pending_bytes() const { return queued_ + (ch_ ? ch_->buffered_amount() : 0); }
  bool bypass_ = true;  // the interactive bypass (tests turn it off to compare)
  uint64_t bypassed_ = 0;  // frames sent through the interactive bypass
  std::map<uint32_t, uint32_t> small_;  // small body frames sent through the bypass, per stream
  std::unordered_set<uint64_t> traced_;  // TUNNEL_TRACE: (stream, kind) whose first body frame was stamped
  size_t queued_bytes() const { return queued_; }
  // Send-path stall watchdog, called about once a second: true when frames
  // or channel bytes are waiting and neither moved since the previous call.
  bool stalled_tick();
  std::string debug_state() const;
  // Bytes of `sid` held in the scheduler (not yet handed to the channel).
  size_t stream_queued(uint32_t sid) const {
    auto it = streams_.find(sid);
    return it == streams_.end() ? 0 : it->second.bytes;
  }
  // Global watermarks: `cb` fires when pending_bytes() drops to `low` after
  // having exceeded `high`.
  void set_watermarks(size_t high, size_t low, std::function<void()> cb);
  bool over_high() const { return pending_bytes() > high_; }
  // Fires after a pump that released frames (producers re-check paused streams).
  std::function<void()> on_progress;
  void pump();
  MessageChannel* channel() const { return ch_.get(); }
  size_t body_chunk() const { return ch_ ? ch_->body_chunk() : proto::kMaxBodyChunk; }
  // Bytes kept queued in the channel: the configured window, or a quarter of
  // the transport's congestion window when that is smaller (at least 2 KiB),
  // so queued bulk ahead of a token stays below ~1/4 round trip of sending.
  size_t window() const {
    size_t h = ch_ ? ch_->send_window_hint() : 0;
    return h ? std::min(window_, std::max<size_t>(2048, h / 4)) : window_;
  }

 private:
  struct StreamQ {
    std::deque<proto::Frame> q;
    size_t bytes = 0;
    uint64_t sent = 0;  // bytes released so far (attained service)
    bool listed = false;
  };
  bool emit(const proto::Frame& f, bool urgent = false);
  void list(uint32_t sid, StreamQ& s);
  bool pop_from(std::deque<uint32_t>& lane);
  bool pop_fifo();
  static bool last_frame(const proto::Frame& f);
  void remember(const proto::Frame& f);
  static constexpr size_t kRemember = 4096;  // streams whose attained service is kept while their queue is empty
  bool release(uint32_t sid, StreamQ& s, std::unordered_map<uint32_t, StreamQ>::iterator it);

  std::shared_ptr<MessageChannel> ch_;
  size_t window_;
  std::deque<proto::Frame> control_;
  std::unordered_map<uint32_t, StreamQ> streams_;
  std::deque<uint32_t> interactive_, bulk_;
  std::set<uint32_t> fifo_;  // bulk streams within their first kFifoBytes, oldest (lowest id) first
  std::map<uint32_t, uint64_t> sent_;  // attained service of open streams whose queue ran dry
  size_t queued_ = 0;
  size_t released_ = 0;   // wire bytes of the last frame release() handed to the channel
  uint64_t fifo_run_ = 0;  // oldest-first bytes released since the round-robin lane last had a turn
  uint64_t emitted_ = 0;  // frames handed to the channel
  uint64_t wd_emitted_ = 0;
  size_t wd_buffered_ = 0;
  size_t high_ = SIZE_MAX, low_ = 0;
  bool was_high_ = false;
  std::function<void()> low_cb_;
  bool pumping_ = false;
};

}  // namespace p2pt
