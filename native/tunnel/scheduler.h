// Fair frame scheduler in front of the single ordered message channel.
//
// The reference writes every frame straight into the data channel with no
// back-pressure (reference serve.rs:274, proxy.rs:324), so
// a 1 MB body queued ahead of an SSE token delays that token by the whole
// body. Here frames wait in per-stream FIFOs and are released round-robin
// (one frame per stream per turn, control frames first) only while the
// channel's buffered amount is below a window. Head-of-line delay for a
// token is therefore bounded by the window, not by other streams' bodies.
// Wire format is unchanged: per-stream frame order is preserved.
#pragma once

#include <deque>
#include <functional>
#include <memory>
#include <unordered_map>

#include "proto/frame.h"
#include "tunnel/channel.h"

namespace p2pt {

class FrameScheduler {
 public:
  explicit FrameScheduler(std::shared_ptr<MessageChannel> ch, size_t window = 64 * 1024);
  ~FrameScheduler();

  // Stream 0 frames (HELLO/AGREE/PING/PONG) are control frames and jump the queue.
  void send(proto::Frame f);
  // Bytes held here plus bytes buffered in the channel.
  size_t pending_bytes() const { return queued_ + (ch_ ? ch_->buffered_amount() : 0); }
  size_t queued_bytes() const { return queued_; }
  // Back-pressure hook: `cb` fires when pending_bytes() drops below `low`
  // after having exceeded `high`. Producers pause when pending_bytes() > high.
  void set_watermarks(size_t high, size_t low, std::function<void()> cb);
  bool over_high() const { return pending_bytes() > high_; }
  void pump();
  MessageChannel* channel() const { return ch_.get(); }
  size_t body_chunk() const { return ch_ ? ch_->body_chunk() : proto::kMaxBodyChunk; }

 private:
  bool emit(const proto::Frame& f);
  std::shared_ptr<MessageChannel> ch_;
  size_t window_;
  std::deque<proto::Frame> control_;
  std::unordered_map<uint32_t, std::deque<proto::Frame>> streams_;
  std::deque<uint32_t> rr_;
  size_t queued_ = 0;
  size_t high_ = SIZE_MAX, low_ = 0;
  bool was_high_ = false;
  std::function<void()> low_cb_;
  bool pumping_ = false;
};

}  // namespace p2pt
