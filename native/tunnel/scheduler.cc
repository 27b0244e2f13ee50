#include "tunnel/scheduler.h"

#include "tunnel/metrics.h"

namespace p2pt {

FrameScheduler::FrameScheduler(std::shared_ptr<MessageChannel> ch, size_t window)
    : ch_(std::move(ch)), window_(window) {
  ch_->buffered_low_threshold = window_ / 2;
}

FrameScheduler::~FrameScheduler() = default;

void FrameScheduler::set_watermarks(size_t high, size_t low, std::function<void()> cb) {
  high_ = high;
  low_ = low;
  low_cb_ = std::move(cb);
}

bool FrameScheduler::emit(const proto::Frame& f) {
  uint8_t hdr[proto::kHeaderLen];
  f.header(hdr);
  metrics::frame_sent(uint8_t(f.type), f.wire_size());
  return ch_->send(hdr, sizeof hdr, f.payload);
}

void FrameScheduler::send(proto::Frame f) {
  if (!ch_ || !ch_->is_open()) return;
  // Fast path: nothing queued and the channel has room.
  if (queued_ == 0 && ch_->buffered_amount() < window_) {
    emit(f);
    if (pending_bytes() > high_) was_high_ = true;
    return;
  }
  queued_ += f.wire_size();
  if (f.stream_id == 0) {
    control_.push_back(std::move(f));
  } else {
    auto& q = streams_[f.stream_id];
    if (q.empty()) rr_.push_back(f.stream_id);
    q.push_back(std::move(f));
  }
  if (pending_bytes() > high_) was_high_ = true;
  pump();
}

void FrameScheduler::pump() {
  if (pumping_ || !ch_) return;
  pumping_ = true;
  while (ch_->is_open() && queued_ && ch_->buffered_amount() < window_) {
    if (!control_.empty()) {
      proto::Frame f = std::move(control_.front());
      control_.pop_front();
      queued_ -= f.wire_size();
      emit(f);
      continue;
    }
    if (rr_.empty()) break;
    uint32_t sid = rr_.front();
    rr_.pop_front();
    auto it = streams_.find(sid);
    if (it == streams_.end() || it->second.empty()) continue;
    proto::Frame f = std::move(it->second.front());
    it->second.pop_front();
    queued_ -= f.wire_size();
    if (it->second.empty()) streams_.erase(it);
    else rr_.push_back(sid);
    emit(f);
  }
  pumping_ = false;
  if (was_high_ && pending_bytes() <= low_) {
    was_high_ = false;
    if (low_cb_) low_cb_();
  }
}

}  // namespace p2pt
