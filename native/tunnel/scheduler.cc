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

bool FrameScheduler::emit(const proto::Frame& f, bool urgent) {
  uint8_t hdr[proto::kHeaderLen];
  f.header(hdr);
  // Trace: a stream's first body frame and its end frame leave the scheduler
  // for the channel (serve sends RES_*, the proxy REQ_*).
  if (trace::enabled()) {
    if (traced_.size() >= (1u << 16)) traced_.clear();  // bounded on long traced runs
    const uint64_t key = uint64_t(f.stream_id) << 8;
    switch (f.type) {
      case proto::MsgType::ResBody:
        if (traced_.insert(key | 1).second) {
          trace::event("serve", f.stream_id, "chan_tx");
          trace::mark_tx("serve", f.stream_id);
        }
        break;
      case proto::MsgType::ReqHeaders:
        trace::mark_tx("proxy", f.stream_id);
        break;
      case proto::MsgType::ReqBody:
        if (traced_.insert(key | 2).second) trace::event("proxy", f.stream_id, "chan_tx");
        break;
      case proto::MsgType::ResEnd: trace::event("serve", f.stream_id, "chan_end"); break;
      case proto::MsgType::ReqEnd: trace::event("proxy", f.stream_id, "chan_end"); break;
      default: break;
    }
  }
  metrics::frame_sent(uint8_t(f.type), f.wire_size());
  emitted_++;
  return urgent ? ch_->send_urgent(hdr, sizeof hdr, f.payload) : ch_->send(hdr, sizeof hdr, f.payload);
}

bool FrameScheduler::stalled_tick() {
  const size_t buffered = ch_ ? ch_->buffered_amount() : 0;
  const bool waiting = queued_ > 0 || buffered > 0;
  const bool stalled = waiting && emitted_ == wd_emitted_ && buffered == wd_buffered_;
  wd_emitted_ = emitted_;
  wd_buffered_ = buffered;
  return stalled;
}

std::string FrameScheduler::debug_state() const {
  std::string s = "sched{queued=" + std::to_string(queued_) + " control=" + std::to_string(control_.size()) +
                  " interactive=" + std::to_string(interactive_.size()) + " fifo=" + std::to_string(fifo_.size()) +
                  " bulk=" + std::to_string(bulk_.size()) +
                  " streams=" + std::to_string(streams_.size()) + " window=" + std::to_string(window()) +
                  " emitted=" + std::to_string(emitted_) + " pumping=" + std::to_string(int(pumping_)) + "} ";
  return s + (ch_ ? ch_->debug_state() : "");
}

void FrameScheduler::list(uint32_t sid, StreamQ& s) {
  s.listed = true;
  if (s.bytes <= kInteractive) interactive_.push_back(sid);
  else if (s.sent < kFifoBytes) fifo_.insert(sid);
  else bulk_.push_back(sid);
}

void FrameScheduler::send(proto::Frame f) {
  if (!ch_ || !ch_->is_open()) return;
  // Fast path: nothing queued and the channel has room. The channel's
  // low-water mark follows the (adaptive) window so the pump is woken again.
  size_t win = window();
  ch_->buffered_low_threshold = win / 2;
  const size_t buffered = ch_->buffered_amount();
  if (queued_ == 0 && buffered < win) {
    if (f.stream_id && f.type != proto::MsgType::Credit) remember(f);
    emit(f);
    if (pending_bytes() > high_) was_high_ = true;
    return;
  }
  // Interactive bypass: a token-sized frame of a stream with nothing queued
  // here goes straight to the channel even while bulk keeps it over its
  // window. Queued behind the window, the first SSE token next to 8 bulk
  // downloads waited 0.4 ms p50 in this scheduler alone (ttft_breakdown
  // --bulk 8: serve sched_in -> chan_tx). Bounded: past 4 windows of unsent
  // bytes the frame queues as before, so a stream of small frames cannot
  // flood the association.
  if (f.stream_id && f.type != proto::MsgType::Credit && f.wire_size() <= kInteractive && buffered < 4 * win &&
      bypass_) {
    auto it = streams_.find(f.stream_id);
    if (it == streams_.end() || it->second.q.empty()) {
      // A small body frame of a stream that has not moved bulk is a token
      // (headers and end frames, and the short last body frame of a 1 MB
      // upload, take this path too but say nothing about interactivity).
      // Evidence is a stream's second small body frame: a bulk response's
      // first read from its upstream is often small too, and counting it kept
      // the tighter bound on through a 64 x 1 MB echo.
      // Only a token takes the transport's priority path: headers and end
      // frames of bulk streams gain nothing from it (advice r3).
      bool token = false;
      if (f.type == proto::MsgType::ResBody || f.type == proto::MsgType::ReqBody) {
        auto sv = sent_.find(f.stream_id);
        if ((sv == sent_.end() || sv->second < kBulkSent) && ++small_[f.stream_id] >= 2) {
          ch_->note_interactive();
          token = true;
        }
        if (small_.size() > kRemember) small_.erase(small_.begin());
      } else if (last_frame(f) && !small_.empty()) {
        small_.erase(f.stream_id);
      }
      emit(f, token);
      bypassed_++;
      return;
    }
  }
  size_t sz = f.wire_size();
  queued_ += sz;
  if (f.stream_id == 0 || f.type == proto::MsgType::Credit) {  // credit is cumulative: no ordering with data
    control_.push_back(std::move(f));
  } else {
    uint32_t sid = f.stream_id;
    auto [it, fresh] = streams_.try_emplace(sid);
    auto& s = it->second;
    if (fresh) {  // a stream that emptied its queue before keeps its attained service
      auto sv = sent_.find(sid);
      if (sv != sent_.end()) {
        s.sent = sv->second;
        sent_.erase(sv);
      }
    }
    s.q.push_back(std::move(f));
    s.bytes += sz;
    if (!s.listed) list(sid, s);
  }
  if (pending_bytes() > high_) was_high_ = true;
  pump();
}

bool FrameScheduler::last_frame(const proto::Frame& f) {
  return f.type == proto::MsgType::ReqEnd || f.type == proto::MsgType::ResEnd || f.type == proto::MsgType::Error ||
         f.type == proto::MsgType::Cancel;
}

// A frame sent on the fast path (nothing queued) counts toward its stream's
// attained service too; small frames are left out (they decide nothing and
// an SSE token should not pay a map update).
void FrameScheduler::remember(const proto::Frame& f) {
  if (last_frame(f)) {
    if (!sent_.empty()) sent_.erase(f.stream_id);
    if (!small_.empty()) small_.erase(f.stream_id);
  } else if (f.wire_size() > kInteractive) {
    sent_[f.stream_id] += f.wire_size();
    if (sent_.size() > kRemember) sent_.erase(sent_.begin());
  }
}

// Releases the head frame of a listed stream; false if its queue was empty.
bool FrameScheduler::release(uint32_t sid, StreamQ& s, std::unordered_map<uint32_t, StreamQ>::iterator it) {
  s.listed = false;
  if (s.q.empty()) {
    streams_.erase(it);
    return false;
  }
  proto::Frame f = std::move(s.q.front());
  s.q.pop_front();
  size_t sz = f.wire_size();
  s.bytes -= sz;
  s.sent += sz;
  queued_ -= sz;
  released_ = sz;
  if (s.q.empty()) {
    if (!last_frame(f)) {  // attained service outlives an empty queue while the stream may still produce
      sent_[sid] = s.sent;
      if (sent_.size() > kRemember) sent_.erase(sent_.begin());
    }
    streams_.erase(it);
  } else {
    list(sid, s);  // re-queued behind the others, in the lane its backlog now calls for
  }
  emit(f);
  return true;
}

// Releases the head frame of the first stream in `lane`; false if the lane is empty.
bool FrameScheduler::pop_from(std::deque<uint32_t>& lane) {
  while (!lane.empty()) {
    uint32_t sid = lane.front();
    lane.pop_front();
    auto it = streams_.find(sid);
    if (it == streams_.end()) continue;
    if (release(sid, it->second, it)) return true;
  }
  return false;
}

// The oldest bulk stream still within its first kFifoBytes.
bool FrameScheduler::pop_fifo() {
  while (!fifo_.empty()) {
    uint32_t sid = *fifo_.begin();
    fifo_.erase(fifo_.begin());
    auto it = streams_.find(sid);
    if (it == streams_.end()) continue;
    if (release(sid, it->second, it)) return true;
  }
  return false;
}

void FrameScheduler::pump() {
  if (pumping_ || !ch_) return;
  pumping_ = true;
  bool progressed = false;
  size_t win = window();
  ch_->buffered_low_threshold = win / 2;
  while (ch_->is_open() && queued_ && ch_->buffered_amount() < win) {
    if (!control_.empty()) {
      proto::Frame f = std::move(control_.front());
      control_.pop_front();
      queued_ -= f.wire_size();
      emit(f);
      progressed = true;
      continue;
    }
    if (pop_from(interactive_)) {
      progressed = true;
      continue;
    }
    // The round-robin lane's guaranteed share: without it a transfer past
    // kFifoBytes got no turn while newer streams kept the oldest-first lane
    // busy (a steady load of 1 MB requests starved a large download).
    if (fifo_run_ >= kBulkShareBytes && pop_from(bulk_)) {
      fifo_run_ = 0;
      progressed = true;
      continue;
    }
    const bool rr_waiting = !bulk_.empty();
    if (pop_fifo()) {
      fifo_run_ = rr_waiting ? fifo_run_ + released_ : 0;  // the share accrues while round-robin waits
      progressed = true;
      continue;
    }
    if (pop_from(bulk_)) {
      fifo_run_ = 0;
      progressed = true;
      continue;
    }
    break;
  }
  pumping_ = false;
  if (was_high_ && pending_bytes() <= low_) {
    was_high_ = false;
    if (low_cb_) low_cb_();
  }
  if (progressed && on_progress) on_progress();
}

}  // namespace p2pt
