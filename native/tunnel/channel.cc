#include "tunnel/channel.h"

#include <algorithm>
#include <cstring>

#include "core/log.h"

namespace p2pt {

static constexpr size_t kMaxTcpMessage = 16 * 1024 * 1024;

std::shared_ptr<TcpMessageChannel> TcpMessageChannel::wrap(std::shared_ptr<TcpConn> c) {
  auto ch = std::shared_ptr<TcpMessageChannel>(new TcpMessageChannel());
  ch->conn_ = std::move(c);
  std::weak_ptr<TcpMessageChannel> w = ch;
  ch->conn_->on_data([w](const uint8_t* p, size_t n) {
    if (auto s = w.lock()) s->on_data(p, n);
  });
  ch->conn_->on_close([w](const std::string& err) {
    if (auto s = w.lock()) {
      auto cb = s->on_closed;
      if (cb) cb(err.empty() ? "connection closed" : err);
    }
  });
  ch->conn_->on_drain(
      [w] {
        if (auto s = w.lock())
          if (s->on_buffered_low) s->on_buffered_low();
      },
      ch->buffered_low_threshold);
  return ch;
}

bool TcpMessageChannel::send(const uint8_t* hdr, size_t hlen, const Bytes& payload) {
  if (!is_open()) return false;
  uint8_t pre[4 + 16];
  size_t total = hlen + payload.size();
  wr32(pre, uint32_t(total));
  memcpy(pre + 4, hdr, hlen);
  conn_->write(Bytes::copy(pre, 4 + hlen));
  if (!payload.empty()) conn_->write(payload);
  return true;
}

// Messages wholly inside one read are delivered as views of the connection's
// receive buffer (zero-copy); a message split over reads is assembled once,
// straight into a buffer of its own size (it used to be copied into a staging
// vector and then again into the message: two copies per byte on the one
// thread that also runs the session).
void TcpMessageChannel::on_data(const uint8_t* p, size_t n) {
  auto self = shared_from_this();
  while (n) {
    if (need_ == 0) {  // reading the 4-byte length prefix
      while (n && hdr_len_ < 4) {
        hdr_[hdr_len_++] = *p++;
        n--;
      }
      if (hdr_len_ < 4) return;
      hdr_len_ = 0;
      const uint32_t len = rd32(hdr_);
      if (len > kMaxTcpMessage) {
        LOG_ERROR("tunnel::transport", "tcp transport: oversized message (%u bytes)", len);
        close();
        return;
      }
      if (len == 0) {
        if (on_message) on_message(Bytes());
        if (!conn_) return;
        continue;
      }
      if (n >= len) {  // whole message in this read
        Bytes msg = conn_ ? conn_->rx_view(p, len) : Bytes::copy(p, len);
        p += len;
        n -= len;
        if (on_message) on_message(std::move(msg));
        if (!conn_) return;
        continue;
      }
      need_ = len;
      cur_.clear();
      // Up front only what arrived plus a window's worth: the length prefix
      // alone must not make a peer's 16 MiB allocation (it grows as data does).
      cur_.reserve(std::min<size_t>(len, std::max<size_t>(n, 256 * 1024)));
    }
    const size_t take = std::min(n, need_ - cur_.size());
    cur_.insert(cur_.end(), p, p + take);
    p += take;
    n -= take;
    if (cur_.size() == need_) {
      need_ = 0;
      Bytes msg = Bytes::take(std::move(cur_));
      cur_ = std::vector<uint8_t>();
      if (on_message) on_message(std::move(msg));
      if (!conn_) return;
    }
  }
}

void TcpMessageChannel::close() {
  if (conn_) {
    auto c = conn_;
    c->on_close(nullptr);
    c->close();
  }
}

std::string TcpMessageChannel::describe() const {
  return conn_ ? "tcp:" + conn_->peer().str() : "tcp:closed";
}

}  // namespace p2pt
