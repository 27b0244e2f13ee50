#include "tunnel/channel.h"

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

void TcpMessageChannel::on_data(const uint8_t* p, size_t n) {
  inbuf_.insert(inbuf_.end(), p, p + n);
  auto self = shared_from_this();
  while (inbuf_.size() - inoff_ >= 4) {
    uint32_t len = rd32(inbuf_.data() + inoff_);
    if (len > kMaxTcpMessage) {
      LOG_ERROR("tunnel::transport", "tcp transport: oversized message (%u bytes)", len);
      close();
      return;
    }
    if (inbuf_.size() - inoff_ < 4 + size_t(len)) break;
    Bytes msg = Bytes::copy(inbuf_.data() + inoff_ + 4, len);
    inoff_ += 4 + len;
    if (on_message) on_message(std::move(msg));
    if (!conn_) return;
  }
  if (inoff_ == inbuf_.size()) {
    inbuf_.clear();
    inoff_ = 0;
  } else if (inoff_ > 1 << 20) {
    inbuf_.erase(inbuf_.begin(), inbuf_.begin() + long(inoff_));
    inoff_ = 0;
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
