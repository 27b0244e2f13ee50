#include "ws/ws.h"

#include <cstring>

#include "core/crypto.h"
#include "core/log.h"

namespace p2pt::ws {

static const char* kT = "tunnel::ws";

std::string encode_frame(Op op, std::string_view payload, bool mask, bool fin) {
  std::string out;
  out.reserve(payload.size() + 14);
  out.push_back(char((fin ? 0x80 : 0) | uint8_t(op)));
  uint8_t mbit = mask ? 0x80 : 0;
  size_t n = payload.size();
  if (n < 126) {
    out.push_back(char(mbit | n));
  } else if (n <= 0xFFFF) {
    out.push_back(char(mbit | 126));
    out.push_back(char(n >> 8));
    out.push_back(char(n));
  } else {
    out.push_back(char(mbit | 127));
    for (int i = 7; i >= 0; i--) out.push_back(char(uint64_t(n) >> (8 * i)));
  }
  if (mask) {
    uint8_t key[4];
    random_bytes(key, 4);
    out.append(reinterpret_cast<char*>(key), 4);
    size_t base = out.size();
    out.append(payload);
    for (size_t i = 0; i < n; i++) out[base + i] = char(out[base + i] ^ key[i & 3]);
  } else {
    out.append(payload);
  }
  return out;
}

std::string accept_key(std::string_view key) {
  std::string s(key);
  s += "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
  auto d = sha1(s.data(), s.size());
  return base64_encode(d.data(), d.size());
}

bool FrameParser::feed(const uint8_t* p, size_t n, const std::function<void(Op, bool, std::string&&)>& on_frame) {
  buf_.append(reinterpret_cast<const char*>(p), n);
  size_t off = 0;
  while (true) {
    size_t avail = buf_.size() - off;
    if (avail < 2) break;
    const uint8_t* b = reinterpret_cast<const uint8_t*>(buf_.data() + off);
    bool fin = b[0] & 0x80;
    if (b[0] & 0x70) {
      err_ = "reserved bits set";
      return false;
    }
    uint8_t opc = b[0] & 0x0F;
    bool masked = b[1] & 0x80;
    uint64_t len = b[1] & 0x7F;
    size_t hl = 2;
    if (len == 126) {
      if (avail < 4) break;
      len = uint64_t(b[2]) << 8 | b[3];
      hl = 4;
    } else if (len == 127) {
      if (avail < 10) break;
      len = 0;
      for (int i = 0; i < 8; i++) len = len << 8 | b[2 + i];
      hl = 10;
    }
    if (masked != expect_masked_) {
      err_ = expect_masked_ ? "client frame not masked" : "server frame masked";
      return false;
    }
    if (len > max_frame_) {
      err_ = "frame too large";
      return false;
    }
    if (opc >= 8 && (len > 125 || !fin)) {
      err_ = "invalid control frame";
      return false;
    }
    if (!(opc <= 2 || (opc >= 8 && opc <= 10))) {
      err_ = "unknown opcode";
      return false;
    }
    size_t mk = masked ? 4 : 0;
    if (avail < hl + mk + len) break;
    std::string payload(buf_.data() + off + hl + mk, size_t(len));
    if (masked) {
      const uint8_t* key = b + hl;
      for (size_t i = 0; i < payload.size(); i++) payload[i] = char(payload[i] ^ key[i & 3]);
    }
    off += hl + mk + size_t(len);
    on_frame(Op(opc), fin, std::move(payload));
  }
  buf_.erase(0, off);
  return true;
}

WsConn::WsConn(Reactor& r, std::shared_ptr<TcpConn> c, bool client)
    : r_(r), conn_(std::move(c)), client_(client), parser_(!client) {}

WsConn::~WsConn() {
  if (conn_) {
    conn_->on_close(nullptr);
    conn_->on_data(nullptr);
    conn_->close();
  }
}

void WsConn::wire() {
  std::weak_ptr<WsConn> w = shared_from_this();
  conn_->on_data([w](const uint8_t* p, size_t n) {
    if (auto s = w.lock()) s->on_data(p, n);
  });
  conn_->on_close([w](const std::string& err) {
    if (auto s = w.lock()) s->closed(err);
  });
}

void WsConn::on_data(const uint8_t* p, size_t n) {
  auto self = shared_from_this();
  bool ok = parser_.feed(p, n, [this](Op op, bool fin, std::string&& pl) { on_frame(op, fin, std::move(pl)); });
  if (!ok) {
    LOG_DEBUG(kT, "websocket protocol error: %s", parser_.error().c_str());
    if (conn_ && !conn_->closed()) {
      conn_->write(encode_frame(Op::Close, std::string("\x03\xea", 2), client_));
      conn_->close_after_flush();
    }
    closed("protocol error: " + parser_.error());
  }
}

void WsConn::on_frame(Op op, bool fin, std::string&& payload) {
  if (closed_fired_) return;
  switch (op) {
    case Op::Ping:
      if (conn_ && !close_sent_) conn_->write(encode_frame(Op::Pong, payload, client_));
      return;
    case Op::Pong:
      return;
    case Op::Close: {
      if (!close_sent_ && conn_) {
        std::string body = payload.size() >= 2 ? payload.substr(0, 2) : std::string();
        conn_->write(encode_frame(Op::Close, body, client_));
        close_sent_ = true;
      }
      if (conn_) conn_->close_after_flush();
      closed("");
      return;
    }
    case Op::Text:
    case Op::Binary:
      if (frag_op_ != Op::Cont) {
        closed("protocol error: new message inside fragmented message");
        return;
      }
      if (!fin) {
        frag_op_ = op;
        frag_ = std::move(payload);
        return;
      }
      break;
    case Op::Cont:
      if (frag_op_ == Op::Cont) {
        closed("protocol error: unexpected continuation");
        return;
      }
      frag_ += payload;
      if (!fin) return;
      op = frag_op_;
      payload = std::move(frag_);
      frag_.clear();
      frag_op_ = Op::Cont;
      break;
  }
  if (op == Op::Text) {
    if (on_text) on_text(std::move(payload));
  } else if (on_binary) {
    on_binary(std::move(payload));
  }
}

void WsConn::closed(const std::string& err) {
  if (closed_fired_) return;
  closed_fired_ = true;
  auto cb = std::move(on_closed);
  on_closed = nullptr;
  if (cb) cb(err);
}

void WsConn::send(Op op, std::string_view s) {
  if (!is_open()) return;
  conn_->write(encode_frame(op, s, client_));
}

void WsConn::send_text(std::string_view s) { send(Op::Text, s); }
void WsConn::send_binary(std::string_view s) { send(Op::Binary, s); }
void WsConn::ping(std::string_view s) { send(Op::Ping, s); }

void WsConn::close(uint16_t code, std::string_view reason) {
  if (!conn_ || conn_->closed() || close_sent_) return;
  std::string body;
  body.push_back(char(code >> 8));
  body.push_back(char(code));
  body.append(reason.substr(0, 123));
  conn_->write(encode_frame(Op::Close, body, client_));
  close_sent_ = true;
  conn_->close_after_flush();
}

struct WsConnectOp : std::enable_shared_from_this<WsConnectOp> {
  Reactor* r;
  http::Url url;
  std::string key;
  WsConn::ConnectCb cb;
  std::shared_ptr<TcpConn> conn;
  std::string buf;
  uint64_t timer = 0;
  bool done = false;

  void finish(std::shared_ptr<WsConn> ws, const std::string& err) {
    if (done) return;
    done = true;
    if (timer) r->cancel(timer);
    if (!ws && conn) {
      conn->on_close(nullptr);
      conn->close();
    }
    conn.reset();
    auto f = std::move(cb);
    f(std::move(ws), err);
  }
};

void WsConn::connect(Reactor& r, const std::string& url_s, ConnectCb cb, uint64_t timeout_ms) {
  auto op = std::make_shared<WsConnectOp>();
  op->r = &r;
  op->cb = std::move(cb);
  std::string err;
  if (!http::parse_url(url_s, op->url, &err) || (op->url.scheme != "ws" && op->url.scheme != "wss")) {
    if (err.empty()) err = "URL scheme not supported";
    r.post([op, err] { op->finish(nullptr, err); });
    return;
  }
  uint8_t k[16];
  random_bytes(k, 16);
  op->key = base64_encode(k, 16);
  std::weak_ptr<WsConnectOp> w = op;
  op->timer = r.call_later_ms(timeout_ms, [w] {
    if (auto o = w.lock()) {
      o->timer = 0;
      o->finish(nullptr, "websocket connect timed out");
    }
  });
  TcpConn::connect(r, op->url.host, op->url.port, op->url.tls(), [op](std::shared_ptr<TcpConn> c, std::string e) {
    if (op->done) {
      if (c) c->close();
      return;
    }
    if (!c) {
      op->finish(nullptr, e);
      return;
    }
    op->conn = c;
    std::string req = "GET " + op->url.path + " HTTP/1.1\r\nHost: " + op->url.host_header() +
                      "\r\nConnection: Upgrade\r\nUpgrade: websocket\r\nSec-WebSocket-Version: 13\r\n"
                      "Sec-WebSocket-Key: " + op->key + "\r\n\r\n";
    // The handshake callbacks own the op until the socket is handed to the
    // WsConn (wire() replaces them) or closed.
    c->on_close([op](const std::string& err) {
      op->finish(nullptr, "connection closed during handshake" + (err.empty() ? "" : ": " + err));
    });
    c->on_data([op](const uint8_t* p, size_t n) {
      auto o = op;
      if (o->done) return;
      o->buf.append(reinterpret_cast<const char*>(p), n);
      http::Head h;
      size_t used = 0;
      std::string perr;
      auto res = http::parse_response_head(o->buf, h, used, &perr);
      if (res == http::ParseResult::Incomplete) return;
      if (res == http::ParseResult::Error) {
        o->finish(nullptr, "invalid handshake response: " + perr);
        return;
      }
      if (h.status != 101) {
        o->finish(nullptr, "HTTP error: " + std::to_string(h.status) + " " + h.reason);
        return;
      }
      const std::string* acc = h.get("sec-websocket-accept");
      if (!acc || *acc != accept_key(o->key) || !h.has_token("upgrade", "websocket")) {
        o->finish(nullptr, "invalid websocket handshake (accept key mismatch)");
        return;
      }
      auto ws = std::shared_ptr<WsConn>(new WsConn(*o->r, o->conn, true));
      std::string rest = o->buf.substr(used);
      ws->wire();
      auto keep = ws;
      o->finish(ws, "");
      if (!rest.empty()) keep->on_data(reinterpret_cast<const uint8_t*>(rest.data()), rest.size());
    });
    c->write(std::move(req));
  });
}

std::shared_ptr<WsConn> WsConn::accept(Reactor& r, std::shared_ptr<TcpConn> c, const http::Head& head,
                                       std::string leftover) {
  const std::string* key = head.get("sec-websocket-key");
  const std::string* ver = head.get("sec-websocket-version");
  if (head.method != "GET" || !key || !head.has_token("upgrade", "websocket") ||
      !head.has_token("connection", "upgrade") || !ver || *ver != "13") {
    std::string body = "Bad Request";
    c->write("HTTP/1.1 400 Bad Request\r\nConnection: close\r\nContent-Length: " + std::to_string(body.size()) +
             "\r\n\r\n" + body);
    c->close_after_flush();
    return nullptr;
  }
  c->write("HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Accept: " +
           accept_key(*key) + "\r\n\r\n");
  auto ws = std::shared_ptr<WsConn>(new WsConn(r, std::move(c), false));
  ws->wire();
  if (!leftover.empty()) {
    auto w = std::weak_ptr<WsConn>(ws);
    r.post([w, leftover] {
      if (auto s = w.lock()) s->on_data(reinterpret_cast<const uint8_t*>(leftover.data()), leftover.size());
    });
  }
  return ws;
}

}  // namespace p2pt::ws
