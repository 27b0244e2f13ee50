// RFC 6455 WebSocket: frame codec, client handshake, server upgrade.
//
// Client side replaces tokio-tungstenite (reference signaling.rs:83-85,
// ws:// and wss://); server side replaces the Node `ws` package used by the
// signal server (reference signal-server/src/index.ts:93; its default
// maxPayload is 100 MiB, node_modules/ws/lib/websocket-server.js:68).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <string_view>

#include "core/net.h"
#include "http/http.h"

namespace p2pt::ws {

enum class Op : uint8_t { Cont = 0, Text = 1, Binary = 2, Close = 8, Ping = 9, Pong = 10 };

// Serialise one frame. Clients must mask (RFC 6455 §5.3).
std::string encode_frame(Op op, std::string_view payload, bool mask, bool fin = true);
// Sec-WebSocket-Accept for a Sec-WebSocket-Key.
std::string accept_key(std::string_view key);

// Incremental frame parser. on_frame(op, fin, payload) for each complete frame.
class FrameParser {
 public:
  explicit FrameParser(bool expect_masked, size_t max_frame = 100u << 20)
      : expect_masked_(expect_masked), max_frame_(max_frame) {}
  // Returns false on protocol error (see error()).
  bool feed(const uint8_t* p, size_t n, const std::function<void(Op, bool, std::string&&)>& on_frame);
  const std::string& error() const { return err_; }

 private:
  bool expect_masked_;
  size_t max_frame_;
  std::string buf_;
  std::string err_;
};

class WsConn : public std::enable_shared_from_this<WsConn> {
 public:
  using ConnectCb = std::function<void(std::shared_ptr<WsConn>, std::string err)>;
  // ws:// or wss:// URL. Performs the HTTP/1.1 upgrade handshake.
  static void connect(Reactor& r, const std::string& url, ConnectCb cb, uint64_t timeout_ms = 30000);
  // Server side: `head` is the parsed upgrade request; `leftover` is any data
  // read past it. Writes the 101 response (or 400 and returns nullptr).
  static std::shared_ptr<WsConn> accept(Reactor& r, std::shared_ptr<TcpConn> c, const http::Head& head,
                                        std::string leftover);

  ~WsConn();
  void send_text(std::string_view s);
  void send_binary(std::string_view s);
  void ping(std::string_view s = "");
  // Sends a close frame and closes after flush.
  void close(uint16_t code = 1000, std::string_view reason = "");
  bool is_open() const { return conn_ && !conn_->closed() && !close_sent_; }

  std::function<void(std::string&&)> on_text;
  std::function<void(std::string&&)> on_binary;
  // Fired once: clean close ("") or error text.
  std::function<void(const std::string&)> on_closed;

 private:
  WsConn(Reactor& r, std::shared_ptr<TcpConn> c, bool client);
  void wire();
  void on_data(const uint8_t* p, size_t n);
  void on_frame(Op op, bool fin, std::string&& payload);
  void closed(const std::string& err);
  void send(Op op, std::string_view s);

  Reactor& r_;
  std::shared_ptr<TcpConn> conn_;
  bool client_;
  FrameParser parser_;
  Op frag_op_ = Op::Cont;
  std::string frag_;
  bool close_sent_ = false;
  bool closed_fired_ = false;
  friend struct WsConnectOp;
};

}  // namespace p2pt::ws
