// Sockets: addresses, non-blocking TCP connections (optionally TLS), TCP
// listeners, async name resolution and local interface enumeration.
//
// TcpConn is the byte-stream used by the HTTP server (proxy side, reference
// proxy.rs:175-220 via hyper), the HTTP client (serve side, reference
// serve.rs:187-294 via reqwest) and the WebSocket client/server (reference
// signaling.rs:80-151 via tokio-tungstenite; signal-server/src/index.ts:93).
#pragma once

#include <netinet/in.h>
#include <sys/socket.h>

#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/buf.h"
#include "core/reactor.h"

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace p2pt {

struct SockAddr {
  sockaddr_storage ss{};
  socklen_t len = 0;

  static bool parse(const std::string& host, uint16_t port, SockAddr& out);  // numeric only
  // "1.2.3.4:80", "[::1]:80"
  static bool parse_hostport(const std::string& hp, SockAddr& out);
  int family() const { return ss.ss_family; }
  uint16_t port() const;
  void set_port(uint16_t p);
  std::string ip() const;
  std::string str() const;  // ip:port / [ip]:port
  bool is_loopback() const;
  bool is_link_local() const;
  const sockaddr* sa() const { return reinterpret_cast<const sockaddr*>(&ss); }
  sockaddr* sa() { return reinterpret_cast<sockaddr*>(&ss); }
  bool operator==(const SockAddr& o) const;
  bool operator!=(const SockAddr& o) const { return !(*this == o); }
};

// UDP socket receive-side accounting (Linux SO_MEMINFO): datagrams dropped
// because the receive buffer was full (sk_drops, what SO_RXQ_OVFL reports per
// datagram) and the effective receive buffer size. 0 when unavailable.
uint64_t udp_socket_drops(int fd);
size_t udp_socket_rcvbuf(int fd);
// Bytes (truesize) queued in the socket's receive buffer, and its limit.
bool udp_socket_rmem(int fd, size_t* alloc, size_t* limit);
// Sets SO_RCVBUF / SO_SNDBUF to `bytes`, retrying with the *FORCE variants
// (CAP_NET_ADMIN) when net.core.[rw]mem_max clamps the request, and enables
// SO_RXQ_OVFL. Returns the effective receive buffer.
size_t udp_socket_buffers(int fd, int bytes);

struct IfaceAddr {
  std::string name;
  SockAddr addr;
};
// Up, non-tentative interface addresses (IPv4 + global/ULA IPv6).
std::vector<IfaceAddr> local_addresses(bool include_loopback, bool include_ipv6);

// Resolve host asynchronously (numeric hosts resolve inline). Callback runs on
// the reactor thread with an empty vector on failure.
void resolve_async(Reactor& r, const std::string& host, uint16_t port,
                   std::function<void(std::vector<SockAddr>, std::string err)> cb);

int set_nonblocking(int fd);
std::string errno_str(int e);

// Shared TLS client context (system trust store, hostname verification).
SSL_CTX* tls_client_ctx();

class TcpConn : public std::enable_shared_from_this<TcpConn> {
 public:
  using DataFn = std::function<void(const uint8_t*, size_t)>;
  using CloseFn = std::function<void(const std::string& err)>;  // empty err == clean EOF

  // Wrap an accepted / already-connected fd.
  static std::shared_ptr<TcpConn> adopt(Reactor& r, int fd);
  // Async connect (resolves, connects, optional TLS with SNI + verification).
  static void connect(Reactor& r, const std::string& host, uint16_t port, bool tls,
                      std::function<void(std::shared_ptr<TcpConn>, std::string err)> cb,
                      uint64_t timeout_ms = 30000);

  ~TcpConn();

  // The callback may replace itself (e.g. an HTTP upgrade handing the socket
  // to a WebSocket): it is held by shared_ptr and pinned during each call.
  void on_data(DataFn f) { on_data_ = f ? std::make_shared<DataFn>(std::move(f)) : nullptr; }
  void on_close(CloseFn f) { on_close_ = std::move(f); }
  // Fires when the output buffer drains below `low_water` after having been above it.
  void on_drain(Fn f, size_t low_water = 0) {
    on_drain_ = std::move(f);
    low_water_ = low_water;
  }

  void write(Bytes b);
  void write(std::string s);
  void write(const void* p, size_t n) { write(Bytes::copy(p, n)); }
  size_t pending_out() const { return out_bytes_; }
  void pause_reading();
  void resume_reading();
  bool reading_paused() const { return paused_; }
  // Close after all pending output is written.
  void close_after_flush();
  // Immediate close (RST semantics not forced). Fires on_close("") if not yet closed.
  void close(const std::string& why = "");
  bool closed() const { return fd_ < 0; }
  // Hands the socket over (another reactor adopts it): deregistered, not
  // closed, no callbacks fire. Only for a plain-TCP connection with nothing
  // left to write; -1 otherwise (the connection is unchanged).
  int release_fd();
  int fd() const { return fd_; }
  SockAddr peer() const { return peer_; }
  void set_nodelay(bool on);
  // Inside an on_data callback: a Bytes for [p, p+n). Large ranges of the
  // receive buffer become zero-copy views (the next read then uses a fresh
  // buffer); small ones, and bytes from anywhere else, are copied.
  Bytes rx_view(const uint8_t* p, size_t n) const;

 private:
  TcpConn(Reactor& r, int fd);
  void on_events(uint32_t ev);
  size_t do_read();  // bytes read
  void do_write();
  void update_interest();
  void fail(const std::string& err);
  void tls_handshake_step();

  Reactor& r_;
  int fd_;
  SockAddr peer_;
  SSL* ssl_ = nullptr;
  bool handshaking_ = false;
  std::function<void(std::string)> handshake_cb_;
  bool want_write_for_read_ = false;
  bool paused_ = false;
  bool close_after_flush_ = false;
  bool in_write_ = false;
  bool write_scheduled_ = false;
  std::deque<Bytes> out_;
  size_t out_off_ = 0;
  size_t out_bytes_ = 0;
  bool above_low_ = false;
  size_t low_water_ = 0;
  std::shared_ptr<DataFn> on_data_;
  RawBufPtr rx_;  // receive buffer; replaced when views into it are alive
  CloseFn on_close_;
  Fn on_drain_;
  uint32_t interest_ = 0;
  friend struct ConnectOp;
};

class TcpListener {
 public:
  using AcceptFn = std::function<void(int fd, SockAddr peer)>;
  // host:port; port 0 picks an ephemeral port (see local_addr()).
  static std::unique_ptr<TcpListener> bind(Reactor& r, const std::string& hostport, AcceptFn cb,
                                           std::string* err);
  ~TcpListener();
  SockAddr local_addr() const;
  int fd() const { return fd_; }

 private:
  TcpListener(Reactor& r, int fd, AcceptFn cb);
  Reactor& r_;
  int fd_;
  AcceptFn cb_;
};

}  // namespace p2pt
