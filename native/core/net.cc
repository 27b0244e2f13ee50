#include "core/net.h"

#include <linux/sock_diag.h>

#include <arpa/inet.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/epoll.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <thread>

#include "core/log.h"

namespace p2pt {

uint64_t udp_socket_drops(int fd) {
#ifdef SO_MEMINFO
  uint32_t mi[SK_MEMINFO_VARS] = {};
  socklen_t l = sizeof mi;
  if (fd >= 0 && getsockopt(fd, SOL_SOCKET, SO_MEMINFO, mi, &l) == 0 && l > SK_MEMINFO_DROPS * sizeof(uint32_t))
    return mi[SK_MEMINFO_DROPS];
#endif
  return 0;
}

bool udp_socket_rmem(int fd, size_t* alloc, size_t* limit) {
#ifdef SO_MEMINFO
  uint32_t mi[SK_MEMINFO_VARS] = {};
  socklen_t l = sizeof mi;
  if (fd >= 0 && getsockopt(fd, SOL_SOCKET, SO_MEMINFO, mi, &l) == 0 && l > SK_MEMINFO_RCVBUF * sizeof(uint32_t)) {
    *alloc = mi[SK_MEMINFO_RMEM_ALLOC];
    *limit = mi[SK_MEMINFO_RCVBUF];
    return true;
  }
#endif
  return false;
}

size_t udp_socket_rcvbuf(int fd) {
  int v = 0;
  socklen_t l = sizeof v;
  if (fd < 0 || getsockopt(fd, SOL_SOCKET, SO_RCVBUF, &v, &l) != 0) return 0;
  return size_t(v);
}

size_t udp_socket_buffers(int fd, int bytes) {
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof bytes);
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof bytes);
  // The kernel doubles the request (bookkeeping overhead) and clamps it to
  // net.core.rmem_max / wmem_max first; a clamped buffer holds only a few
  // GSO-coalesced bursts, so try the privileged variants.
  if (udp_socket_rcvbuf(fd) < size_t(bytes)) setsockopt(fd, SOL_SOCKET, SO_RCVBUFFORCE, &bytes, sizeof bytes);
  int sb = 0;
  socklen_t l = sizeof sb;
  if (getsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sb, &l) == 0 && sb < bytes)
    setsockopt(fd, SOL_SOCKET, SO_SNDBUFFORCE, &bytes, sizeof bytes);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_RXQ_OVFL, &one, sizeof one);
  return udp_socket_rcvbuf(fd);
}

// ---------------------------------------------------------------- SockAddr

bool SockAddr::parse(const std::string& host_in, uint16_t port, SockAddr& out) {
  std::string host = host_in;
  if (host.size() >= 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  out = SockAddr{};
  auto* v4 = reinterpret_cast<sockaddr_in*>(&out.ss);
  if (inet_pton(AF_INET, host.c_str(), &v4->sin_addr) == 1) {
    v4->sin_family = AF_INET;
    v4->sin_port = htons(port);
    out.len = sizeof(sockaddr_in);
    return true;
  }
  auto* v6 = reinterpret_cast<sockaddr_in6*>(&out.ss);
  std::string h6 = host;
  size_t pct = h6.find('%');
  uint32_t scope = 0;
  if (pct != std::string::npos) {
    scope = if_nametoindex(h6.substr(pct + 1).c_str());
    h6 = h6.substr(0, pct);
  }
  if (inet_pton(AF_INET6, h6.c_str(), &v6->sin6_addr) == 1) {
    v6->sin6_family = AF_INET6;
    v6->sin6_port = htons(port);
    v6->sin6_scope_id = scope;
    out.len = sizeof(sockaddr_in6);
    return true;
  }
  return false;
}

bool SockAddr::parse_hostport(const std::string& hp, SockAddr& out) {
  size_t colon = hp.rfind(':');
  if (colon == std::string::npos) return false;
  std::string host = hp.substr(0, colon);
  int port = atoi(hp.c_str() + colon + 1);
  if (port < 0 || port > 65535) return false;
  if (host.empty()) host = "0.0.0.0";
  return parse(host, uint16_t(port), out);
}

uint16_t SockAddr::port() const {
  if (ss.ss_family == AF_INET) return ntohs(reinterpret_cast<const sockaddr_in*>(&ss)->sin_port);
  if (ss.ss_family == AF_INET6) return ntohs(reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_port);
  return 0;
}

void SockAddr::set_port(uint16_t p) {
  if (ss.ss_family == AF_INET) reinterpret_cast<sockaddr_in*>(&ss)->sin_port = htons(p);
  if (ss.ss_family == AF_INET6) reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port = htons(p);
}

std::string SockAddr::ip() const {
  char buf[INET6_ADDRSTRLEN] = {0};
  if (ss.ss_family == AF_INET)
    inet_ntop(AF_INET, &reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr, buf, sizeof buf);
  else if (ss.ss_family == AF_INET6)
    inet_ntop(AF_INET6, &reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_addr, buf, sizeof buf);
  return buf;
}

std::string SockAddr::str() const {
  if (ss.ss_family == AF_INET6) return "[" + ip() + "]:" + std::to_string(port());
  return ip() + ":" + std::to_string(port());
}

bool SockAddr::is_loopback() const {
  if (ss.ss_family == AF_INET)
    return (ntohl(reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr.s_addr) >> 24) == 127;
  if (ss.ss_family == AF_INET6) return IN6_IS_ADDR_LOOPBACK(&reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_addr);
  return false;
}

bool SockAddr::is_link_local() const {
  if (ss.ss_family == AF_INET)
    return (ntohl(reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr.s_addr) >> 16) == 0xA9FE;
  if (ss.ss_family == AF_INET6) return IN6_IS_ADDR_LINKLOCAL(&reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_addr);
  return false;
}

bool SockAddr::operator==(const SockAddr& o) const {
  if (ss.ss_family != o.ss.ss_family) return false;
  if (ss.ss_family == AF_INET) {
    auto a = reinterpret_cast<const sockaddr_in*>(&ss), b = reinterpret_cast<const sockaddr_in*>(&o.ss);
    return a->sin_port == b->sin_port && a->sin_addr.s_addr == b->sin_addr.s_addr;
  }
  if (ss.ss_family == AF_INET6) {
    auto a = reinterpret_cast<const sockaddr_in6*>(&ss), b = reinterpret_cast<const sockaddr_in6*>(&o.ss);
    return a->sin6_port == b->sin6_port && memcmp(&a->sin6_addr, &b->sin6_addr, 16) == 0;
  }
  return false;
}

std::vector<IfaceAddr> local_addresses(bool include_loopback, bool include_ipv6) {
  std::vector<IfaceAddr> out;
  ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return out;
  for (ifaddrs* p = ifa; p; p = p->ifa_next) {
    if (!p->ifa_addr || !(p->ifa_flags & IFF_UP)) continue;
    int fam = p->ifa_addr->sa_family;
    if (fam != AF_INET && !(include_ipv6 && fam == AF_INET6)) continue;
    IfaceAddr a;
    a.name = p->ifa_name;
    size_t sl = fam == AF_INET ? sizeof(sockaddr_in) : sizeof(sockaddr_in6);
    memcpy(&a.addr.ss, p->ifa_addr, sl);
    a.addr.len = socklen_t(sl);
    a.addr.set_port(0);
    if (a.addr.is_loopback() && !include_loopback) continue;
    if (a.addr.is_link_local()) continue;
    out.push_back(a);
  }
  freeifaddrs(ifa);
  return out;
}

void resolve_async(Reactor& r, const std::string& host, uint16_t port,
                   std::function<void(std::vector<SockAddr>, std::string)> cb) {
  SockAddr a;
  if (SockAddr::parse(host, port, a)) {
    r.post([cb, a] { cb({a}, ""); });
    return;
  }
  if (host == "localhost") {
    SockAddr v4;
    SockAddr::parse("127.0.0.1", port, v4);
    r.post([cb, v4] { cb({v4}, ""); });
    return;
  }
  // getaddrinfo blocks (offline DNS can take seconds): run it off-loop.
  Reactor* rp = &r;
  std::thread([rp, host, port, cb] {
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    std::vector<SockAddr> out;
    std::string err;
    if (rc != 0) {
      err = gai_strerror(rc);
    } else {
      for (addrinfo* p = res; p; p = p->ai_next) {
        SockAddr s;
        memcpy(&s.ss, p->ai_addr, p->ai_addrlen);
        s.len = p->ai_addrlen;
        out.push_back(s);
      }
      freeaddrinfo(res);
    }
    rp->post_threadsafe([cb, out, err] { cb(out, err); });
  }).detach();
}

int set_nonblocking(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  return fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

std::string errno_str(int e) { return strerror(e); }

SSL_CTX* tls_client_ctx() {
  static SSL_CTX* ctx = [] {
    SSL_CTX* c = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_default_verify_paths(c);
    SSL_CTX_set_verify(c, getenv("TUNNEL_TLS_INSECURE") ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
    SSL_CTX_set_min_proto_version(c, TLS1_2_VERSION);
    SSL_CTX_set_mode(c, SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER | SSL_MODE_ENABLE_PARTIAL_WRITE);
    return c;
  }();
  return ctx;
}

static std::string ssl_err_str() {
  unsigned long e = ERR_get_error();
  if (!e) return "tls error";
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  ERR_clear_error();
  return buf;
}

// ---------------------------------------------------------------- TcpConn

TcpConn::TcpConn(Reactor& r, int fd) : r_(r), fd_(fd) {
  sockaddr_storage ss{};
  socklen_t sl = sizeof ss;
  if (getpeername(fd, reinterpret_cast<sockaddr*>(&ss), &sl) == 0) {
    peer_.ss = ss;
    peer_.len = sl;
  }
}

TcpConn::~TcpConn() {
  if (fd_ >= 0) {
    r_.remove(fd_);
    ::close(fd_);
  }
  if (ssl_) SSL_free(ssl_);
}

std::shared_ptr<TcpConn> TcpConn::adopt(Reactor& r, int fd) {
  set_nonblocking(fd);
  std::shared_ptr<TcpConn> c(new TcpConn(r, fd));
  c->set_nodelay(true);
  std::weak_ptr<TcpConn> w = c;
  c->interest_ = EPOLLIN | EPOLLRDHUP;
  r.add(fd, c->interest_, [w](uint32_t ev) {
    if (auto s = w.lock()) s->on_events(ev);
  });
  return c;
}

void TcpConn::set_nodelay(bool on) {
  int v = on ? 1 : 0;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &v, sizeof v);
}

void TcpConn::update_interest() {
  if (fd_ < 0) return;
  uint32_t want = EPOLLRDHUP;
  if (!paused_ || handshaking_) want |= EPOLLIN;
  if (!out_.empty() || want_write_for_read_ || handshaking_) want |= EPOLLOUT;
  if (want != interest_) {
    interest_ = want;
    r_.modify(fd_, want);
  }
}

// After each batch of reads, TCP_QUICKACK on the socket (not sticky in
// Linux), so the ACKs and window updates for what was just consumed leave now
// instead of after the delayed-ACK timer: a flow-controlled reader (the proxy
// pausing an upload for credit) otherwise leaves the sender window-limited
// with a sub-MSS segment unacknowledged. On the MI355X host's 64 x 1 MB echo:
// +7 % (1200 MTU) and +10 % (jumbo) tunneled req/s (profiles/r04/qa19), and
// on top of one CPU per thread +21 % / +29 % over neither (pt20).

void TcpConn::on_events(uint32_t ev) {
  auto self = shared_from_this();
  if (handshaking_) {
    tls_handshake_step();
    return;
  }
  if (ev & EPOLLOUT) {
    if (want_write_for_read_) {
      want_write_for_read_ = false;
      do_read();
      if (fd_ < 0) return;
    }
    do_write();
    if (fd_ < 0) return;
  }
  if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
    if (!paused_ || (ev & (EPOLLHUP | EPOLLERR))) {
      // Bulk reads only: a token-sized read keeps the delayed ACK (one ACK
      // per SSE token would double the loopback packets of a node's streams).
      if (do_read() >= 16384 && fd_ >= 0 && !ssl_) {
        int one = 1;
        setsockopt(fd_, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof one);
      }
    }
  }
}

Bytes TcpConn::rx_view(const uint8_t* p, size_t n) const {
  constexpr size_t kMinView = 2048;  // smaller pieces are copied: never pin 64 KiB for a token
  if (rx_ && n >= kMinView && p >= rx_->data.get() && p + n <= rx_->data.get() + rx_->cap)
    return Bytes::adopt(rx_, p, n);
  return slab_copy(p, n);
}

size_t TcpConn::do_read() {
  constexpr size_t kRx = 65536;
  size_t total = 0;
  // Bounded number of reads per wakeup keeps the loop fair across sockets.
  for (int iter = 0; iter < 16 && fd_ >= 0 && !paused_; iter++) {
    if (!rx_ || rx_.use_count() > 1) {
      // Views of the previous buffer are still alive (body frames queued for
      // the channel, possibly on another thread): take a recycled one from
      // this thread's pool instead of allocating — and later freeing across
      // threads — 64 KiB per read.
      thread_local BufPool pool(kRx, 1024);
      rx_ = pool.get();
    } else {
      reuse_fence();  // the last view may have been dropped on another thread
    }
    uint8_t* buf = rx_->data.get();
    ssize_t n;
    if (ssl_) {
      ERR_clear_error();
      n = SSL_read(ssl_, buf, int(kRx));
      if (n <= 0) {
        int e = SSL_get_error(ssl_, int(n));
        if (e == SSL_ERROR_WANT_READ) return total;
        if (e == SSL_ERROR_WANT_WRITE) {
          want_write_for_read_ = true;
          update_interest();
          return total;
        }
        if (e == SSL_ERROR_ZERO_RETURN) {
          fail("");
          return total;
        }
        if (e == SSL_ERROR_SYSCALL && ERR_peek_error() == 0) {
          fail(errno ? errno_str(errno) : "");  // unexpected EOF
          return total;
        }
        fail(ssl_err_str());
        return total;
      }
    } else {
      n = ::read(fd_, buf, kRx);
      if (n < 0) {
        if (errno == EAGAIN || errno == EINTR) return total;
        fail(errno_str(errno));
        return total;
      }
      if (n == 0) {
        fail("");
        return total;
      }
    }
    total += size_t(n);
    if (auto cb = on_data_) (*cb)(buf, size_t(n));
    if (size_t(n) < kRx && !ssl_) return total;
  }
  return total;
}

void TcpConn::write(std::string s) {
  if (s.empty()) return;
  write(Bytes::copy(s));
}

void TcpConn::write(Bytes b) {
  if (fd_ < 0 || b.empty()) return;
  out_bytes_ += b.size();
  out_.push_back(std::move(b));
  // Writes issued while handling one reactor batch are coalesced into a single
  // writev at the end of the batch (e.g. chunk header + payload + CRLF of a
  // relayed SSE event go out as one syscall / one TCP segment).
  if (!write_scheduled_ && !handshaking_ && out_.size() == 1) {
    write_scheduled_ = true;
    std::weak_ptr<TcpConn> w = shared_from_this();
    r_.post([w] {
      if (auto s = w.lock()) {
        s->write_scheduled_ = false;
        s->do_write();
      }
    });
  } else if (!write_scheduled_) {
    update_interest();
  }
  if (low_water_ && out_bytes_ > low_water_) above_low_ = true;
}

void TcpConn::do_write() {
  while (fd_ >= 0 && !out_.empty() && !handshaking_) {
    ssize_t n;
    if (ssl_) {
      const Bytes& f = out_.front();
      ERR_clear_error();
      n = SSL_write(ssl_, f.data() + out_off_, int(f.size() - out_off_));
      if (n <= 0) {
        int e = SSL_get_error(ssl_, int(n));
        if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) break;
        fail(ssl_err_str());
        return;
      }
    } else {
      // Up to 512 pieces per writev: a body relayed as a chain of SCTP
      // fragment views (PcConfig::message_chains) is ~55 pieces per 64 KiB frame.
      constexpr int kIov = 512;
      iovec iov[kIov];
      int cnt = 0;
      size_t off = out_off_;
      for (auto it = out_.begin(); it != out_.end() && cnt < kIov; ++it) {
        iov[cnt].iov_base = const_cast<uint8_t*>(it->data() + off);
        iov[cnt].iov_len = it->size() - off;
        off = 0;
        cnt++;
      }
      n = ::writev(fd_, iov, cnt);
      if (n < 0) {
        if (errno == EAGAIN || errno == EINTR) break;
        fail(errno_str(errno));
        return;
      }
    }
    size_t left = size_t(n);
    out_bytes_ -= left;
    while (left) {
      size_t avail = out_.front().size() - out_off_;
      if (left >= avail) {
        left -= avail;
        out_.pop_front();
        out_off_ = 0;
      } else {
        out_off_ += left;
        left = 0;
      }
    }
  }
  if (fd_ < 0) return;
  update_interest();
  if (out_.empty() && close_after_flush_) {
    fail("");
    return;
  }
  if (above_low_ && out_bytes_ <= low_water_) {
    above_low_ = false;
    if (on_drain_) {
      auto self = shared_from_this();
      on_drain_();
    }
  }
}

void TcpConn::pause_reading() {
  if (paused_) return;
  paused_ = true;
  update_interest();
}

void TcpConn::resume_reading() {
  if (!paused_) return;
  paused_ = false;
  update_interest();
  // Data may already be buffered inside OpenSSL; poll once.
  if (ssl_ && SSL_pending(ssl_) > 0) {
    std::weak_ptr<TcpConn> w = shared_from_this();
    r_.post([w] {
      if (auto s = w.lock()) s->do_read();
    });
  }
}

void TcpConn::close_after_flush() {
  if (fd_ < 0) return;
  if (out_.empty()) close("");
  else close_after_flush_ = true;
}

void TcpConn::fail(const std::string& err) {
  if (in_write_) {
    std::weak_ptr<TcpConn> w = shared_from_this();
    r_.post([w, err] {
      if (auto s = w.lock()) s->close(err);
    });
    return;
  }
  close(err);
}

void TcpConn::close(const std::string& why) {
  if (fd_ < 0) return;
  auto keep = shared_from_this();
  if (ssl_ && why.empty()) SSL_shutdown(ssl_);
  r_.remove(fd_);
  ::close(fd_);
  fd_ = -1;
  out_.clear();
  out_bytes_ = 0;
  CloseFn cb = std::move(on_close_);
  on_close_ = nullptr;
  on_data_ = nullptr;
  on_drain_ = nullptr;
  if (cb) cb(why);
}

int TcpConn::release_fd() {
  if (fd_ < 0 || ssl_ || out_bytes_ || in_write_) return -1;
  r_.remove(fd_);
  int fd = fd_;
  fd_ = -1;
  out_.clear();
  on_close_ = nullptr;
  on_data_ = nullptr;
  on_drain_ = nullptr;
  return fd;
}

void TcpConn::tls_handshake_step() {
  ERR_clear_error();
  int rc = SSL_connect(ssl_);
  if (rc == 1) {
    handshaking_ = false;
    update_interest();
    auto cb = std::move(handshake_cb_);
    if (cb) cb("");
    return;
  }
  int e = SSL_get_error(ssl_, rc);
  if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) {
    update_interest();
    return;
  }
  std::string err = "TLS handshake failed: " + ssl_err_str();
  long vr = SSL_get_verify_result(ssl_);
  if (vr != X509_V_OK) err += std::string(" (") + X509_verify_cert_error_string(vr) + ")";
  handshaking_ = false;
  auto cb = std::move(handshake_cb_);
  close(err);
  if (cb) cb(err);
}

struct ConnectOp : std::enable_shared_from_this<ConnectOp> {
  Reactor* r;
  std::string host;
  uint16_t port;
  bool tls;
  std::function<void(std::shared_ptr<TcpConn>, std::string)> cb;
  std::vector<SockAddr> addrs;
  size_t idx = 0;
  int fd = -1;
  Reactor::TimerId timer = 0;
  bool done = false;
  std::string last_err;

  void finish(std::shared_ptr<TcpConn> c, const std::string& err) {
    if (done) return;
    done = true;
    if (timer) r->cancel(timer);
    if (fd >= 0) {
      r->remove(fd);
      ::close(fd);
      fd = -1;
    }
    auto f = std::move(cb);
    f(std::move(c), err);
  }

  void try_next() {
    if (done) return;
    if (idx >= addrs.size()) {
      finish(nullptr, last_err.empty() ? "connection failed" : last_err);
      return;
    }
    const SockAddr& a = addrs[idx++];
    fd = ::socket(a.family(), SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) {
      last_err = errno_str(errno);
      try_next();
      return;
    }
    int rc = ::connect(fd, a.sa(), a.len);
    if (rc == 0) {
      connected();
      return;
    }
    if (errno != EINPROGRESS) {
      last_err = "connect " + a.str() + ": " + errno_str(errno);
      ::close(fd);
      fd = -1;
      try_next();
      return;
    }
    auto self = shared_from_this();
    r->add(fd, EPOLLOUT, [self, a](uint32_t) {
      int err = 0;
      socklen_t sl = sizeof err;
      getsockopt(self->fd, SOL_SOCKET, SO_ERROR, &err, &sl);
      self->r->remove(self->fd);
      if (err) {
        self->last_err = "connect " + a.str() + ": " + errno_str(err);
        ::close(self->fd);
        self->fd = -1;
        self->try_next();
      } else {
        self->connected();
      }
    });
  }

  void connected() {
    int cfd = fd;
    fd = -1;
    r->remove(cfd);
    auto conn = TcpConn::adopt(*r, cfd);
    if (!tls) {
      finish(conn, "");
      return;
    }
    conn->ssl_ = SSL_new(tls_client_ctx());
    SSL_set_fd(conn->ssl_, cfd);
    SockAddr dummy;
    if (SockAddr::parse(host, 0, dummy)) {
      // IP literal: no SNI (RFC 6066 §3); the certificate must carry it as an IP SAN.
      X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(conn->ssl_), host.c_str());
    } else {
      SSL_set_tlsext_host_name(conn->ssl_, host.c_str());
      SSL_set1_host(conn->ssl_, host.c_str());
    }
    conn->handshaking_ = true;
    auto self = shared_from_this();
    conn->handshake_cb_ = [self, conn](std::string err) {
      if (err.empty()) self->finish(conn, "");
      else self->finish(nullptr, err);
    };
    conn->update_interest();
    conn->tls_handshake_step();
  }
};

void TcpConn::connect(Reactor& r, const std::string& host, uint16_t port, bool tls,
                      std::function<void(std::shared_ptr<TcpConn>, std::string)> cb, uint64_t timeout_ms) {
  auto op = std::make_shared<ConnectOp>();
  op->r = &r;
  op->host = host;
  op->port = port;
  op->tls = tls;
  op->cb = std::move(cb);
  std::weak_ptr<ConnectOp> w = op;
  op->timer = r.call_later_ms(timeout_ms, [w] {
    if (auto o = w.lock()) {
      o->timer = 0;
      o->finish(nullptr, "connect timed out");
    }
  });
  resolve_async(r, host, port, [op](std::vector<SockAddr> addrs, std::string err) {
    if (op->done) return;
    if (addrs.empty()) {
      op->finish(nullptr, "resolve " + op->host + ": " + err);
      return;
    }
    op->addrs = std::move(addrs);
    op->try_next();
  });
}

// ---------------------------------------------------------------- TcpListener

TcpListener::TcpListener(Reactor& r, int fd, AcceptFn cb) : r_(r), fd_(fd), cb_(std::move(cb)) {
  r_.add(fd_, EPOLLIN, [this](uint32_t) {
    for (int i = 0; i < 64; i++) {
      sockaddr_storage ss{};
      socklen_t sl = sizeof ss;
      int c = accept4(fd_, reinterpret_cast<sockaddr*>(&ss), &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (c < 0) {
        if (errno == EAGAIN || errno == EINTR) return;
        if (errno == EMFILE || errno == ENFILE) {
          LOG_WARN("tunnel::net", "accept: %s", strerror(errno));
          return;
        }
        return;
      }
      SockAddr p;
      p.ss = ss;
      p.len = sl;
      cb_(c, p);
    }
  });
}

TcpListener::~TcpListener() {
  r_.remove(fd_);
  ::close(fd_);
}

std::unique_ptr<TcpListener> TcpListener::bind(Reactor& r, const std::string& hostport, AcceptFn cb,
                                               std::string* err) {
  SockAddr a;
  if (!SockAddr::parse_hostport(hostport, a)) {
    if (err) *err = "invalid socket address syntax: " + hostport;
    return nullptr;
  }
  int fd = ::socket(a.family(), SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    if (err) *err = errno_str(errno);
    return nullptr;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (::bind(fd, a.sa(), a.len) < 0 || ::listen(fd, 1024) < 0) {
    if (err) *err = "bind " + hostport + ": " + errno_str(errno);
    ::close(fd);
    return nullptr;
  }
  return std::unique_ptr<TcpListener>(new TcpListener(r, fd, std::move(cb)));
}

SockAddr TcpListener::local_addr() const {
  SockAddr a;
  a.len = sizeof a.ss;
  getsockname(fd_, a.sa(), &a.len);
  return a;
}

}  // namespace p2pt
