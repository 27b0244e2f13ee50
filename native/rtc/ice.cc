#include "rtc/ice.h"

#include "tunnel/metrics.h"

#include <netinet/udp.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <sstream>

#include "core/crypto.h"
#include "core/log.h"
#include "rtc/turn.h"

namespace p2pt::rtc {

static const char* kT = "tunnel::ice";

// ---------------------------------------------------------------- Candidate

uint32_t candidate_priority(const std::string& type, uint32_t local_pref, int component) {
  uint32_t tp = type == "host" ? 126 : type == "prflx" ? 110 : type == "srflx" ? 100 : 0;
  return (tp << 24) | ((local_pref & 0xFFFF) << 8) | uint32_t(256 - component);
}

std::string Candidate::to_sdp() const {
  std::ostringstream o;
  o << "candidate:" << foundation << " " << component << " " << transport << " " << priority << " " << addr.ip()
    << " " << addr.port() << " typ " << type;
  if (has_related) o << " raddr " << related.ip() << " rport " << related.port();
  return o.str();
}

bool Candidate::parse(const std::string& s_in, Candidate& out, std::string* err) {
  std::string s = s_in;
  if (s.rfind("a=", 0) == 0) s = s.substr(2);
  if (s.rfind("candidate:", 0) == 0) s = s.substr(10);
  std::istringstream in(s);
  std::vector<std::string> tok;
  std::string t;
  while (in >> t) tok.push_back(t);
  if (tok.size() < 8 || tok[6] != "typ") {
    if (err) *err = "malformed candidate: " + s_in;
    return false;
  }
  out = Candidate{};
  out.foundation = tok[0];
  out.component = atoi(tok[1].c_str());
  std::string tr = tok[2];
  for (auto& c : tr) c = char(tolower(c));
  out.transport = tr;
  if (tr != "udp") {
    if (err) *err = "unsupported candidate transport: " + tok[2];
    return false;
  }
  out.priority = uint32_t(strtoul(tok[3].c_str(), nullptr, 10));
  int port = atoi(tok[5].c_str());
  if (!SockAddr::parse(tok[4], uint16_t(port), out.addr)) {
    if (err) *err = "unresolvable candidate address (mDNS?): " + tok[4];
    return false;
  }
  out.type = tok[7];
  for (size_t i = 8; i + 1 < tok.size(); i += 2) {
    if (tok[i] == "raddr") {
      int rport = 0;
      if (i + 3 < tok.size() && tok[i + 2] == "rport") rport = atoi(tok[i + 3].c_str());
      out.has_related = SockAddr::parse(tok[i + 1], uint16_t(rport), out.related);
    }
  }
  return true;
}

const char* ice_state_name(IceState s) {
  switch (s) {
    case IceState::New: return "new";
    case IceState::Checking: return "checking";
    case IceState::Connected: return "connected";
    case IceState::Disconnected: return "disconnected";
    case IceState::Failed: return "failed";
    case IceState::Closed: return "closed";
  }
  return "?";
}

// ---------------------------------------------------------------- agent

std::shared_ptr<IceAgent> IceAgent::create(Reactor& r, IceConfig cfg, bool controlling) {
  return std::shared_ptr<IceAgent>(new IceAgent(r, std::move(cfg), controlling));
}

IceAgent::IceAgent(Reactor& r, IceConfig cfg, bool controlling)
    : r_(r), cfg_(std::move(cfg)), controlling_(controlling), tiebreaker_(random_u64()) {
  ufrag_ = random_ice_chars(16);
  pwd_ = random_ice_chars(32);
  rxpool_.resize(32);
  if (const char* e = getenv("TUNNEL_NAT")) {
    std::string m = e;
    nat_mode_ = m == "port-restricted" ? 1 : m == "symmetric" ? 2 : 0;
    if (nat_mode_) LOG_INFO(kT, "NAT emulation: %s", m.c_str());
  }
}

IceAgent::~IceAgent() { close(); }

void IceAgent::close() {
  if (closed_) return;
  closed_ = true;
  if (tick_timer_) r_.cancel(tick_timer_);
  tick_timer_ = 0;
  if (flush_hook_) r_.remove_flush_hook(flush_hook_);
  flush_hook_ = 0;
  if (turn_) turn_->close();
  turn_.reset();
  for (auto& s : socks_) {
    if (s.fd >= 0) {
      r_.remove(s.fd);
      ::close(s.fd);
      s.fd = -1;
    }
  }
  for (auto& np : nat_ports_) {
    if (np.fd >= 0) {
      r_.remove(np.fd);
      ::close(np.fd);
      np.fd = -1;
    }
  }
  if (nat_mode_) LOG_INFO(kT, "NAT emulation: %llu inbound datagrams filtered", (unsigned long long)nat_dropped_);
  state_ = IceState::Closed;
}

void IceAgent::set_state(IceState s) {
  if (s == state_) return;
  state_ = s;
  LOG_DEBUG(kT, "ICE state: %s", ice_state_name(s));
  if (on_state) {
    auto cb = on_state;
    cb(s);
  }
}

bool udp_offload_enabled(const char* which) {
  const char* e = getenv("TUNNEL_UDP_OFFLOAD");
  if (!e) return true;
  const std::string list = std::string(",") + e + ",";
  return list.find(std::string(",") + which + ",") != std::string::npos;
}

void IceAgent::enable_gro(int fd) {
  int one = 1;
  // Traced runs: kernel receive timestamps (the udp_kernel hop of a frame).
  if (trace::enabled()) setsockopt(fd, SOL_SOCKET, SO_TIMESTAMPNS, &one, sizeof one);
  if (!udp_offload_enabled("gro")) return;
  if (setsockopt(fd, SOL_UDP, UDP_GRO, &one, sizeof one) == 0) gro_enabled_ = true;
}

size_t IceAgent::gro_segment(const msghdr* mh) {
  for (cmsghdr* c = CMSG_FIRSTHDR(const_cast<msghdr*>(mh)); c; c = CMSG_NXTHDR(const_cast<msghdr*>(mh), c)) {
    if (c->cmsg_level == SOL_UDP && c->cmsg_type == UDP_GRO) {
      int v = 0;
      memcpy(&v, CMSG_DATA(c), sizeof v);
      return v > 0 ? size_t(v) : 0;
    }
  }
  return 0;
}

uint64_t IceAgent::rx_overflow() const {
  uint64_t n = 0;
  for (auto& s : socks_) n += udp_socket_drops(s.fd);
  for (auto& np : nat_ports_) n += udp_socket_drops(np.fd);
  return n;
}

size_t IceAgent::rcvbuf_bytes() const {
  if (sel_local_ < 0 || sel_local_ >= int(locals_.size())) return 0;
  const int si = locals_[size_t(sel_local_)].sock;
  return si >= 0 && si < int(socks_.size()) ? udp_socket_rcvbuf(socks_[size_t(si)].fd) : 0;
}

void IceAgent::open_sockets() {
  auto addrs = local_addresses(cfg_.include_loopback, cfg_.include_ipv6 || cfg_.ipv6_only);
  if (cfg_.ipv6_only)
    addrs.erase(std::remove_if(addrs.begin(), addrs.end(), [](const IfaceAddr& a) { return a.addr.family() != AF_INET6; }),
                addrs.end());
  // Non-loopback first so they get the higher local preference.
  std::stable_sort(addrs.begin(), addrs.end(),
                   [](const IfaceAddr& a, const IfaceAddr& b) { return !a.addr.is_loopback() && b.addr.is_loopback(); });
  std::weak_ptr<IceAgent> w = shared_from_this();
  for (auto& ia : addrs) {
    int fd = ::socket(ia.addr.family(), SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) continue;
    if (ia.addr.family() == AF_INET6) {
      int one = 1;
      setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &one, sizeof one);
    }
    const char* kb = getenv("TUNNEL_UDP_BUF_KB");  // tests / A-B: the socket buffers asked for (default 4 MiB)
    const size_t rb = udp_socket_buffers(fd, kb && *kb ? std::max(16, atoi(kb)) * 1024 : 4 << 20);
    LOG_DEBUG(kT, "UDP socket %s: receive buffer %zu bytes", ia.addr.str().c_str(), rb);
    enable_gro(fd);
    SockAddr a = ia.addr;
    a.set_port(0);
    if (::bind(fd, a.sa(), a.len) < 0) {
      ::close(fd);
      continue;
    }
    SockAddr bound;
    bound.len = sizeof bound.ss;
    getsockname(fd, bound.sa(), &bound.len);
    Sock s;
    s.fd = fd;
    s.addr = bound;
    s.loopback = bound.is_loopback();
    int si = int(socks_.size());
    socks_.push_back(s);
    r_.add(fd, EPOLLIN, [w, si](uint32_t) {
      if (auto self = w.lock()) self->on_readable(si);
    });
  }
}

void IceAgent::add_local(Candidate c, int sock, bool relay) {
  locals_.push_back(Local{c, sock, relay});
  if (cfg_.relay_only && !relay) return;  // kept as a socket base, never advertised or paired
  local_cands_.push_back(c);
  int li = int(locals_.size()) - 1;
  for (int ri = 0; ri < int(remotes_.size()); ri++) pair_up(li, ri);
  LOG_DEBUG(kT, "local candidate: %s", c.to_sdp().c_str());
  if (on_candidate) on_candidate(c);
}

void IceAgent::gather() {
  if (gather_started_ || closed_) return;
  gather_started_ = true;
  open_sockets();
  if (cfg_.auto_flush) flush_hook_ = r_.add_flush_hook([this] { flush(); });
  uint32_t pref = 65535;
  for (int si = 0; si < int(socks_.size()); si++) {
    Candidate c;
    c.type = "host";
    c.addr = socks_[si].addr;
    c.priority = candidate_priority("host", pref);
    pref -= 256;
    c.foundation = std::to_string(crc32_ieee(("host" + c.addr.ip()).data(), 4 + c.addr.ip().size()));
    add_local(c, si, false);
  }
  if (socks_.empty()) LOG_WARN(kT, "no usable network interfaces for ICE");
  start_srflx();
  start_relay();
  std::weak_ptr<IceAgent> w = shared_from_this();
  tick_timer_ = r_.call_later_ms(20, [w] {
    if (auto s = w.lock()) {
      s->tick_timer_ = 0;
      s->tick();
    }
  });
  maybe_gathering_done();
}

static bool parse_server_url(const std::string& url, std::string& host, uint16_t& port, uint16_t dflt) {
  std::string s = url;
  size_t colon = s.find(':');
  if (colon == std::string::npos) return false;
  s = s.substr(colon + 1);  // strip scheme
  if (s.rfind("//", 0) == 0) s = s.substr(2);
  size_t q = s.find('?');
  if (q != std::string::npos) s = s.substr(0, q);
  port = dflt;
  if (!s.empty() && s[0] == '[') {
    size_t rb = s.find(']');
    if (rb == std::string::npos) return false;
    host = s.substr(1, rb - 1);
    if (rb + 1 < s.size() && s[rb + 1] == ':') port = uint16_t(atoi(s.c_str() + rb + 2));
    return true;
  }
  size_t pc = s.rfind(':');
  if (pc != std::string::npos) {
    host = s.substr(0, pc);
    port = uint16_t(atoi(s.c_str() + pc + 1));
  } else {
    host = s;
  }
  return !host.empty();
}

void IceAgent::start_srflx() {
  std::weak_ptr<IceAgent> w = shared_from_this();
  for (auto& url : cfg_.stun_urls) {
    std::string host;
    uint16_t port;
    if (!parse_server_url(url, host, port, 3478)) {
      LOG_WARN(kT, "ignoring invalid STUN URL %s", url.c_str());
      continue;
    }
    pending_gather_++;
    // Bound the whole srflx attempt (DNS included) so gathering can finish
    // offline without waiting for the resolver; it closes earlier once every
    // request to this server has been answered.
    auto win = std::make_shared<SrflxWindow>();
    r_.call_later_ms(cfg_.stun_timeout_ms, [w, win] {
      if (auto s = w.lock()) s->srflx_window_done(win);
    });
    resolve_async(r_, host, port, [w, win, url](std::vector<SockAddr> addrs, std::string err) {
      auto s = w.lock();
      if (!s || win->done) return;
      if (addrs.empty()) {
        LOG_DEBUG(kT, "STUN server %s unresolvable: %s", url.c_str(), err.c_str());
        s->srflx_window_done(win);
        return;
      }
      for (int si = 0; si < int(s->socks_.size()); si++) {
        if (s->socks_[si].loopback) continue;
        for (auto& a : addrs) {
          if (a.family() != s->socks_[si].addr.family()) continue;
          auto m = stun::Message::make(stun::kBindingRequest);
          SrflxReq rq{si, a, m.tid_key(), 1, win};
          auto bytes = m.serialize(nullptr, true);
          s->send_raw(-1 - si, a, bytes.data(), bytes.size());
          s->srflx_.push_back(rq);
          win->outstanding++;
          break;
        }
      }
      // Responses are matched in handle_response.
      if (win->outstanding == 0) s->srflx_window_done(win);
    });
  }
}

void IceAgent::srflx_window_done(const std::shared_ptr<SrflxWindow>& win) {
  if (win->done) return;
  win->done = true;
  pending_gather_--;
  maybe_gathering_done();
}

void IceAgent::start_relay() {
  if (cfg_.turn_url.empty()) return;
  TurnUrl url;
  std::string err;
  if (!TurnClient::parse_url(cfg_.turn_url, url, &err)) {
    LOG_ERROR(kT, "%s", err.c_str());  // the CLI refuses such URLs before any session
    return;
  }
  // A loopback TURN server (tests, same-host relays) is reached from the
  // loopback socket; anything else from the first routable IPv4 socket.
  // (Over TCP/TLS the socket is only the relayed candidate's base.)
  SockAddr probe;
  bool server_loopback = SockAddr::parse(url.host, url.port, probe) && probe.is_loopback();
  int si = -1;
  for (int i = 0; i < int(socks_.size()); i++)
    if (socks_[i].loopback == server_loopback && socks_[i].addr.family() == AF_INET) {
      si = i;
      break;
    }
  if (si < 0) {
    LOG_WARN(kT, "TURN: no suitable IPv4 socket to allocate from");
    return;
  }
  pending_gather_++;
  std::weak_ptr<IceAgent> w = shared_from_this();
  turn_ = TurnClient::create(r_, this, si, url, cfg_.turn_user, cfg_.turn_pass,
                             [w, si](bool ok, const SockAddr& relayed, const SockAddr& mapped) {
                               auto s = w.lock();
                               if (!s) return;
                               if (ok) {
                                 Candidate c;
                                 c.type = "relay";
                                 c.addr = relayed;
                                 c.related = mapped;
                                 c.has_related = true;
                                 c.priority = candidate_priority("relay", 65535);
                                 c.foundation = std::to_string(
                                     crc32_ieee(("relay" + relayed.ip()).data(), 5 + relayed.ip().size()));
                                 s->add_local(c, si, true);
                               }
                               s->pending_gather_--;
                               s->maybe_gathering_done();
                             });
}

void IceAgent::maybe_gathering_done() {
  if (gathering_done_ || pending_gather_ > 0) return;
  gathering_done_ = true;
  LOG_DEBUG(kT, "ICE gathering complete (%zu local candidates)", local_cands_.size());
  if (on_gathering_done) {
    auto cb = on_gathering_done;
    std::weak_ptr<IceAgent> w = shared_from_this();
    r_.post([w, cb] {
      if (w.lock()) cb();
    });
  }
}

void IceAgent::kick() {
  // Run the check scheduler now instead of waiting for the next pacing tick.
  if (closed_ || !gather_started_ || state_ == IceState::Failed) return;
  if (tick_timer_) r_.cancel(tick_timer_);
  std::weak_ptr<IceAgent> w = shared_from_this();
  tick_timer_ = r_.call_later_us(0, [w] {
    if (auto s = w.lock()) {
      s->tick_timer_ = 0;
      s->tick();
    }
  });
}

void IceAgent::set_remote_credentials(const std::string& ufrag, const std::string& pwd) {
  remote_ufrag_ = ufrag;
  remote_pwd_ = pwd;
  if (state_ == IceState::New) {
    checking_since_ = Reactor::now_ms();
    set_state(IceState::Checking);
  }
  kick();
}

int IceAgent::find_remote(const SockAddr& a) const {
  for (int i = 0; i < int(remotes_.size()); i++)
    if (remotes_[i].addr == a) return i;
  return -1;
}

void IceAgent::add_remote_candidate(const Candidate& c) {
  if (closed_ || c.component != 1) return;
  if (find_remote(c.addr) >= 0) return;
  remotes_.push_back(c);
  int ri = int(remotes_.size()) - 1;
  LOG_DEBUG(kT, "remote candidate: %s", c.to_sdp().c_str());
  for (int li = 0; li < int(locals_.size()); li++) pair_up(li, ri);
  if (state_ == IceState::New && !remote_pwd_.empty()) {
    checking_since_ = Reactor::now_ms();
    set_state(IceState::Checking);
  }
  if (!remote_pwd_.empty() && sel_pair_ < 0) kick();
}

uint64_t IceAgent::pair_priority(const Local& l, const Candidate& r) const {
  uint64_t g = controlling_ ? l.c.priority : r.priority;
  uint64_t d = controlling_ ? r.priority : l.c.priority;
  return (std::min(g, d) << 32) + 2 * std::max(g, d) + (g > d ? 1 : 0);
}

void IceAgent::pair_up(int li, int ri) {
  const Local& l = locals_[li];
  const Candidate& rc = remotes_[ri];
  if (l.c.type == "srflx") return;  // checks run from the base (host) candidate
  if (cfg_.relay_only && !l.relay) return;
  SockAddr laddr = l.relay ? l.c.addr : socks_[l.sock].addr;
  if (laddr.family() != rc.addr.family()) return;
  // Loopback sockets only talk to loopback remotes and vice versa.
  if (!l.relay && socks_[l.sock].loopback != rc.addr.is_loopback()) return;
  add_pair(li, ri);
}

int IceAgent::add_pair(int li, int ri) {
  for (int pi = 0; pi < int(pairs_.size()); pi++)
    if (pairs_[pi].local == li && pairs_[pi].remote == ri) return pi;
  const Local& l = locals_[li];
  const Candidate& rc = remotes_[ri];
  Pair p;
  p.local = li;
  p.remote = ri;
  p.prio = pair_priority(l, rc);
  pairs_.push_back(p);
  if (l.relay && turn_) turn_->permit(rc.addr);
  return int(pairs_.size()) - 1;
}

void IceAgent::send_raw(int local_idx, const SockAddr& to, const uint8_t* p, size_t n) {
  Out o;
  o.local = local_idx;
  o.to = to;
  if (!spare_.empty()) {
    o.data = std::move(spare_.back());
    spare_.pop_back();
  }
  o.data.assign(p, p + n);
  outq_.push_back(std::move(o));
}

uint8_t* IceAgent::reserve_append(size_t max) {
  if (sel_local_ < 0 || closed_) {
    drop_.resize(max);
    append_at_ = SIZE_MAX;
    return drop_.data();
  }
  if (!outq_.empty()) {
    Out& b = outq_.back();
    if (b.coalesce && b.local == sel_local_ && b.to == sel_remote_ && b.data.size() + max <= coalesce_limit_) {
      append_at_ = b.data.size();
      b.data.resize(append_at_ + max);
      return b.data.data() + append_at_;
    }
  }
  Out o;
  o.local = sel_local_;
  o.to = sel_remote_;
  o.coalesce = coalesce_limit_ > 0 && !locals_[sel_local_].relay;
  if (!spare_.empty()) {
    o.data = std::move(spare_.back());
    spare_.pop_back();
  }
  o.data.reserve(std::max(coalesce_limit_, max));
  o.data.resize(max);
  outq_.push_back(std::move(o));
  append_at_ = 0;
  return outq_.back().data.data();
}

void IceAgent::commit_append(size_t used) {
  if (append_at_ == SIZE_MAX || outq_.empty()) return;
  outq_.back().data.resize(append_at_ + used);
}

void IceAgent::send(const uint8_t* p, size_t n) {
  if (sel_local_ < 0 || closed_) return;
  send_raw(sel_local_, sel_remote_, p, n);
}

// Test-only fault injection on the datagram path (SURVEY §4.2 "fault
// injection"), one switch: TUNNEL_FAULT="key=value,..." with
//   drop (alias loss), dup   probabilities per outbound datagram;
//   delay_ms                 a uniform random extra delay (which also reorders);
//     STUN (connectivity checks) is exempt from those so the path still comes up;
//   blackhole=START:LEN      (ms) drops every outbound datagram, STUN included,
//     in that window after the first send (a path that dies and comes back).
// WAN emulation (order-preserving, every datagram): rtt_ms adds half the
// given round-trip time to each outbound datagram (set it on both peers for
// that RTT); rate_mbps makes the outbound path a bottleneck link of that rate
// with a drop-tail queue of queue_kb (default 256) — serialization and
// queueing delay, congestion losses — so SCTP's congestion control meets a
// realistic path. assoc_down_ms=N: this process's extra associations ("assoc"
// extension, tunnel/assoc.cc) fail N ms after they come up (fail-over tests).
namespace {
struct FaultCfg {
  double drop = 0, dup = 0;
  uint64_t delay_us = 0;
  uint64_t fixed_us = 0;    // one-way propagation delay
  double rate_bps = 0;      // bottleneck rate (0 = unlimited)
  uint64_t queue_bytes = 256 * 1024;
  uint64_t bh_start_ms = 0, bh_len_ms = 0, t0_ms = 0;
  uint64_t assoc_down_ms = 0;
  bool on = false;
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  FaultCfg() {
    const char* spec = getenv("TUNNEL_FAULT");
    std::string s = spec ? spec : "";
    for (size_t p = 0; p < s.size();) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      const std::string kv = s.substr(p, q - p);
      p = q + 1;
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) continue;
      const std::string k = kv.substr(0, eq);
      const char* v = kv.c_str() + eq + 1;
      if (k == "drop" || k == "loss") drop = atof(v);
      else if (k == "dup") dup = atof(v);
      else if (k == "delay_ms") delay_us = uint64_t(atof(v) * 1000);
      else if (k == "rtt_ms") fixed_us = uint64_t(atof(v) * 500);
      else if (k == "rate_mbps") rate_bps = atof(v) * 1e6;
      else if (k == "queue_kb") queue_bytes = uint64_t(atof(v) * 1024);
      else if (k == "assoc_down_ms") assoc_down_ms = strtoull(v, nullptr, 10);
      else if (k == "blackhole") {
        bh_start_ms = strtoull(v, nullptr, 10);
        if (const char* c = strchr(v, ':')) bh_len_ms = strtoull(c + 1, nullptr, 10);
      } else {
        LOG_WARN(kT, "TUNNEL_FAULT: unknown key '%s'", k.c_str());
      }
    }
    t0_ms = Reactor::now_ms();
    on = drop > 0 || dup > 0 || delay_us > 0 || bh_len_ms > 0 || fixed_us > 0 || rate_bps > 0;
    rng ^= uint64_t(getpid()) << 20;
  }
  bool wan() const { return fixed_us > 0 || rate_bps > 0; }
  bool blackholed() const {
    uint64_t t = Reactor::now_ms() - t0_ms;
    return bh_len_ms && t >= bh_start_ms && t < bh_start_ms + bh_len_ms;
  }
  double uni() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return double(rng >> 11) / double(1ull << 53);
  }
};
FaultCfg& fault() {
  static FaultCfg f;
  return f;
}
}  // namespace

uint64_t fault_assoc_down_ms() { return fault().assoc_down_ms; }

bool IceAgent::direct_target(int* fd, SockAddr* to, size_t* coalesce) const {
  if (sel_local_ < 0 || closed_ || nat_mode_ || fault().on || locals_[sel_local_].relay) return false;
  *fd = socks_[locals_[sel_local_].sock].fd;
  *to = sel_remote_;
  *coalesce = coalesce_limit_;
  return true;
}

bool IceAgent::detach_reader(int* fd, int* si, SockAddr* remote) {
  size_t co;
  if (detached_ >= 0 || !direct_target(fd, remote, &co)) return false;
  *si = locals_[sel_local_].sock;
  detached_ = *si;
  r_.modify(*fd, 0);
  return true;
}

bool IceAgent::reader_target(int* fd, int* si, SockAddr* remote) const {
  size_t co;
  if (detached_ >= 0 || !direct_target(fd, remote, &co)) return false;
  *si = locals_[sel_local_].sock;
  return true;
}

void IceAgent::reattach_reader(int si) {
  if (detached_ != si) return;
  detached_ = -1;
  if (!closed_ && si >= 0 && si < int(socks_.size()) && socks_[si].fd >= 0) {
    r_.modify(socks_[si].fd, EPOLLIN);
    on_readable(si);  // whatever arrived in between
  }
}

void IceAgent::inject(int si, const SockAddr& from, const RawBufPtr& owner, size_t off, size_t len) {
  if (closed_ || nat_mode_) return;
  dispatch_rx(si, from, owner, len, off);
}

void IceAgent::note_rx() {
  last_rx_ = Reactor::now_ms();
  if (state_ == IceState::Disconnected && sel_local_ >= 0) set_state(IceState::Connected);
}

// Releases the WAN-emulation queue's due datagrams into the send queue (the
// flush hook that follows the timer sends them).
void IceAgent::arm_delay_timer() {
  std::weak_ptr<IceAgent> w = shared_from_this();
  delay_timer_ = r_.call_at(delayq_.front().first, [w] {
    auto s = w.lock();
    if (!s) return;
    s->delay_timer_ = 0;
    if (s->closed_) return;
    uint64_t now = Reactor::now_us();
    while (!s->delayq_.empty() && s->delayq_.front().first <= now) {
      s->outq_.push_back(std::move(s->delayq_.front().second));
      s->delayq_.pop_front();
    }
    if (!s->delayq_.empty()) s->arm_delay_timer();
  });
}

void IceAgent::flush() {
  struct Recycle {
    IceAgent* a;
    ~Recycle() {
      for (auto& o : a->outq_)
        if (a->spare_.size() < 64 && o.data.capacity() >= 2048) {
          o.data.clear();
          a->spare_.push_back(std::move(o.data));
        }
      a->outq_.clear();
    }
  } recycle{this};
  if (outq_.empty() || closed_) return;
  if (fault().on) {
    if (fault().blackholed()) return;
    std::vector<Out> keep;
    FaultCfg& f = fault();
    for (auto& o : outq_) {
      if (o.faulted || o.local < 0) {
        keep.push_back(std::move(o));
        continue;
      }
      bool stun = stun::looks_like_stun(o.data.data(), o.data.size());
      if (!stun && f.uni() < f.drop) continue;
      if (f.wan()) {  // bottleneck link + propagation delay, in order
        uint64_t now = Reactor::now_us();
        uint64_t start = std::max(now, link_free_us_);
        if (f.rate_bps > 0 && double(start - now) * f.rate_bps / 8e6 > double(f.queue_bytes)) {
          wan_queue_drops_++;  // drop-tail: the bottleneck queue is full
          continue;
        }
        uint64_t tx = f.rate_bps > 0 ? uint64_t(double(o.data.size()) * 8e6 / f.rate_bps) : 0;
        link_free_us_ = start + tx;
        o.faulted = true;
        delayq_.emplace_back(link_free_us_ + f.fixed_us, std::move(o));
        continue;
      }
      if (stun) {
        keep.push_back(std::move(o));
        continue;
      }
      int copies = f.uni() < f.dup ? 2 : 1;
      for (int c = 0; c < copies; c++) {
        if (f.delay_us) {
          uint64_t d = uint64_t(f.uni() * double(f.delay_us));
          auto held = std::make_shared<Out>(o);
          held->faulted = true;
          std::weak_ptr<IceAgent> w = shared_from_this();
          r_.call_later_us(d, [w, held] {
            auto s = w.lock();
            if (!s || s->closed_) return;
            s->outq_.push_back(std::move(*held));
          });
        } else {
          keep.push_back(o);
        }
      }
    }
    outq_.swap(keep);
    if (!delayq_.empty() && !delay_timer_) arm_delay_timer();
    if (outq_.empty()) return;
  }
  // Group consecutive datagrams by socket for sendmmsg; within a group, runs
  // of equal-size datagrams to one destination become one UDP GSO message
  // (UDP_SEGMENT): one skb through the stack instead of one per datagram,
  // delivered whole to a GRO-enabled receiver on the same host. Standard-MTU
  // bulk traffic is exactly that: full SCTP packets -> equal DTLS records.
  constexpr int kBatch = 64, kIov = 512;
  mmsghdr msgs[kBatch];
  iovec iovs[kIov];
  alignas(cmsghdr) char ctrl[kBatch][CMSG_SPACE(sizeof(uint16_t))];
  // udp_tx is stamped before the send syscall: on loopback the kernel
  // delivers inside sendmmsg, so a stamp after it read as 1-5 us *after* the
  // receiver's udp_kernel (profiles/r05/b30/ttft8.json).
  trace::tx_done();
  size_t i = 0;
  while (i < outq_.size()) {
    // Resolve the socket (relay locals go through TURN).
    int li = outq_[i].local;
    if (li >= 0 && locals_[li].relay) {
      if (turn_) turn_->send_to(outq_[i].to, outq_[i].data.data(), outq_[i].data.size());
      i++;
      continue;
    }
    int si = li >= 0 ? locals_[li].sock : (-1 - li);
    int fd = nat_mode_ ? nat_fd_for(si, outq_[i].to) : socks_[si].fd;
    int cnt = 0, niov = 0;
    size_t j = i;
    while (j < outq_.size() && cnt < kBatch && niov < kIov) {
      int lj = outq_[j].local;
      if (lj >= 0 && locals_[lj].relay) break;
      int sj = lj >= 0 ? locals_[lj].sock : (-1 - lj);
      if (sj != si) break;
      if (nat_mode_ && nat_fd_for(sj, outq_[j].to) != fd) break;
      // One message: datagram j plus following ones of the same size to the
      // same address (the run's last datagram may be shorter).
      size_t seg = outq_[j].data.size();
      int first = niov;
      size_t total = 0;
      size_t k = j;
      while (k < outq_.size() && niov < kIov) {
        const Out& o = outq_[k];
        if (k > j) {
          if (!gso_ok_ || o.local != outq_[j].local || o.to != outq_[j].to || o.data.size() > seg) break;
          if (niov - first >= kGsoMaxSegs || total + o.data.size() > kGsoMaxBytes) break;
        }
        iovs[niov].iov_base = const_cast<uint8_t*>(o.data.data());
        iovs[niov].iov_len = o.data.size();
        niov++;
        total += o.data.size();
        k++;
        if (o.data.size() < seg) break;  // a short datagram ends the run
      }
      mmsghdr& m = msgs[cnt];
      memset(&m, 0, sizeof m);
      m.msg_hdr.msg_iov = &iovs[first];
      m.msg_hdr.msg_iovlen = size_t(niov - first);
      m.msg_hdr.msg_name = const_cast<sockaddr*>(outq_[j].to.sa());
      m.msg_hdr.msg_namelen = outq_[j].to.len;
      if (niov - first > 1) {
        m.msg_hdr.msg_control = ctrl[cnt];
        m.msg_hdr.msg_controllen = sizeof ctrl[cnt];
        cmsghdr* c = CMSG_FIRSTHDR(&m.msg_hdr);
        c->cmsg_level = SOL_UDP;
        c->cmsg_type = UDP_SEGMENT;
        c->cmsg_len = CMSG_LEN(sizeof(uint16_t));
        uint16_t gs = uint16_t(seg);
        memcpy(CMSG_DATA(c), &gs, sizeof gs);
        gso_sends_++;
      }
      cnt++;
      j = k;
    }
    int sent = 0;
    while (sent < cnt) {
      int rc = sendmmsg(fd, msgs + sent, unsigned(cnt - sent), 0);
      if (rc < 0) {
        if (errno == EINTR) continue;
        if ((errno == EIO || errno == EINVAL || errno == ENOPROTOOPT) && gso_ok_ &&
            msgs[sent].msg_hdr.msg_controllen) {
          // No UDP GSO here (old kernel, device without it): send this
          // message's datagrams one by one and stop using GSO.
          LOG_DEBUG(kT, "UDP GSO unavailable (%s); sending datagrams individually", strerror(errno));
          gso_ok_ = false;
          mmsghdr& m = msgs[sent];
          for (size_t q = 0; q < m.msg_hdr.msg_iovlen; q++)
            sendto(fd, m.msg_hdr.msg_iov[q].iov_base, m.msg_hdr.msg_iov[q].iov_len, 0,
                   static_cast<const sockaddr*>(m.msg_hdr.msg_name), m.msg_hdr.msg_namelen);
          sent++;
          continue;
        }
        // EAGAIN (socket buffer full) or unreachable: drop (counted); SCTP
        // retransmits.
        if (errno != EAGAIN) LOG_TRACE(kT, "sendmmsg: %s", strerror(errno));
        send_drops_ += uint64_t(cnt - sent);
        break;
      }
      sent += rc;
    }
    i = j;
  }
}

int IceAgent::local_for_socket(int si, bool relay) const {
  for (int i = 0; i < int(locals_.size()); i++)
    if (locals_[i].sock == si && locals_[i].relay == relay && locals_[i].c.type != "srflx") return i;
  return -1;
}

void IceAgent::on_readable(int si) {
  // A socket handed to the outside reader (detach_reader) is read there only:
  // an event for it queued earlier in this reactor turn, or a detach made by a
  // callback of this very loop (a flush hook engaging the reader), must not
  // read it here too, or datagrams of one flow overtake each other between
  // the two paths (past DTLS's replay window, they are dropped as old).
  if (closed_ || si == detached_) return;
  auto self = shared_from_this();
  constexpr int kBatch = 32;
  mmsghdr msgs[kBatch];
  iovec iovs[kBatch];
  sockaddr_storage from[kBatch];
  // Room for UDP_GRO and SO_RXQ_OVFL (a truncated GRO cmsg would read a
  // coalesced burst as one datagram).
  alignas(cmsghdr) char ctrl[kBatch][CMSG_SPACE(sizeof(int)) + CMSG_SPACE(sizeof(uint32_t)) +
                                      CMSG_SPACE(sizeof(timespec))];
  for (int round = 0; round < 8 && !closed_ && si != detached_; round++) {
    for (int i = 0; i < kBatch; i++) rxpool_[i].reset();
    for (int i = 0; i < kBatch; i++) {
      // Buffers whose datagrams are still referenced (zero-copy views handed
      // up the stack, possibly to worker threads) stay out of the pool's
      // rotation until the views are gone.
      rxpool_[i] = rxbufs_.get();
      memset(&msgs[i], 0, sizeof msgs[i]);
      iovs[i].iov_base = rxpool_[i]->data.get();
      iovs[i].iov_len = 65536;
      msgs[i].msg_hdr.msg_iov = &iovs[i];
      msgs[i].msg_hdr.msg_iovlen = 1;
      msgs[i].msg_hdr.msg_name = &from[i];
      msgs[i].msg_hdr.msg_namelen = sizeof from[i];
      msgs[i].msg_hdr.msg_control = ctrl[i];
      msgs[i].msg_hdr.msg_controllen = sizeof ctrl[i];
    }
    int n = recvmmsg(socks_[si].fd, msgs, kBatch, MSG_DONTWAIT, nullptr);
    if (n <= 0) break;
    const bool traced = trace::enabled();
    const uint64_t t_read = traced ? Reactor::now_us() : 0;
    for (int i = 0; i < n && !closed_; i++) {
      // Each datagram's own kernel receive time (the batch's first one made a
      // frame from a later datagram read as queued before it was sent:
      // req_end -> udp_kernel < 0 in the hop tables).
      if (traced) trace::set_rx(trace::kernel_rx_us(&msgs[i].msg_hdr), t_read, t_read);
      if (nat_mode_) {  // private address: unreachable from outside the emulated NAT
        nat_dropped_++;
        continue;
      }
      SockAddr a;
      memcpy(&a.ss, &from[i], msgs[i].msg_hdr.msg_namelen);
      a.len = msgs[i].msg_hdr.msg_namelen;
      rx_bytes_ += msgs[i].msg_len;
      dispatch_segments(si, a, rxpool_[i], msgs[i].msg_len, gro_segment(&msgs[i].msg_hdr));
    }
    if (n < kBatch) break;
  }
  if (on_rx_burst_end && !closed_) on_rx_burst_end();
}

void IceAgent::dispatch_rx(int si, const SockAddr& a, const RawBufPtr& owner, size_t len, size_t off) {
  const uint8_t* p = owner->data.get() + off;
  if (turn_ && turn_->is_server(si, a)) {
    turn_->on_packet(p, len);
    return;
  }
  handle_datagram(-1, si, a, p, len, false, owner);
}

// A GRO-coalesced receive holds several datagrams of `seg` bytes back to back
// (the last may be shorter); each is its own DTLS datagram. Zero-copy: every
// segment is handed up as a view of the same pooled buffer.
void IceAgent::dispatch_segments(int si, const SockAddr& a, const RawBufPtr& owner, size_t len, size_t seg) {
  if (!seg || seg >= len) {
    dispatch_rx(si, a, owner, len, 0);
    return;
  }
  gro_batches_++;
  for (size_t off = 0; off < len && !closed_; off += seg) dispatch_rx(si, a, owner, std::min(seg, len - off), off);
}

int IceAgent::nat_fd_for(int si, const SockAddr& to) {
  std::string key = std::to_string(si);
  if (nat_mode_ == 2) key += "|" + to.str();
  auto it = nat_map_.find(key);
  int pi;
  if (it != nat_map_.end()) {
    pi = it->second;
  } else {
    NatPort np;
    np.si = si;
    np.fd = ::socket(socks_[si].addr.family(), SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    SockAddr a = socks_[si].addr;
    a.set_port(0);
    udp_socket_buffers(np.fd, 4 << 20);  // no GRO: read with plain recvfrom
    if (np.fd < 0 || ::bind(np.fd, a.sa(), a.len) < 0) return socks_[si].fd;
    np.ext.len = sizeof np.ext.ss;
    getsockname(np.fd, np.ext.sa(), &np.ext.len);
    pi = int(nat_ports_.size());
    nat_ports_.push_back(np);
    nat_map_[key] = pi;
    std::weak_ptr<IceAgent> w = shared_from_this();
    r_.add(np.fd, EPOLLIN, [w, pi](uint32_t) {
      if (auto self = w.lock()) self->on_nat_readable(pi);
    });
    LOG_DEBUG(kT, "NAT emulation: %s -> external %s%s", socks_[si].addr.str().c_str(), np.ext.str().c_str(),
              nat_mode_ == 2 ? (" for " + to.str()).c_str() : "");
  }
  nat_ports_[pi].sent.insert(to.str());
  return nat_ports_[pi].fd;
}

void IceAgent::on_nat_readable(int pi) {
  if (closed_) return;
  auto self = shared_from_this();
  for (int round = 0; round < 64 && !closed_; round++) {
    rxpool_[0].reset();
    rxpool_[0] = rxbufs_.get();
    SockAddr a;
    a.len = sizeof a.ss;
    ssize_t n = recvfrom(nat_ports_[pi].fd, rxpool_[0]->data.get(), 65536, MSG_DONTWAIT, a.sa(), &a.len);
    if (n < 0) return;
    if (!nat_ports_[pi].sent.count(a.str())) {  // address+port-dependent filtering
      nat_dropped_++;
      continue;
    }
    dispatch_rx(nat_ports_[pi].si, a, rxpool_[0], size_t(n));
  }
}

void IceAgent::handle_datagram(int, int si, const SockAddr& from, const uint8_t* p, size_t n, bool via_relay,
                               const RawBufPtr& owner) {
  if (n == 0) return;
  last_rx_ = Reactor::now_ms();
  if (stun::looks_like_stun(p, n)) {
    handle_stun(si, from, p, n, via_relay);
    return;
  }
  if (state_ == IceState::Disconnected && sel_local_ >= 0) set_state(IceState::Connected);
  // Data before we selected a pair (the peer nominated first): use the path it used.
  if (sel_local_ < 0) {
    int li = local_for_socket(si, via_relay);
    if (li >= 0 && find_remote(from) >= 0) {
      sel_local_ = li;
      sel_remote_ = from;
      path_gen_++;
    }
  }
  if (!on_data) return;
  if (owner && p >= owner->data.get() && p + n <= owner->data.get() + owner->cap) {
    on_data(owner, owner->data.get() + (p - owner->data.get()), n);
  } else {  // relayed (inside a TURN message): private copy
    auto b = std::make_shared<RawBuf>(n ? n : 1);
    memcpy(b->data.get(), p, n);
    uint8_t* d = b->data.get();
    on_data(std::move(b), d, n);
  }
}

void IceAgent::handle_stun(int si, const SockAddr& from, const uint8_t* p, size_t n, bool via_relay) {
  stun::Message m;
  if (!stun::Message::parse(p, n, m)) return;
  if (m.fingerprint_off >= 0 && !stun::verify_fingerprint(p, n, m)) return;
  if (m.cls() == 0 && m.method() == 1) {
    handle_request(si, from, m, p, n, via_relay);
  } else if (m.cls() == 2 || m.cls() == 3) {
    handle_response(from, m, p, n);
  }
  // Binding indications (keepalives) need no action beyond last_rx_.
}

void IceAgent::handle_request(int si, const SockAddr& from, const stun::Message& m, const uint8_t* p, size_t n,
                              bool via_relay) {
  const stun::Attr* user = m.get(stun::kUsername);
  if (!user || !stun::verify_integrity(p, n, m, pwd_)) {
    auto resp = stun::Message{};
    resp.type = stun::kBindingError;
    memcpy(resp.tid, m.tid, 12);
    resp.add_error(user ? 401 : 400, user ? "Unauthorized" : "Bad Request");
    auto b = resp.serialize(nullptr, true);
    int li = local_for_socket(si, via_relay);
    send_raw(li >= 0 ? li : -1 - si, from, b.data(), b.size());
    return;
  }
  size_t colon = user->value.find(':');
  if (colon == std::string::npos || user->value.substr(0, colon) != ufrag_) return;
  // Role conflict (RFC 8445 §7.3.1.1).
  uint64_t their_tb;
  bool conflict = false;
  if (controlling_ && m.get_u64(stun::kIceControlling, their_tb)) {
    if (tiebreaker_ >= their_tb) conflict = true;
    else {
      controlling_ = false;
      LOG_DEBUG(kT, "ICE role conflict: switching to controlled");
    }
  } else if (!controlling_ && m.get_u64(stun::kIceControlled, their_tb)) {
    if (tiebreaker_ >= their_tb) {
      controlling_ = true;
      LOG_DEBUG(kT, "ICE role conflict: switching to controlling");
    } else {
      conflict = true;
    }
  }
  int li = local_for_socket(si, via_relay);
  if (conflict) {
    stun::Message resp;
    resp.type = stun::kBindingError;
    memcpy(resp.tid, m.tid, 12);
    resp.add_error(487, "Role Conflict");
    auto b = resp.serialize(&pwd_, true);
    send_raw(li >= 0 ? li : -1 - si, from, b.data(), b.size());
    return;
  }
  stun::Message resp;
  resp.type = stun::kBindingSuccess;
  memcpy(resp.tid, m.tid, 12);
  resp.add_xor_addr(stun::kXorMappedAddress, from);
  auto b = resp.serialize(&pwd_, true);
  send_raw(li >= 0 ? li : -1 - si, from, b.data(), b.size());
  if (li < 0) return;
  // Peer-reflexive remote candidate.
  int ri = find_remote(from);
  if (ri < 0) {
    Candidate c;
    c.type = "prflx";
    c.addr = from;
    uint32_t prio = 0;
    m.get_u32(stun::kPriority, prio);
    c.priority = prio;
    c.foundation = "prflx" + std::to_string(remotes_.size());
    remotes_.push_back(c);
    ri = int(remotes_.size()) - 1;
    for (int l = 0; l < int(locals_.size()); l++) pair_up(l, ri);
    if (state_ == IceState::New) {
      checking_since_ = Reactor::now_ms();
      set_state(IceState::Checking);
    }
  }
  // The peer reached us on this socket from that address, so the pair works
  // even where our own pairing rules left it out (a TURN relay on loopback
  // forwarding to a non-loopback host candidate): add it, as a triggered
  // check would (RFC 8445 §7.3.1.4), so that a nomination of it counts here.
  // Without it the controlling agent selected a pair this agent never had.
  if (!(cfg_.relay_only && !locals_[li].relay) && locals_[li].c.type != "srflx") add_pair(li, ri);
  bool use_cand = m.get(stun::kUseCandidate) != nullptr;
  for (int pi = 0; pi < int(pairs_.size()); pi++) {
    Pair& pr = pairs_[pi];
    if (pr.local != li || pr.remote != ri) continue;
    if (use_cand && !controlling_) {
      // Nominated by the controlling agent. Select right away (its check of
      // this pair just succeeded end-to-end with our response). Aggressive
      // nomination nominates every pair it checks, so a later nomination of
      // a higher-priority pair moves the selection there: both agents end on
      // the highest-priority nominated pair (RFC 8445 §8.1.1) — the first to
      // arrive here and the first to succeed there may differ.
      if (sel_pair_ < 0 || pr.prio > pairs_[sel_pair_].prio) select_pair(pi);
    }
    if (pr.st == Pair::St::Waiting || pr.st == Pair::St::Failed) {
      pr.st = Pair::St::Waiting;  // triggered check
      pr.next_tx = 0;
      if (sel_pair_ < 0 && !remote_pwd_.empty()) kick();
    }
  }
}

void IceAgent::handle_response(const SockAddr& from, const stun::Message& m, const uint8_t* p, size_t n) {
  std::string tid = m.tid_key();
  for (size_t i = 0; i < srflx_.size(); i++) {
    if (srflx_[i].tid != tid) continue;
    SockAddr mapped;
    if (m.cls() == 2 && (m.get_xor_addr(stun::kXorMappedAddress, mapped) || m.get_addr(stun::kMappedAddress, mapped))) {
      int si = srflx_[i].sock;
      bool dup = false;
      for (auto& l : locals_)
        if (l.c.addr == mapped) dup = true;
      if (!dup) {
        Candidate c;
        c.type = "srflx";
        c.addr = mapped;
        c.related = socks_[si].addr;
        c.has_related = true;
        c.priority = candidate_priority("srflx", 65535 - uint32_t(si) * 256);
        c.foundation = std::to_string(crc32_ieee(("srflx" + socks_[si].addr.ip()).data(), 5 + socks_[si].addr.ip().size()));
        add_local(c, si, false);
      }
    }
    auto win = srflx_[i].win;
    srflx_.erase(srflx_.begin() + long(i));
    if (win && --win->outstanding == 0) srflx_window_done(win);
    return;
  }
  auto it = tx_pairs_.find(tid);
  if (it == tx_pairs_.end()) return;
  int pi = it->second;
  tx_pairs_.erase(it);
  if (pi >= int(pairs_.size())) return;
  Pair& pr = pairs_[pi];
  if (!remote_pwd_.empty() && !stun::verify_integrity(p, n, m, remote_pwd_)) return;
  if (m.cls() == 3) {
    if (m.error_code() == 487) {
      controlling_ = !controlling_;
      LOG_DEBUG(kT, "ICE 487 role conflict: now %s", controlling_ ? "controlling" : "controlled");
      pr.st = Pair::St::Waiting;
      pr.next_tx = 0;
      pr.tries = 0;
    } else {
      pr.st = Pair::St::Failed;
    }
    return;
  }
  (void)from;
  if (pr.sent_us) {
    const uint64_t rtt = std::max<uint64_t>(1, Reactor::now_us() - pr.sent_us);
    if (!check_rtt_us_ || rtt < check_rtt_us_) check_rtt_us_ = rtt;
  }
  pr.st = Pair::St::Succeeded;
  if (controlling_ && pr.use_cand) {
    // The first nominated pair to succeed carries the connection at once; a
    // higher-priority one that succeeds later takes over (the controlled
    // agent moves to it too when its nomination arrives).
    if (sel_pair_ < 0 || pr.prio > pairs_[sel_pair_].prio) select_pair(pi);
  } else if (controlling_ && sel_pair_ < 0) {
    // Regular nomination: follow up with USE-CANDIDATE on the first valid pair.
    pr.use_cand = true;
    pr.st = Pair::St::Waiting;
    pr.next_tx = 0;
    pr.tries = 0;
  }
}

void IceAgent::select_pair(int pi) {
  Pair& pr = pairs_[pi];
  const bool switched = sel_pair_ >= 0 && sel_pair_ != pi;
  sel_pair_ = pi;
  if (sel_local_ != pr.local || sel_remote_ != remotes_[pr.remote].addr) path_gen_++;
  sel_local_ = pr.local;
  sel_remote_ = remotes_[pr.remote].addr;
  if (switched) LOG_INFO(kT, "ICE pair switched to %s (higher-priority nominated pair)", selected_desc().c_str());
  else LOG_DEBUG(kT, "ICE selected pair %s", selected_desc().c_str());
  last_rx_ = Reactor::now_ms();
  set_state(IceState::Connected);
}

std::string IceAgent::selected_desc() const {
  if (sel_local_ < 0) return "(none)";
  const Local& l = locals_[sel_local_];
  return l.c.type + ":" + (l.relay ? l.c.addr.str() : socks_[l.sock].addr.str()) + " <-> " + sel_remote_.str();
}

bool IceAgent::selected_same_host() const {
  if (sel_local_ < 0 || locals_[sel_local_].relay) return false;
  if (sel_remote_.is_loopback()) return true;
  for (auto& s : socks_) {
    SockAddr a = s.addr, b = sel_remote_;
    a.set_port(0);
    b.set_port(0);
    if (a == b) return true;
  }
  return false;
}

void IceAgent::send_check(Pair& pr) {
  const Candidate& rc = remotes_[pr.remote];
  const Local& l = locals_[pr.local];
  auto m = stun::Message::make(stun::kBindingRequest);
  m.add(stun::kUsername, remote_ufrag_ + ":" + ufrag_);
  m.add_u32(stun::kPriority, candidate_priority("prflx", (l.c.priority >> 8) & 0xFFFF));
  if (controlling_) {
    m.add_u64(stun::kIceControlling, tiebreaker_);
    // Aggressive nomination: the first pair to succeed is used.
    pr.use_cand = true;
    m.add(stun::kUseCandidate, "");
  } else {
    m.add_u64(stun::kIceControlled, tiebreaker_);
  }
  auto b = m.serialize(&remote_pwd_, true);
  if (!pr.tid.empty()) tx_pairs_.erase(pr.tid);
  pr.tid = m.tid_key();
  pr.sent_us = Reactor::now_us();
  int pi = int(&pr - pairs_.data());
  tx_pairs_[pr.tid] = pi;
  send_raw(pr.local, rc.addr, b.data(), b.size());
}

void IceAgent::tick() {
  if (closed_) return;
  uint64_t now = Reactor::now_ms();
  std::weak_ptr<IceAgent> w = shared_from_this();
  if (!remote_pwd_.empty() && (sel_pair_ < 0 || controlling_)) {
    // Retransmit in-progress checks; start the highest-priority waiting check
    // (pacing Ta = 20 ms). Once a pair is selected, only the controlling
    // agent's checks of higher-priority pairs still run (a lost check or
    // response must not leave the two agents on different pairs).
    const uint64_t floor = sel_pair_ < 0 ? 0 : pairs_[sel_pair_].prio + 1;
    for (auto& pr : pairs_) {
      if (pr.st != Pair::St::InProgress || now < pr.next_tx || pr.prio < floor) continue;
      if (pr.tries >= 7) {
        pr.st = Pair::St::Failed;
        continue;
      }
      send_check(pr);
      pr.tries++;
      pr.rto = std::min<uint64_t>(pr.rto * 2, 1600);
      pr.next_tx = now + pr.rto;
    }
    Pair* best = nullptr;
    for (auto& pr : pairs_)
      if (pr.st == Pair::St::Waiting && pr.prio >= floor && (!best || pr.prio > best->prio)) best = &pr;
    if (best) {
      best->st = Pair::St::InProgress;
      best->tries = 1;
      best->rto = 100;
      best->next_tx = now + best->rto;
      send_check(*best);
    }
  }
  if (state_ == IceState::Checking && sel_pair_ < 0 && sel_local_ < 0 && checking_since_ &&
      now - checking_since_ > cfg_.failed_ms) {
    LOG_WARN(kT, "ICE connectivity checks failed after %llu ms", static_cast<unsigned long long>(now - checking_since_));
    set_state(IceState::Failed);
    return;
  }
  if (sel_local_ >= 0) {
    if (sel_pair_ < 0 && state_ != IceState::Connected && state_ != IceState::Disconnected) {
      // Path learned from inbound data before our own nomination completed.
      set_state(IceState::Connected);
    }
    // Consent freshness / keepalive on the selected pair (RFC 7675).
    if (now - last_keepalive_ >= cfg_.keepalive_ms && !remote_pwd_.empty()) {
      last_keepalive_ = now;
      auto m = stun::Message::make(stun::kBindingRequest);
      m.add(stun::kUsername, remote_ufrag_ + ":" + ufrag_);
      m.add_u32(stun::kPriority, candidate_priority("prflx", 65535));
      if (controlling_) m.add_u64(stun::kIceControlling, tiebreaker_);
      else m.add_u64(stun::kIceControlled, tiebreaker_);
      auto b = m.serialize(&remote_pwd_, true);
      send_raw(sel_local_, sel_remote_, b.data(), b.size());
    }
    uint64_t idle = now - last_rx_;
    if (idle > cfg_.failed_ms) {
      LOG_WARN(kT, "ICE: no traffic from peer for %llu ms", static_cast<unsigned long long>(idle));
      set_state(IceState::Failed);
      return;
    }
    if (idle > cfg_.disconnected_ms && state_ == IceState::Connected) set_state(IceState::Disconnected);
  }
  if (closed_ || state_ == IceState::Failed) return;
  uint64_t next = (sel_pair_ < 0 && !remote_pwd_.empty()) ? 20 : 250;
  tick_timer_ = r_.call_later_ms(next, [w] {
    if (auto s = w.lock()) {
      s->tick_timer_ = 0;
      s->tick();
    }
  });
}

}  // namespace p2pt::rtc
