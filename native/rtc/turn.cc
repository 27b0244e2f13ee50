#include "rtc/turn.h"

#include <cstring>

#include "core/buf.h"
#include "core/log.h"
#include "rtc/ice.h"

namespace p2pt::rtc {

static const char* kT = "tunnel::turn";

bool TurnClient::parse_url(const std::string& url, TurnUrl& out, std::string* err) {
  auto fail = [&](const std::string& why) {
    if (err) *err = why;
    return false;
  };
  size_t colon = url.find(':');
  if (colon == std::string::npos) return fail("TURN URL '" + url + "' has no scheme (turn: or turns:)");
  const std::string scheme = url.substr(0, colon);
  if (scheme == "turn") {
    out.transport = TurnUrl::Transport::Udp;
    out.port = 3478;
  } else if (scheme == "turns") {
    out.transport = TurnUrl::Transport::Tls;
    out.port = 5349;
  } else {
    return fail("unsupported TURN URL scheme '" + scheme + ":' in '" + url + "' (use turn: or turns:)");
  }
  std::string s = url.substr(colon + 1);
  if (s.rfind("//", 0) == 0) s = s.substr(2);
  std::string query;
  if (size_t q = s.find('?'); q != std::string::npos) {
    query = s.substr(q + 1);
    s = s.substr(0, q);
  }
  for (size_t a = 0; a < query.size();) {
    size_t amp = query.find('&', a);
    if (amp == std::string::npos) amp = query.size();
    std::string kv = query.substr(a, amp - a);
    a = amp + 1;
    if (kv.rfind("transport=", 0) != 0) continue;  // other parameters carry no meaning here
    std::string tr = kv.substr(10);
    for (auto& c : tr) c = char(tolower(static_cast<unsigned char>(c)));
    if (tr == "tcp") {
      if (out.transport == TurnUrl::Transport::Udp) out.transport = TurnUrl::Transport::Tcp;
    } else if (tr == "udp") {
      if (out.transport == TurnUrl::Transport::Tls)
        return fail("unsupported TURN transport in '" + url + "': turns: over udp (DTLS) is not supported");
    } else {
      return fail("unsupported TURN transport '" + tr + "' in '" + url + "' (udp or tcp)");
    }
  }
  if (!s.empty() && s[0] == '[') {
    size_t rb = s.find(']');
    if (rb == std::string::npos) return fail("malformed IPv6 host in TURN URL '" + url + "'");
    out.host = s.substr(1, rb - 1);
    if (rb + 1 < s.size()) {
      if (s[rb + 1] != ':') return fail("malformed TURN URL '" + url + "'");
      out.port = uint16_t(atoi(s.c_str() + rb + 2));
    }
  } else if (size_t pc = s.rfind(':'); pc != std::string::npos) {
    out.host = s.substr(0, pc);
    out.port = uint16_t(atoi(s.c_str() + pc + 1));
  } else {
    out.host = s;
  }
  if (out.host.empty() || out.port == 0) return fail("malformed TURN URL '" + url + "'");
  return true;
}

std::shared_ptr<TurnClient> TurnClient::create(Reactor& r, IceAgent* agent, int sock, const TurnUrl& url,
                                               const std::string& user, const std::string& pass, AllocCb cb) {
  auto t = std::shared_ptr<TurnClient>(new TurnClient(r, agent, sock));
  t->user_ = user;
  t->pass_ = pass;
  t->alloc_cb_ = std::move(cb);
  if (url.transport != TurnUrl::Transport::Udp) {
    t->stream_ = true;
    t->connect_stream(url);
    return t;
  }
  const std::string host = url.host;
  const uint16_t port = url.port;
  std::weak_ptr<TurnClient> w = t;
  resolve_async(r, host, port, [w, host](std::vector<SockAddr> addrs, std::string err) {
    auto s = w.lock();
    if (!s || s->closed_) return;
    for (auto& a : addrs)
      if (a.family() == AF_INET) {
        s->server_ = a;
        s->resolved_ = true;
        break;
      }
    if (!s->resolved_) {
      LOG_WARN(kT, "TURN server %s unresolvable: %s", host.c_str(), err.c_str());
      auto cb = std::move(s->alloc_cb_);
      if (cb) cb(false, {}, {});
      return;
    }
    s->allocate();
  });
  return t;
}

// TCP / TLS control connection (TLS verified against the system trust store,
// SNI and host/IP checks, as for wss:// and https://).
void TurnClient::connect_stream(const TurnUrl& url) {
  std::weak_ptr<TurnClient> w = shared_from_this();
  const bool tls = url.transport == TurnUrl::Transport::Tls;
  const std::string desc = url.host + ":" + std::to_string(url.port) + " (" + url.transport_name() + ")";
  TcpConn::connect(
      r_, url.host, url.port, tls,
      [w, desc](std::shared_ptr<TcpConn> c, std::string err) {
        auto s = w.lock();
        if (!s || s->closed_) {
          if (c) c->close();
          return;
        }
        if (!c) {
          LOG_WARN(kT, "TURN server %s unreachable: %s", desc.c_str(), err.c_str());
          s->fail_alloc();
          return;
        }
        s->conn_ = c;
        s->server_ = c->peer();
        s->resolved_ = true;
        c->on_data([w](const uint8_t* p, size_t n) {
          if (auto x = w.lock()) x->on_stream_data(p, n);
        });
        c->on_close([w, desc](const std::string& why) {
          auto x = w.lock();
          if (!x || x->closed_) return;
          LOG_WARN(kT, "TURN connection to %s closed%s%s", desc.c_str(), why.empty() ? "" : ": ", why.c_str());
          x->conn_.reset();
          if (!x->allocated_) x->fail_alloc();
        });
        LOG_DEBUG(kT, "TURN control connection to %s up", desc.c_str());
        s->allocate();
      },
      10000);
}

// Stream framing (RFC 8656 §12.5 / RFC 5389 §7.2.2): ChannelData (first byte
// 0x40-0x7F) is 4 + length bytes padded to 4; a STUN message is 20 + length.
void TurnClient::on_stream_data(const uint8_t* p, size_t n) {
  inbuf_.append(reinterpret_cast<const char*>(p), n);
  size_t off = 0;
  auto self = shared_from_this();
  while (inbuf_.size() - off >= 4 && !closed_) {
    const uint8_t* m = reinterpret_cast<const uint8_t*>(inbuf_.data()) + off;
    size_t len;
    if (m[0] >= 0x40 && m[0] <= 0x7F) len = (4 + size_t(rd16(m + 2)) + 3) & ~size_t(3);
    else if (m[0] < 4) len = 20 + size_t(rd16(m + 2));
    else {  // not STUN or ChannelData: the stream is out of sync
      LOG_WARN(kT, "TURN stream framing lost; closing the connection");
      inbuf_.clear();
      if (conn_) conn_->close("framing");
      return;
    }
    if (inbuf_.size() - off < len) break;
    on_packet(m, len);
    off += len;
  }
  inbuf_.erase(0, off);
}

void TurnClient::fail_alloc() {
  auto cb = std::move(alloc_cb_);
  alloc_cb_ = nullptr;
  if (cb) cb(false, {}, {});
}

TurnClient::~TurnClient() { close(); }

void TurnClient::close() {
  if (closed_) return;
  closed_ = true;
  if (refresh_timer_) r_.cancel(refresh_timer_);
  if (perm_timer_) r_.cancel(perm_timer_);
  for (auto& kv : pending_)
    if (kv.second.timer) r_.cancel(kv.second.timer);
  pending_.clear();
  if (allocated_ && resolved_ && agent_) {
    // Best-effort deallocation: Refresh with LIFETIME 0.
    auto m = stun::Message::make(stun::kRefreshRequest);
    m.add_u32(stun::kLifetime, 0);
    sign(m);
    auto b = m.serialize(key_.empty() ? nullptr : &key_, true);
    raw_send(b.data(), b.size());
    if (!stream_) agent_->flush();
  }
  if (conn_) {
    conn_->on_data(nullptr);
    conn_->on_close(nullptr);
    conn_->close_after_flush();
    conn_.reset();
  }
  agent_ = nullptr;
}

void TurnClient::raw_send(const uint8_t* p, size_t n) {
  if (stream_) {
    if (conn_ && !conn_->closed()) conn_->write(Bytes::copy(p, n));
    return;
  }
  if (agent_) agent_->send_raw(-1 - sock_, server_, p, n);
}

void TurnClient::sign(stun::Message& m) {
  if (realm_.empty()) return;
  m.add(stun::kUsername, user_);
  m.add(stun::kRealm, realm_);
  m.add(stun::kNonce, nonce_);
}

void TurnClient::send_request(stun::Message m, std::function<void(const stun::Message&, const uint8_t*, size_t)> cb) {
  if (closed_) return;
  auto b = m.serialize(key_.empty() ? nullptr : &key_, true);
  std::string tid = m.tid_key();
  Pending& pd = pending_[tid];
  pd.cb = std::move(cb);
  pd.bytes = b;
  pd.tries = 1;
  raw_send(b.data(), b.size());
  // A reliable stream delivers the request or fails: no retransmissions, one
  // overall timeout (7 tries' worth) instead.
  if (stream_) pd.tries = 6;
  arm_retransmit(tid, stream_ ? 9500 : 500);
}

// STUN request retransmission: RTO doubling from 500 ms (capped at 3.2 s), 6 tries.
void TurnClient::arm_retransmit(const std::string& tid, uint64_t rto) {
  auto it = pending_.find(tid);
  if (it == pending_.end()) return;
  std::weak_ptr<TurnClient> w = shared_from_this();
  it->second.timer = r_.call_later_ms(rto, [w, tid, rto] {
    auto s = w.lock();
    if (!s) return;
    auto it2 = s->pending_.find(tid);
    if (it2 == s->pending_.end()) return;
    if (it2->second.tries >= 6) {
      auto cb2 = std::move(it2->second.cb);
      s->pending_.erase(it2);
      LOG_WARN(kT, "TURN request timed out");
      stun::Message none;
      none.type = 0;
      if (cb2) cb2(none, nullptr, 0);
      return;
    }
    it2->second.tries++;
    s->raw_send(it2->second.bytes.data(), it2->second.bytes.size());
    s->arm_retransmit(tid, std::min<uint64_t>(rto * 2, 3200));
  });
}

void TurnClient::allocate() {
  auto m = stun::Message::make(stun::kAllocateRequest);
  uint8_t rt[4] = {17, 0, 0, 0};  // UDP
  m.add(stun::kRequestedTransport, rt, 4);
  m.add_u32(stun::kLifetime, 600);
  sign(m);
  std::weak_ptr<TurnClient> w = shared_from_this();
  send_request(m, [w](const stun::Message& resp, const uint8_t*, size_t) {
    auto s = w.lock();
    if (!s || s->closed_) return;
    if (resp.type == 0) {
      auto cb = std::move(s->alloc_cb_);
      if (cb) cb(false, {}, {});
      return;
    }
    int code = resp.error_code();
    if (resp.cls() == 3 && (code == 401 || code == 438) && s->nonce_.empty() == (code == 401)) {
      const stun::Attr* realm = resp.get(stun::kRealm);
      const stun::Attr* nonce = resp.get(stun::kNonce);
      if (!nonce || (!realm && s->realm_.empty())) {
        auto cb = std::move(s->alloc_cb_);
        if (cb) cb(false, {}, {});
        return;
      }
      if (realm) s->realm_ = realm->value;
      s->nonce_ = nonce->value;
      s->key_ = stun::long_term_key(s->user_, s->realm_, s->pass_);
      s->allocate();
      return;
    }
    if (resp.cls() == 3 && code == 438) {
      if (const stun::Attr* nonce = resp.get(stun::kNonce)) {
        s->nonce_ = nonce->value;
        s->allocate();
        return;
      }
    }
    if (resp.cls() != 2 || !resp.get_xor_addr(stun::kXorRelayedAddress, s->relayed_)) {
      LOG_WARN(kT, "TURN allocation failed (error %d)", code);
      auto cb = std::move(s->alloc_cb_);
      if (cb) cb(false, {}, {});
      return;
    }
    resp.get_xor_addr(stun::kXorMappedAddress, s->mapped_);
    uint32_t lifetime = 600;
    resp.get_u32(stun::kLifetime, lifetime);
    s->allocated_ = true;
    LOG_INFO(kT, "TURN allocation: relayed %s (mapped %s, lifetime %us)", s->relayed_.str().c_str(),
             s->mapped_.str().c_str(), lifetime);
    s->refresh(lifetime);
    auto cb = std::move(s->alloc_cb_);
    if (cb) cb(true, s->relayed_, s->mapped_);
  });
}

void TurnClient::refresh(uint32_t lifetime) {
  uint64_t in_ms = (lifetime > 120 ? lifetime - 60 : lifetime / 2) * 1000ull;
  std::weak_ptr<TurnClient> w = shared_from_this();
  refresh_timer_ = r_.call_later_ms(in_ms, [w] {
    auto s = w.lock();
    if (!s || s->closed_) return;
    s->refresh_timer_ = 0;
    auto m = stun::Message::make(stun::kRefreshRequest);
    m.add_u32(stun::kLifetime, 600);
    s->sign(m);
    s->send_request(m, [w](const stun::Message& resp, const uint8_t*, size_t) {
      auto s2 = w.lock();
      if (!s2 || s2->closed_) return;
      if (resp.cls() == 3 && resp.error_code() == 438) {
        if (const stun::Attr* nonce = resp.get(stun::kNonce)) s2->nonce_ = nonce->value;
        s2->refresh(2);
        return;
      }
      uint32_t lt = 600;
      resp.get_u32(stun::kLifetime, lt);
      s2->refresh(lt);
    });
  });
  // Permissions expire after 300 s; refresh them every 240 s.
  if (!perm_timer_) {
    perm_timer_ = r_.call_later_ms(240000, [w] {
      auto s = w.lock();
      if (!s || s->closed_) return;
      s->perm_timer_ = 0;
      for (auto& kv : s->peers_) {
        SockAddr a;
        if (SockAddr::parse_hostport(kv.first, a)) s->create_permission(a);
      }
      s->refresh(600);
    });
  }
}

void TurnClient::create_permission(const SockAddr& peer) {
  auto m = stun::Message::make(stun::kCreatePermissionRequest);
  m.add_xor_addr(stun::kXorPeerAddress, peer);
  sign(m);
  std::weak_ptr<TurnClient> w = shared_from_this();
  std::string key = peer.str();
  send_request(m, [w, key, peer](const stun::Message& resp, const uint8_t*, size_t) {
    auto s = w.lock();
    if (!s || s->closed_) return;
    if (resp.cls() == 2) {
      auto& ps = s->peers_[key];
      if (!ps.permitted) {
        ps.permitted = true;
        s->channel_bind(peer);
      }
    } else if (resp.cls() == 3 && resp.error_code() == 438) {
      if (const stun::Attr* nonce = resp.get(stun::kNonce)) s->nonce_ = nonce->value;
      s->create_permission(peer);
    }
  });
}

void TurnClient::channel_bind(const SockAddr& peer) {
  auto& ps = peers_[peer.str()];
  if (ps.channel == 0) {
    if (next_channel_ > 0x7FFE) return;
    ps.channel = next_channel_++;
  }
  uint16_t ch = ps.channel;
  auto m = stun::Message::make(stun::kChannelBindRequest);
  uint8_t cn[4] = {uint8_t(ch >> 8), uint8_t(ch), 0, 0};
  m.add(stun::kChannelNumber, cn, 4);
  m.add_xor_addr(stun::kXorPeerAddress, peer);
  sign(m);
  std::weak_ptr<TurnClient> w = shared_from_this();
  std::string key = peer.str();
  send_request(m, [w, key, ch, peer](const stun::Message& resp, const uint8_t*, size_t) {
    auto s = w.lock();
    if (!s || s->closed_) return;
    if (resp.cls() == 2) {
      s->peers_[key].bound = true;
      s->channels_[ch] = peer;
    }
  });
}

void TurnClient::permit(const SockAddr& peer) {
  if (closed_ || !allocated_) return;
  if (peers_.count(peer.str())) return;
  peers_[peer.str()] = PeerState{};
  create_permission(peer);
}

void TurnClient::send_to(const SockAddr& peer, const uint8_t* p, size_t n) {
  if (closed_ || !allocated_) return;
  auto it = peers_.find(peer.str());
  if (it == peers_.end()) {
    permit(peer);
    it = peers_.find(peer.str());
  }
  if (it->second.bound) {
    std::vector<uint8_t> b(4 + n + ((4 - n % 4) % 4), 0);
    wr16(b.data(), it->second.channel);
    wr16(b.data() + 2, uint16_t(n));
    memcpy(b.data() + 4, p, n);
    raw_send(b.data(), b.size());
    return;
  }
  auto m = stun::Message::make(stun::kSendIndication);
  m.add_xor_addr(stun::kXorPeerAddress, peer);
  m.add(stun::kData, p, n);
  auto b = m.serialize(nullptr, false);
  raw_send(b.data(), b.size());
}

void TurnClient::on_packet(const uint8_t* p, size_t n) {
  if (closed_ || !agent_ || n < 4) return;
  if (p[0] >= 0x40 && p[0] <= 0x7F) {  // ChannelData
    uint16_t ch = rd16(p);
    uint16_t len = rd16(p + 2);
    if (size_t(len) + 4 > n) return;
    auto it = channels_.find(ch);
    if (it == channels_.end()) return;
    agent_->handle_datagram(-1, sock_, it->second, p + 4, len, true);
    return;
  }
  stun::Message m;
  if (!stun::Message::parse(p, n, m)) return;
  if (m.type == stun::kDataIndication) {
    SockAddr peer;
    const stun::Attr* data = m.get(stun::kData);
    if (data && m.get_xor_addr(stun::kXorPeerAddress, peer))
      agent_->handle_datagram(-1, sock_, peer, reinterpret_cast<const uint8_t*>(data->value.data()), data->value.size(),
                              true);
    return;
  }
  auto it = pending_.find(m.tid_key());
  if (it == pending_.end()) return;
  if (!key_.empty() && m.integrity_off >= 0 && !stun::verify_integrity(p, n, m, key_)) return;
  auto cb = std::move(it->second.cb);
  if (it->second.timer) r_.cancel(it->second.timer);
  pending_.erase(it);
  if (cb) cb(m, p, n);
}

}  // namespace p2pt::rtc
