#include "rtc/sctp.h"

#include <openssl/hmac.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "core/crypto.h"
#include "core/log.h"

namespace p2pt::rtc {

static const char* kT = "tunnel::sctp";

namespace {
enum : uint8_t {
  kData = 0,
  kInit = 1,
  kInitAck = 2,
  kSack = 3,
  kHeartbeat = 4,
  kHeartbeatAck = 5,
  kAbort = 6,
  kShutdown = 7,
  kShutdownAck = 8,
  kError = 9,
  kCookieEcho = 10,
  kCookieAck = 11,
  kShutdownComplete = 14,
  kReconfig = 130,
  kForwardTsn = 192,
};
constexpr size_t kCommonHdr = 12;
constexpr size_t kDataHdr = 16;

inline bool tsn_lt(uint32_t a, uint32_t b) { return int32_t(a - b) < 0; }
inline bool tsn_le(uint32_t a, uint32_t b) { return int32_t(a - b) <= 0; }

void put16(std::vector<uint8_t>& v, uint16_t x) {
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}
void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24));
  v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}
// n bytes appended at the end of v (capacity reserved by the caller: no
// reallocation on the per-chunk path), for direct stores.
inline uint8_t* grow(std::vector<uint8_t>& v, size_t n) {
  const size_t o = v.size();
  v.resize(o + n);
  return v.data() + o;
}
void pad4(std::vector<uint8_t>& v) {
  while (v.size() % 4) v.push_back(0);
}
}  // namespace

// A message body shared by its fragments: the body's buffer is referenced
// once per message, and the fragments count their uses here, on the
// association thread only. A per-chunk Bytes copy touched the buffer's atomic
// count ~110 times per 64 KB frame at 1200-byte packets, on a cache line the
// HTTP worker and the TX lane hold too (8-14 % of the association thread in
// _Sp_counted_base::_M_release, profiles/r03/prof_lanes).
struct SctpAssociation::BodyRef {
  Bytes body;
  uint32_t refs = 0;
};

// An outbound DATA fragment: a few inline bytes (the tunnel frame header)
// followed by a zero-copy slice of the message body. Pooled (chunk_free_): a
// frame in flight costs no heap allocation on the association thread.
struct SctpAssociation::Chunk {
  uint32_t tsn;
  uint16_t stream, ssn;
  uint32_t ppid;
  uint8_t flags;  // B=2, E=1, U=4
  uint8_t ilen = 0;
  uint8_t inl[SctpAssociation::kMsgHdrMax];
  BodyRef* ref = nullptr;  // body slice [poff, poff + plen), if any
  uint32_t poff = 0, plen = 0;
  size_t len;
  uint64_t sent_us = 0;
  int tx = 0;
  int miss = 0;
  bool acked = false;       // gap-acked
  bool in_flight = false;   // counted in flight_size_
  bool retransmit = false;  // marked for retransmission
  bool fast = false;        // marked by fast retransmit (may bypass cwnd once)
  bool probe = false;       // latest transmission was a tail-loss probe
  bool copied = false;      // a redundant copy went out (a duplicate report may be that copy's)
};

struct SctpAssociation::InChunk {
  uint32_t tsn;
  uint8_t flags;
  uint16_t stream;
  uint32_t ppid;
  Bytes data;
  uint16_t ssn;
  bool delivered;  // handed up early (stream-independent delivery); kept for TSN accounting
};

namespace {
constexpr size_t kInlineMax = 512;      // payload pieces below this are copied into the packet buffer
constexpr size_t kZeroCopyMin = 2048;   // received messages at least this big are delivered as views
}  // namespace

std::shared_ptr<SctpAssociation> SctpAssociation::create(Reactor& r, SctpConfig cfg, PacketOut out) {
  return std::shared_ptr<SctpAssociation>(new SctpAssociation(r, cfg, std::move(out)));
}

SctpAssociation::SctpAssociation(Reactor& r, SctpConfig cfg, PacketOut out) : r_(r), cfg_(cfg), out_(std::move(out)) {
  do {
    my_vtag_ = random_u32();
  } while (my_vtag_ == 0);
  my_init_tsn_ = random_u32();
  next_tsn_ = my_init_tsn_;
  cum_acked_ = my_init_tsn_ - 1;
  random_bytes(cookie_key_, sizeof cookie_key_);
  reconfig_seq_ = random_u32();
  rto_us_ = cfg_.rto_initial_ms * 1000;
  cwnd_ = cfg_.initial_cwnd ? cfg_.initial_cwnd : std::min<size_t>(4 * cfg_.mtu, std::max<size_t>(2 * cfg_.mtu, 4380));
  ssthresh_ = SIZE_MAX / 2;
  peer_rwnd_ = 0;
  pkt_.reserve(65536);
}

SctpAssociation::~SctpAssociation() {
  if (sack_timer_) r_.cancel(sack_timer_);
  if (t3_timer_) r_.cancel(t3_timer_);
  if (tlp_timer_) r_.cancel(tlp_timer_);
  if (init_timer_) r_.cancel(init_timer_);
  for (auto* c : inflight_) {
    if (c->ref) unref(c->ref);
    delete c;
  }
  for (auto* q : {&sendq_, &sendq_pri_})
    for (auto& m : *q)
      if (m.ref) unref(m.ref);
  for (auto* c : chunk_free_) delete c;
  for (auto* b : ref_free_) delete b;
  for (auto& kv : ooo_) delete kv.second;
}

SctpAssociation::BodyRef* SctpAssociation::new_ref(Bytes body) {
  BodyRef* b;
  if (ref_free_.empty()) {
    b = new BodyRef();
  } else {
    b = ref_free_.back();
    ref_free_.pop_back();
  }
  b->body = std::move(body);
  b->refs = 1;
  return b;
}

void SctpAssociation::unref(BodyRef* b) {
  if (--b->refs) return;
  b->body = Bytes();
  if (ref_free_.size() >= 4096) delete b;
  else ref_free_.push_back(b);
}

// TUNNEL_SCTP_CC: the congestion response. Unset: this build's (Veno-style
// random-loss cut to 80 %, CUBIC's 0.7 on congestion, the short-path queue
// bound). "reno": a Reno-like competitor for the shared-bottleneck fairness
// bench (every loss halves cwnd, no queue bound). "beta=NN": random-loss cut
// to NN % (50..100) (tuning runs).
const CcPolicy& cc_policy() {
  static const CcPolicy p = [] {
    CcPolicy c;
    const char* e = getenv("TUNNEL_SCTP_CC");
    if (!e || !*e) return c;
    const std::string v = e;
    if (v == "reno") {
      c.random_beta_pct = 50;
      c.queue_bound = false;
    } else if (v.rfind("beta=", 0) == 0) {
      c.random_beta_pct = std::clamp(atoi(v.c_str() + 5), 50, 100);
    }
    return c;
  }();
  return p;
}

SctpAssociation::Chunk* SctpAssociation::new_chunk() {
  if (chunk_free_.empty()) return new Chunk();
  Chunk* c = chunk_free_.back();
  chunk_free_.pop_back();
  return c;
}

void SctpAssociation::free_chunk(Chunk* c) {
  if (c->ref) unref(c->ref);
  c->ref = nullptr;
  if (chunk_free_.size() >= 8192) {
    delete c;
    return;
  }
  *c = Chunk();
  chunk_free_.push_back(c);
}

void SctpAssociation::set_mtu(size_t mtu) {
  cfg_.mtu = mtu;
  if (ssthresh_ < 4 * mtu) ssthresh_ = 4 * mtu;
}

// ------------------------------------------------------------------ output

void SctpAssociation::emit_packet(std::vector<uint8_t>& pkt) {
  // CRC32c over the packet with the checksum field zeroed, stored little-endian
  // (RFC 9260 App. B; same byte order as usrsctp / webrtc-rs).
  pkt[8] = pkt[9] = pkt[10] = pkt[11] = 0;
  uint32_t crc = crc32c(pkt.data(), pkt.size());
  pkt[8] = uint8_t(crc);
  pkt[9] = uint8_t(crc >> 8);
  pkt[10] = uint8_t(crc >> 16);
  pkt[11] = uint8_t(crc >> 24);
  stats_.packets_sent++;
  iovec v{pkt.data(), pkt.size()};
  if (out_) out_(&v, nullptr, 1);
}

void SctpAssociation::begin_gather() {
  if (pkt_.capacity() < cfg_.mtu + 64) pkt_.reserve(cfg_.mtu + 64);  // no pointers into pkt_ exist yet
  pkt_.clear();
  uint8_t* h = grow(pkt_, kCommonHdr);
  wr16(h, cfg_.local_port);
  wr16(h + 2, cfg_.remote_port);
  wr32(h + 4, peer_vtag_);
  wr32(h + 8, 0);
  iov_.clear();
  iov_own_.clear();
  run_start_ = 0;
  pkt_len_ = kCommonHdr;
}

void SctpAssociation::close_run() {
  if (pkt_.size() > run_start_) {
    iov_.push_back(iovec{pkt_.data() + run_start_, pkt_.size() - run_start_});
    iov_own_.push_back(nullptr);
  }
  run_start_ = pkt_.size();
}

// CRC32c over the gather list (checksum field zeroed), then hand it to DTLS.
void SctpAssociation::emit_gather() {
  close_run();
  pkt_[8] = pkt_[9] = pkt_[10] = pkt_[11] = 0;
  uint32_t crc = 0;
  // Both sides accept zero checksums over DTLS (RFC 9653): skip the pass.
  bool zero = cfg_.zero_checksum && peer_zero_checksum_ && state_ != State::CookieWait &&
              state_ != State::CookieEchoed && state_ != State::Closed;
  if (!zero)
    for (auto& v : iov_) crc = crc32c(v.iov_base, v.iov_len, crc);
  pkt_[8] = uint8_t(crc);
  pkt_[9] = uint8_t(crc >> 8);
  pkt_[10] = uint8_t(crc >> 16);
  pkt_[11] = uint8_t(crc >> 24);
  stats_.packets_sent++;
  if (out_) out_(iov_.data(), iov_own_.data(), int(iov_.size()));
}

static void begin_packet(std::vector<uint8_t>& pkt, uint16_t sport, uint16_t dport, uint32_t vtag) {
  pkt.clear();
  put16(pkt, sport);
  put16(pkt, dport);
  put32(pkt, vtag);
  put32(pkt, 0);
}

void SctpAssociation::send_control(uint8_t type, uint8_t flags, const std::vector<uint8_t>& body, uint32_t vtag) {
  std::vector<uint8_t> pkt;
  begin_packet(pkt, cfg_.local_port, cfg_.remote_port, vtag);
  pkt.push_back(type);
  pkt.push_back(flags);
  put16(pkt, uint16_t(4 + body.size()));
  pkt.insert(pkt.end(), body.begin(), body.end());
  pad4(pkt);
  emit_packet(pkt);
}

void SctpAssociation::queue_control(uint8_t type, uint8_t flags, std::vector<uint8_t> body) {
  std::vector<uint8_t> ch;
  ch.push_back(type);
  ch.push_back(flags);
  put16(ch, uint16_t(4 + body.size()));
  ch.insert(ch.end(), body.begin(), body.end());
  pad4(ch);
  ctrl_.push_back(std::move(ch));
}

void SctpAssociation::append_init_params(std::vector<uint8_t>& v) {
  // Supported Extensions: FORWARD-TSN (0xC0), RE-CONFIG (0x82).
  put16(v, 0x8008);
  put16(v, 6);
  v.push_back(0xC0);
  v.push_back(0x82);
  pad4(v);
  // Forward-TSN-Supported.
  put16(v, 0xC000);
  put16(v, 4);
  if (cfg_.zero_checksum) {  // Zero Checksum Acceptable, EDMID 1 = DTLS (RFC 9653 §4)
    put16(v, 0x8001);
    put16(v, 8);
    put32(v, 1);
  }
}

bool SctpAssociation::peer_offers_zero_checksum(const uint8_t* c, size_t len) const {
  for (size_t off = 0; off + 4 <= len;) {
    uint16_t pt = rd16(c + off), pl = rd16(c + off + 2);
    if (pl < 4 || off + pl > len) break;
    if (pt == 0x8001 && pl >= 8 && rd32(c + off + 4) == 1) return true;
    off += (pl + 3u) & ~3u;
  }
  return false;
}

void SctpAssociation::send_init() {
  std::vector<uint8_t> b;
  put32(b, my_vtag_);
  put32(b, cfg_.rwnd);
  put16(b, 65535);  // outbound streams
  put16(b, 65535);  // max inbound streams
  put32(b, my_init_tsn_);
  append_init_params(b);
  send_control(kInit, 0, b, 0);
}

void SctpAssociation::connect() {
  if (state_ != State::Closed) return;
  state_ = State::CookieWait;
  init_tries_ = 0;
  send_init();
  std::weak_ptr<SctpAssociation> w = shared_from_this();
  init_timer_ = r_.call_later_ms(cfg_.rto_initial_ms, [w] {
    if (auto s = w.lock()) s->on_init_timer();
  });
}

// INIT / COOKIE-ECHO retransmission with exponential backoff (RFC 9260 §5.1, T1).
void SctpAssociation::on_init_timer() {
  init_timer_ = 0;
  if (state_ != State::CookieWait && state_ != State::CookieEchoed) return;
  if (++init_tries_ > cfg_.max_init_retrans) {
    closed("SCTP association setup timed out");
    return;
  }
  if (state_ == State::CookieWait) send_init();
  else send_control(kCookieEcho, 0, cookie_echo_, peer_vtag_);
  uint64_t t = std::min<uint64_t>(cfg_.rto_initial_ms << std::min(init_tries_, 4), 5000);
  std::weak_ptr<SctpAssociation> w = shared_from_this();
  init_timer_ = r_.call_later_ms(t, [w] {
    if (auto s = w.lock()) s->on_init_timer();
  });
}

std::string SctpAssociation::make_cookie(uint32_t peer_tag, uint32_t peer_tsn, uint32_t peer_rwnd, uint16_t peer_os,
                                         uint16_t peer_mis, uint32_t peer_flags) {
  std::vector<uint8_t> c;
  put32(c, peer_tag);
  put32(c, peer_tsn);
  put32(c, peer_rwnd);
  put16(c, peer_os);
  put16(c, peer_mis);
  put32(c, my_vtag_);
  put32(c, peer_flags);
  uint64_t now = Reactor::now_ms();
  put32(c, uint32_t(now >> 32));
  put32(c, uint32_t(now));
  unsigned int len = 0;
  uint8_t mac[32];
  HMAC(EVP_sha256(), cookie_key_, sizeof cookie_key_, c.data(), c.size(), mac, &len);
  c.insert(c.end(), mac, mac + 32);
  return std::string(c.begin(), c.end());
}

// ------------------------------------------------------------------ input

void SctpAssociation::on_packet(const Bytes& pkt) {
  auto self = shared_from_this();  // callbacks below may drop the last outside reference
  packet_in(pkt);
}

// A receive burst under one reference (one shared_from_this per burst, not
// per packet: after a fragment's copy the reference count's locked update
// waited for the copy's stores, ~15 % of the association thread at 1200 MTU).
void SctpAssociation::on_packets(const Bytes* pkts, size_t n) {
  auto self = shared_from_this();
  for (size_t i = 0; i < n && !closed_fired_; i++) packet_in(pkts[i]);
}

void SctpAssociation::packet_in(const Bytes& pkt) {
  const uint8_t* p = pkt.data();
  size_t n = pkt.size();
  if (n < kCommonHdr + 4) return;
  uint32_t got = uint32_t(p[8]) | uint32_t(p[9]) << 8 | uint32_t(p[10]) << 16 | uint32_t(p[11]) << 24;
  if (!(cfg_.zero_checksum && got == 0)) {  // RFC 9653 §5.2: accept zero, verify anything else
    uint8_t hdr[kCommonHdr];
    memcpy(hdr, p, kCommonHdr);
    hdr[8] = hdr[9] = hdr[10] = hdr[11] = 0;
    // crc32c() chains: the header (checksum zeroed) then the chunks.
    uint32_t crc = crc32c(p + kCommonHdr, n - kCommonHdr, crc32c(hdr, kCommonHdr));
    if (crc != got) {
      LOG_TRACE(kT, "dropping SCTP packet with bad checksum");
      return;
    }
  }
  uint32_t vtag = rd32(p + 4);
  stats_.packets_received++;
  size_t off = kCommonHdr;
  bool first = true;
  uint64_t data_before = stats_.data_chunks_received;
  struct CountPkt {
    SctpAssociation* s;
    uint64_t before;
    ~CountPkt() {
      if (s->stats_.data_chunks_received != before) s->data_pkts_unacked_++;
    }
  } count_pkt{this, data_before};
  while (off + 4 <= n && !closed_fired_) {
    uint8_t type = p[off], flags = p[off + 1];
    size_t clen = rd16(p + off + 2);
    if (clen < 4 || off + clen > n) break;
    const uint8_t* body = p + off + 4;
    size_t blen = clen - 4;
    // Verification tag rules (RFC 9260 §8.5).
    bool ok_tag;
    if (type == kInit) ok_tag = first && vtag == 0;
    else if ((type == kAbort || type == kShutdownComplete) && (flags & 1)) ok_tag = vtag == peer_vtag_;
    else ok_tag = vtag == my_vtag_;
    if (!ok_tag) {
      LOG_TRACE(kT, "dropping chunk %u with bad verification tag", type);
      return;
    }
    switch (type) {
      case kData: handle_data(flags, body, blen, pkt); break;
      case kInit: handle_init(body, blen, vtag); break;
      case kInitAck: handle_init_ack(body, blen); break;
      case kSack: handle_sack(body, blen); break;
      case kHeartbeat: handle_heartbeat(body, blen); break;
      case kHeartbeatAck: break;
      case kAbort: closed("SCTP association aborted by peer"); return;
      case kShutdown: handle_shutdown(body, blen); break;
      case kShutdownAck:
        send_control(kShutdownComplete, 0, {}, peer_vtag_);
        closed("SCTP association shut down");
        return;
      case kShutdownComplete: closed("SCTP association shut down"); return;
      case kError: LOG_DEBUG(kT, "SCTP ERROR chunk from peer"); break;
      case kCookieEcho: handle_cookie_echo(body, blen); break;
      case kCookieAck:
        if (state_ == State::CookieEchoed) enter_established();
        break;
      case kForwardTsn: handle_forward_tsn(body, blen); break;
      case kReconfig: handle_reconfig(body, blen); break;
      default:
        // Unknown chunk: upper two bits say what to do (RFC 9260 §3.2).
        if ((type & 0xC0) == 0x00 || (type & 0xC0) == 0x40) return;  // stop processing packet
        break;
    }
    first = false;
    off += (clen + 3) & ~size_t(3);
  }
}

void SctpAssociation::handle_init(const uint8_t* c, size_t len, uint32_t) {
  if (len < 16) return;
  uint32_t tag = rd32(c), rwnd = rd32(c + 4);
  uint16_t os = rd16(c + 8), mis = rd16(c + 10);
  uint32_t tsn = rd32(c + 12);
  if (tag == 0) return;
  uint32_t flags = peer_offers_zero_checksum(c + 16, len - 16) ? 1 : 0;
  std::string cookie = make_cookie(tag, tsn, rwnd, os, mis, flags);
  std::vector<uint8_t> b;
  put32(b, my_vtag_);
  put32(b, cfg_.rwnd);
  put16(b, 65535);
  put16(b, 65535);
  put32(b, my_init_tsn_);
  append_init_params(b);
  put16(b, 0x0007);  // State Cookie
  put16(b, uint16_t(4 + cookie.size()));
  b.insert(b.end(), cookie.begin(), cookie.end());
  pad4(b);
  send_control(kInitAck, 0, b, tag);
}

void SctpAssociation::handle_init_ack(const uint8_t* c, size_t len) {
  if (state_ != State::CookieWait || len < 16) return;
  peer_vtag_ = rd32(c);
  uint32_t rwnd = rd32(c + 4);
  uint32_t tsn = rd32(c + 12);
  const uint8_t* cookie = nullptr;
  size_t cookie_len = 0;
  size_t off = 16;
  while (off + 4 <= len) {
    uint16_t pt = rd16(c + off), pl = rd16(c + off + 2);
    if (pl < 4 || off + pl > len) break;
    if (pt == 0x0007) {
      cookie = c + off + 4;
      cookie_len = pl - 4u;
    }
    off += (pl + 3u) & ~3u;
  }
  if (!cookie) return;
  peer_zero_checksum_ = peer_offers_zero_checksum(c + 16, len - 16);
  if (!have_peer_tsn_) {
    peer_cum_tsn_ = tsn - 1;
    have_peer_tsn_ = true;
  }
  peer_rwnd_ = rwnd;
  cookie_echo_.assign(cookie, cookie + cookie_len);
  state_ = State::CookieEchoed;
  send_control(kCookieEcho, 0, cookie_echo_, peer_vtag_);
}

void SctpAssociation::handle_cookie_echo(const uint8_t* c, size_t len) {
  constexpr size_t kBody = 32;  // tag, tsn, rwnd, os, mis, my tag, flags, time
  if (len != kBody + 32) return;
  unsigned int mlen = 0;
  uint8_t mac[32];
  HMAC(EVP_sha256(), cookie_key_, sizeof cookie_key_, c, kBody, mac, &mlen);
  if (memcmp(mac, c + kBody, 32) != 0) {
    LOG_DEBUG(kT, "invalid SCTP cookie");
    return;
  }
  uint32_t peer_tag = rd32(c), peer_tsn = rd32(c + 4), peer_rwnd = rd32(c + 8);
  uint32_t my_tag = rd32(c + 16);
  if (my_tag != my_vtag_) return;
  bool peer_zero = rd32(c + 20) & 1;
  if (state_ == State::Established || state_ == State::ShutdownPending) {
    if (peer_tag == peer_vtag_) queue_control(kCookieAck, 0, {});
    return;
  }
  peer_vtag_ = peer_tag;
  peer_zero_checksum_ = peer_zero;
  if (!have_peer_tsn_) {
    peer_cum_tsn_ = peer_tsn - 1;
    have_peer_tsn_ = true;
  }
  if (peer_rwnd_ == 0) peer_rwnd_ = peer_rwnd;
  queue_control(kCookieAck, 0, {});
  enter_established();
}

void SctpAssociation::enter_established() {
  if (state_ == State::Established) return;
  state_ = State::Established;
  if (init_timer_) r_.cancel(init_timer_);
  init_timer_ = 0;
  LOG_DEBUG(kT, "SCTP association established (mtu %zu, cwnd %zu)", cfg_.mtu, cwnd_);
  if (on_established) on_established();
}

void SctpAssociation::closed(const std::string& why) {
  if (closed_fired_) return;
  closed_fired_ = true;
  state_ = State::Closed;
  stop_t3();
  if (tlp_timer_) r_.cancel(tlp_timer_);
  tlp_timer_ = 0;
  if (init_timer_) r_.cancel(init_timer_);
  init_timer_ = 0;
  auto cb = std::move(on_closed);
  on_closed = nullptr;
  if (cb) cb(why);
}

void SctpAssociation::handle_heartbeat(const uint8_t* c, size_t len) {
  // The echo must fit one packet (the peer chose its size; flush() never
  // splits a chunk): oversized probes go unanswered.
  if (len + 4 + kCommonHdr > cfg_.mtu) return;
  queue_control(kHeartbeatAck, 0, std::vector<uint8_t>(c, c + len));
}

void SctpAssociation::handle_shutdown(const uint8_t*, size_t) {
  state_ = State::ShutdownReceived;
  maybe_finish_shutdown();
}

void SctpAssociation::maybe_finish_shutdown() {
  if (!sendq_.empty() || !sendq_pri_.empty() || !inflight_.empty()) return;
  if (state_ == State::ShutdownReceived) {
    state_ = State::ShutdownAckSent;
    send_control(kShutdownAck, 0, {}, peer_vtag_);
  } else if (state_ == State::ShutdownPending) {
    state_ = State::ShutdownSent;
    std::vector<uint8_t> b;
    put32(b, peer_cum_tsn_);
    send_control(kShutdown, 0, b, peer_vtag_);
  }
}

void SctpAssociation::shutdown() {
  if (state_ != State::Established) {
    closed("SCTP association closed");
    return;
  }
  state_ = State::ShutdownPending;
  maybe_finish_shutdown();
}

void SctpAssociation::abort(const std::string& reason) {
  if (peer_vtag_ && !closed_fired_) send_control(kAbort, 0, {}, peer_vtag_);
  closed(reason);
}

// Reassembly of one (possibly fragmented) message on stream `st`, fed in TSN
// order; delivers when the last fragment arrives. With a chain consumer
// (on_message_chain) the fragments' views are handed up as they are: no copy
// (the association thread spent 19-25 % of its time copying fragments of
// bulk frames at 1200-byte MTU, profiles/r03/bulk_threads). `d` is an owning
// view then; without a chain consumer fragments are copied as they come.
void SctpAssociation::deliver_chunk(uint8_t fl, uint16_t st, uint16_t ssn, uint32_t pp, const Bytes& d) {
  bool B = fl & 2, E = fl & 1, U = fl & 4;
  const uint8_t* dp = d.data();
  size_t dn = d.size();
  if (B && E) {
    deliver_message(st, ssn, U, pp, d);
    return;
  }
  Partial& pa = U ? partial_u_[st] : partial_[st];
  const bool chain = bool(on_message_chain);
  if (B) {
    pa.len = 0;
    pa.big.clear();
    pa.frags.clear();
    pa.frag_bytes = 0;
    pa.buf.reset();
    // Reassembled into a pooled buffer sized for a whole tunnel frame (one
    // copy per fragment, no reallocation, recycled once the message's views
    // are gone — possibly on a worker thread).
    if (!chain) pa.buf = reasm_pool_.get();
    pa.ppid = pp;
    pa.active = true;
  }
  if (!pa.active) return;  // middle fragment without a beginning (after FORWARD-TSN)
  if (chain) {
    pa.frags.push_back(d);
    pa.frag_bytes += dn;
  } else if (pa.big.empty() && pa.len + dn <= pa.buf->cap) {
    memcpy(pa.buf->data.get() + pa.len, dp, dn);
    pa.len += dn;
  } else {  // larger than any tunnel frame: fall back to a growing vector
    if (pa.big.empty()) pa.big.assign(pa.buf->data.get(), pa.buf->data.get() + pa.len);
    pa.big.insert(pa.big.end(), dp, dp + dn);
  }
  if (E) {
    pa.active = false;
    if (chain) {
      std::vector<Bytes> frags = std::move(pa.frags);
      pa.frags.clear();
      pa.frag_bytes = 0;
      Bytes first = std::move(frags.front());
      frags.erase(frags.begin());
      deliver_message(st, ssn, U, pa.ppid, std::move(first), std::move(frags));
      return;
    }
    Bytes msg = pa.big.empty() ? Bytes::adopt(pa.buf, pa.buf->data.get(), pa.len) : Bytes::take(std::move(pa.big));
    pa.buf.reset();
    pa.big.clear();
    pa.len = 0;
    deliver_message(st, ssn, U, pa.ppid, std::move(msg));
  }
}

void SctpAssociation::hand_up(uint16_t st, uint32_t pp, Bytes msg, std::vector<Bytes>& more) {
  if (!more.empty() && on_message_chain) {
    on_message_chain(st, pp, std::move(msg), more);
    return;
  }
  if (!more.empty()) {  // no chain consumer any more: one contiguous copy
    size_t total = msg.size();
    for (auto& b : more) total += b.size();
    std::vector<uint8_t> v;
    v.reserve(total);
    v.insert(v.end(), msg.data(), msg.data() + msg.size());
    for (auto& b : more) v.insert(v.end(), b.data(), b.data() + b.size());
    msg = Bytes::take(std::move(v));
  }
  if (on_message) on_message(st, pp, std::move(msg));
}

// Hands a complete message up and keeps the per-stream sequence (SSN) state;
// then releases any later single-chunk messages of that stream that arrived
// early (out of TSN order) and now are next in their stream's sequence.
void SctpAssociation::deliver_message(uint16_t st, uint16_t ssn, bool unordered, uint32_t pp, Bytes msg,
                                      std::vector<Bytes> more) {
  if (!unordered) {
    int16_t ahead = int16_t(uint16_t(ssn - next_ssn_in_[st]));
    if (ahead > 0) {  // an earlier message of this stream is still to come
      size_t n = msg.size();
      for (auto& b : more) n += b.size();
      held_bytes_ += n;
      held_[stream_ssn(st, ssn)] = Held{pp, std::move(msg), std::move(more)};
      return;
    }
    if (ahead < 0) return;  // already delivered
    next_ssn_in_[st] = uint16_t(ssn + 1);
    early_ready_.erase(stream_ssn(st, ssn));
  }
  hand_up(st, pp, std::move(msg), more);
  if (!unordered) release_ready(st);
}

// Delivers, in sequence, the messages of stream `st` that wait for their turn:
// held complete messages and early single-chunk ones still in the gap map.
void SctpAssociation::release_ready(uint16_t st) {
  for (;;) {
    const uint32_t key = stream_ssn(st, next_ssn_in_[st]);
    if (!held_.empty()) {
      auto h = held_.find(key);
      if (h != held_.end()) {
        Held m = std::move(h->second);
        held_.erase(h);
        size_t n = m.msg.size();
        for (auto& b : m.more) n += b.size();
        held_bytes_ -= n;
        early_ready_.erase(key);
        next_ssn_in_[st] = uint16_t(next_ssn_in_[st] + 1);
        hand_up(st, m.ppid, std::move(m.msg), m.more);
        continue;
      }
    }
    if (early_ready_.empty()) return;
    auto it = early_ready_.find(key);
    if (it == early_ready_.end()) return;
    auto oc = ooo_.find(it->second);
    early_ready_.erase(it);
    if (oc == ooo_.end() || oc->second->delivered) continue;
    InChunk* ic = oc->second;
    ic->delivered = true;
    ooo_bytes_ -= ic->data.size();
    Bytes m = std::move(ic->data);
    ic->data = Bytes();
    stats_.early_deliveries++;
    next_ssn_in_[st] = uint16_t(next_ssn_in_[st] + 1);
    if (on_message) on_message(st, ic->ppid, std::move(m));
  }
}

// Delivers the out-of-order chunks that became contiguous with the cumulative
// TSN (those already delivered early only advance it).
void SctpAssociation::drain_in_order() {
  while (!ooo_.empty()) {
    auto it = ooo_.find(peer_cum_tsn_ + 1);
    if (it == ooo_.end()) break;
    InChunk* ic = it->second;
    ooo_.erase(it);
    peer_cum_tsn_ = ic->tsn;
    if (!ic->delivered) {
      ooo_bytes_ -= ic->data.size();
      deliver_chunk(ic->flags, ic->stream, ic->ssn, ic->ppid, ic->data);
    }
    delete ic;
  }
}

void SctpAssociation::handle_data(uint8_t flags, const uint8_t* c, size_t len, const Bytes& pkt) {
  if (len < 12 || !have_peer_tsn_) return;
  uint32_t tsn = rd32(c);
  uint16_t stream = rd16(c + 4);
  uint16_t ssn = rd16(c + 6);
  uint32_t ppid = rd32(c + 8);
  const uint8_t* data = c + 12;
  size_t dlen = len - 12;
  stats_.data_chunks_received++;
  stats_.bytes_received += dlen;
  sack_needed_ = true;
  int32_t d = int32_t(tsn - peer_cum_tsn_);
  // Arrivals below the highest TSN seen: retransmissions filling holes, or
  // packets the path (or this stack) reordered — more of them than the peer
  // retransmitted means reordering.
  if (have_rx_high_ && d > 0 && tsn_lt(tsn, rx_high_tsn_)) stats_.late_tsns++;
  if (!have_rx_high_ || tsn_lt(rx_high_tsn_, tsn)) {
    rx_high_tsn_ = tsn;
    have_rx_high_ = true;
  }
  if (d <= 0) {
    stats_.dup_tsns++;
    if (dups_.size() < 32) dups_.push_back(tsn);
    return;
  }
  // A view of this chunk's payload: zero-copy for big payloads, a private
  // copy for small ones (or when the packet is not a view we may keep).
  // A fragment of a larger message is always a view when the packet has an
  // owner: the message pins its packets' buffers anyway.
  const bool whole = (flags & 3) == 3;
  auto hold = [&pkt, whole](const uint8_t* dp, size_t dn) {
    if ((dn >= kZeroCopyMin || !whole) && pkt.owner() && dp >= pkt.data() && dp + dn <= pkt.data() + pkt.size())
      return pkt.slice(size_t(dp - pkt.data()), dn);
    return slab_copy(dp, dn);  // packed with other small messages (core/buf.h)
  };
  if (d == 1) {
    peer_cum_tsn_ = tsn;
    // Fragments are copied on arrival unless the consumer takes chains, so a
    // non-owning view is enough then.
    deliver_chunk(flags, stream, ssn, ppid,
                  whole || on_message_chain ? hold(data, dlen) : Bytes::adopt(nullptr, data, dlen));
    drain_in_order();
    return;
  }
  if (ooo_.count(tsn)) {
    stats_.dup_tsns++;
    if (dups_.size() < 32) dups_.push_back(tsn);
    return;
  }
  if (ooo_bytes_ + dlen > cfg_.rwnd) {  // window exceeded: drop, peer retransmits
    stats_.rwnd_drops++;
    return;
  }
  auto* ic = new InChunk{tsn, flags, stream, ppid, hold(data, dlen), ssn, false};
  ooo_[tsn] = ic;
  ooo_bytes_ += dlen;
  // Stream-independent delivery (RFC 9260 §6.6: order is per stream): a
  // complete single-chunk message that is next in its own stream goes up now
  // instead of waiting behind a gap in another stream's TSNs — so a lost bulk
  // packet on one stream no longer holds back the tokens of the others.
  if ((flags & 3) == 3) {
    bool unordered = flags & 4;
    if (unordered || ssn == next_ssn_in_[stream]) {
      ic->delivered = true;
      ooo_bytes_ -= dlen;
      Bytes m = std::move(ic->data);
      ic->data = Bytes();
      stats_.early_deliveries++;
      deliver_message(stream, ssn, unordered, ppid, std::move(m));
    } else {
      early_ready_[stream_ssn(stream, ssn)] = tsn;
    }
  }
}

void SctpAssociation::build_sack(std::vector<uint8_t>& b) {
  size_t held = ooo_bytes_ + held_bytes_;
  for (auto& kv : partial_) held += kv.second.size();
  uint32_t a_rwnd = held >= cfg_.rwnd ? 0 : uint32_t(cfg_.rwnd - held);
  // Gap blocks relative to the cumulative TSN (ooo_ keys sorted numerically;
  // sort by serial distance to survive TSN wrap).
  std::vector<uint32_t> offs;
  offs.reserve(ooo_.size());
  for (auto& kv : ooo_) offs.push_back(kv.first - peer_cum_tsn_);
  std::sort(offs.begin(), offs.end());
  // As many blocks as fit in one packet beside the SACK's own headers (a
  // 1200-byte packet: ~290), the lowest first — they hold the holes to repair
  // next. A cap of 65 left every chunk held beyond the 65th block unreported:
  // still "in flight" at the sender, it filled cwnd and kept the known holes
  // from being retransmitted (hundreds of holes after a drop-tail queue
  // overflowed under slow start stalled a relayed 20 ms path for minutes).
  // Duplicate reports only tune the sender's spurious-loss undo: at most an
  // eighth of the room.
  const size_t room = (cfg_.mtu - kCommonHdr - 4 - 12) / 4;
  const size_t ndup = std::min(dups_.size(), room / 8);
  const size_t max_gaps = room - ndup;
  std::vector<std::pair<uint16_t, uint16_t>> gaps;
  for (uint32_t o : offs) {
    if (o > 0xFFFF) break;
    if (!gaps.empty() && uint32_t(gaps.back().second) + 1 == o) {
      gaps.back().second = uint16_t(o);
      continue;
    }
    if (gaps.size() == max_gaps) break;
    gaps.emplace_back(uint16_t(o), uint16_t(o));
  }
  put32(b, peer_cum_tsn_);
  put32(b, a_rwnd);
  put16(b, uint16_t(gaps.size()));
  put16(b, uint16_t(ndup));
  for (auto& g : gaps) {
    put16(b, g.first);
    put16(b, g.second);
  }
  for (size_t i = 0; i < ndup; i++) put32(b, dups_[i]);
  dups_.clear();
}

void SctpAssociation::update_rto(uint64_t r) {
  if (srtt_us_ == 0) {
    srtt_us_ = r;
    rttvar_us_ = r / 2;
  } else {
    uint64_t diff = srtt_us_ > r ? srtt_us_ - r : r - srtt_us_;
    rttvar_us_ = (3 * rttvar_us_ + diff) / 4;
    srtt_us_ = (7 * srtt_us_ + r) / 8;
  }
  uint64_t rto = srtt_us_ + std::max<uint64_t>(4 * rttvar_us_, 1000);
  // Leave room for a tail-loss probe and its SACK before T3: RTO >= PTO +
  // SRTT. With the 100 ms floor alone, a 50 ms path had RTO <= PTO, so every
  // tail loss went to T3 (cwnd collapse to one MTU, RTO doubling): 219 T3
  // expirations in one emulated 50 ms / 2 % loss run and a 2 s SSE stall tail.
  rto = std::max<uint64_t>(rto, 3 * srtt_us_ + cfg_.sack_delay_us);
  rto_us_ = std::clamp<uint64_t>(rto, cfg_.rto_min_ms * 1000, cfg_.rto_max_ms * 1000);
}

void SctpAssociation::handle_sack(const uint8_t* c, size_t len) {
  if (len < 12) return;
  uint32_t cum = rd32(c);
  uint32_t a_rwnd = rd32(c + 4);
  uint16_t ngap = rd16(c + 8), ndup = rd16(c + 10);
  if (len < 12 + 4u * ngap + 4u * ndup) return;
  stats_.sacks_received++;
  if (tsn_lt(cum, cum_acked_)) return;  // stale SACK
  uint64_t now = Reactor::now_us();
  size_t newly_acked = 0;
  size_t flight_before = flight_size_;
  bool cum_advanced = tsn_lt(cum_acked_, cum);
  // RTT: one sample per SACK from a chunk transmitted once (Karn): the
  // highest one the cumulative ack newly covers, else the first newly
  // gap-acked one. A cumulative ack that moved because a tail-loss probe
  // filled a hole gives no sample: the chunks behind the hole waited at the
  // peer for the probe (a tail repaired probe by probe inflated SRTT to
  // seconds, and the RTO and probe timers with it). Taking the newest chunk
  // of every SACK instead, and dropping every cumulative sample that covers
  // any retransmission, kept SRTT lower but tripled the SSE tail next to
  // bulk at 50 ms / 2 % loss (fewer losses read as congestion).
  uint64_t cum_sample = 0, gap_sample = 0;
  bool cum_probe = false;
  uint64_t newest_cum_sent = 0;
  // RACK evidence from a tail-loss probe (RFC 8985 §6.2, §7): an ack that
  // arrives at least one minimum RTT after the probe cannot be for an earlier
  // copy, so the probe was delivered and every chunk sent well before it that
  // is still unacknowledged is lost. (Ordinary retransmissions are not used:
  // behind a standing queue their acks are often the original's, and on a
  // 50 ms / 2 % path treating them as evidence tripled the SSE tail.)
  uint64_t rtx_delivered = 0;
  auto rtx_evidence = [&](const Chunk* ch) {
    if (ch->probe && min_rtt_us_ && now - ch->sent_us >= min_rtt_us_) rtx_delivered = std::max(rtx_delivered, ch->sent_us);
  };
  // The oldest once-sent chunk this SACK newly acknowledges: originals sent
  // before a probe and acknowledged with it show that the path (or a stalled
  // receiver) was slow, not lossy — the probe's ack is then most likely the
  // original's (a receiver asleep past the probe timeout SACKs its backlog in
  // order: the probed chunk, then the rest), and taking it as evidence marked
  // the whole window lost (hundreds of spurious marks per bulk run on the
  // MI355X host, profiles/r03/adaptive2_ab/bulk/fixed.std_{3,4}.json).
  uint64_t oldest_once_acked = UINT64_MAX;
  while (!inflight_.empty() && tsn_le(inflight_.front()->tsn, cum)) {
    Chunk* ch = inflight_.front();
    inflight_.pop_front();
    if (ch->in_flight) flight_size_ -= ch->len;
    if (ch->retransmit) rtx_.erase(ch->tsn);
    if (!ch->acked) {
      newly_acked += ch->len;
      if (ch->tx == 1) {
        cum_sample = now - ch->sent_us;
        newest_cum_sent = std::max(newest_cum_sent, ch->sent_us);
        oldest_once_acked = std::min(oldest_once_acked, ch->sent_us);
      } else {
        cum_probe |= ch->probe;
        rtx_evidence(ch);
      }
    }
    free_chunk(ch);
  }
  cum_acked_ = cum;
  // Gap blocks, processed in O(news): the peer repeats its blocks in every
  // SACK, so only the parts not already known to be acknowledged (gap_known_,
  // the previous SACK's blocks) are walked, by direct index into inflight_
  // (consecutive TSNs from the cumulative ack up). A 1 Gbit/s x 50 ms path
  // has ~5,000 chunks in flight; rescanning them per block was O(window x
  // blocks) per SACK.
  const uint32_t head = inflight_.empty() ? cum + 1 : inflight_.front()->tsn;
  auto at = [&](uint32_t tsn) -> Chunk* {
    uint32_t k = tsn - head;
    return k < inflight_.size() ? inflight_[k] : nullptr;
  };
  const uint32_t top = next_tsn_ - 1;  // highest TSN ever sent
  blocks_.clear();
  for (uint16_t i = 0; i < ngap; i++) {
    uint32_t s0 = cum + rd16(c + 12 + 4 * i), e0 = cum + rd16(c + 14 + 4 * i);
    if (rd16(c + 12 + 4 * i) == 0 || tsn_lt(e0, s0) || tsn_lt(top, s0)) continue;  // malformed / beyond what was sent
    if (tsn_lt(top, e0)) e0 = top;
    blocks_.emplace_back(s0, e0);
  }
  std::sort(blocks_.begin(), blocks_.end(), [cum](const auto& a, const auto& b) { return a.first - cum < b.first - cum; });
  uint32_t highest_gap = cum;
  size_t k = 0;  // cursor into gap_known_ (sorted, absolute TSNs)
  auto ack_range = [&](uint32_t a, uint32_t b) {
    for (uint32_t t = a;; t++) {
      if (Chunk* ch = at(t); ch && !ch->acked) {
        ch->acked = true;
        if (ch->retransmit) {
          ch->retransmit = false;
          rtx_.erase(ch->tsn);
        }
        if (ch->in_flight) {
          flight_size_ -= ch->len;
          ch->in_flight = false;
        }
        newly_acked += ch->len;
        if (ch->tx == 1) {
          if (!gap_sample) gap_sample = std::max<uint64_t>(now - ch->sent_us, 1);
          rack_xmit_us_ = std::max(rack_xmit_us_, ch->sent_us);
          oldest_once_acked = std::min(oldest_once_acked, ch->sent_us);
        } else {
          rtx_evidence(ch);
        }
      }
      if (t == b) break;
    }
  };
  for (auto& blk : blocks_) {
    if (tsn_lt(highest_gap, blk.second)) highest_gap = blk.second;
    uint32_t pos = blk.first;
    while (k < gap_known_.size() && tsn_lt(gap_known_[k].second, pos)) k++;
    while (tsn_le(pos, blk.second)) {
      if (k < gap_known_.size() && tsn_le(gap_known_[k].first, pos)) {  // known part: skip it
        if (tsn_le(blk.second, gap_known_[k].second)) break;
        pos = gap_known_[k].second + 1;
        k++;
        continue;
      }
      uint32_t end = blk.second;
      if (k < gap_known_.size() && tsn_le(gap_known_[k].first, blk.second)) end = gap_known_[k].first - 1;
      ack_range(pos, end);
      if (end == blk.second) break;
      pos = end + 1;
    }
  }
  gap_known_.swap(blocks_);
  if (rtx_delivered && oldest_once_acked < rtx_delivered) {
    rtx_delivered = 0;
    stats_.probe_ambiguous++;
  }
  // Duplicate TSN reports: copies the peer already had. A retransmission of
  // the current loss episode reported back this way was not needed — but only
  // a TSN this episode retransmitted counts, once: a duplicate of a redundant
  // copy (SctpConfig::dup_small) or of an earlier episode's retransmission says
  // nothing about this one's losses.
  if (ep_active_ && ndup && ep_rtx_ > 0) {
    const uint8_t* d = c + 12 + 4u * ngap;
    for (uint16_t i = 0; i < ndup && ep_rtx_ > 0; i++)
      if (ep_rtx_tsns_.erase(rd32(d + 4u * i))) ep_rtx_--;
  }
  if (cum_advanced && newest_cum_sent) rack_xmit_us_ = std::max(rack_xmit_us_, newest_cum_sent);
  const uint64_t rtt_sample = cum_sample && !cum_probe ? cum_sample : (cum_sample ? 0 : gap_sample);
  if (rtt_sample) {
    update_rto(rtt_sample);
    if (!min_rtt_us_ || rtt_sample < min_rtt_us_) min_rtt_us_ = rtt_sample;
  }
  // Loss detection. (1) Miss indications -> fast retransmit (RFC 9260
  // §7.2.4). (2) Time-based, after RACK (RFC 8985): a chunk still missing
  // although a chunk *sent* more than a quarter SRTT after it has been
  // acknowledged is lost — this also catches lost retransmissions and losses
  // in sparse traffic (credit frames, lone SSE tokens) where three miss
  // reports never come, which would otherwise wait for T3 (RTO >= 100 ms,
  // doubling, cwnd collapse to one MTU).
  // Only chunks transmitted once count as evidence: the acknowledgement of a
  // retransmitted chunk may be for its original copy (RFC 8985's ambiguity),
  // which would declare everything sent before the retransmission lost.
  // rack_xmit_us_ is the latest send time of an acknowledged once-sent chunk
  // (RACK.xmit_ts, monotonic), kept as acks arrive instead of rescanned.
  const uint64_t rack_sent = std::max(rack_xmit_us_, rtx_delivered);
  uint64_t reo = std::max<uint64_t>(srtt_us_ / 4, 1000);
  bool new_fast = false;
  size_t marked_now = 0;  // chunks this SACK declared lost
  auto mark = [&](Chunk* ch) {
    marked_now++;
    ch->miss = 0;
    ch->retransmit = true;
    rtx_.insert(ch->tsn);
    ch->fast = true;
    ch->probe = false;
    if (ch->in_flight) {
      flight_size_ -= ch->len;
      ch->in_flight = false;
    }
    new_fast = true;
    stats_.fast_retransmits++;
  };
  // (1) Only the holes below the highest gap-acked TSN can collect miss
  // indications: walk them (lost chunks), not the window.
  if (highest_gap != cum) {
    uint32_t pos = cum + 1;
    for (size_t b = 0; b <= gap_known_.size(); b++) {
      const uint32_t end = b < gap_known_.size() ? gap_known_[b].first - 1 : highest_gap - 1;
      for (uint32_t t = pos; tsn_le(t, end); t++) {
        Chunk* ch = at(t);
        if (!ch || ch->acked || ch->retransmit || ch->tx != 1) continue;
        // Fast retransmit at most once per chunk (RFC 9260 §7.2.4); a lost
        // retransmission is found by the time-based rule, a probe or T3.
        if (++ch->miss == 3) mark(ch);
      }
      if (b < gap_known_.size()) pos = gap_known_[b].second + 1;
    }
  }
  // (2) Transmissions in send order: everything sent more than `reo` before
  // rack_sent and still outstanding is lost; entries for chunks since
  // acknowledged or sent again are dropped on the way.
  while (!sendlog_.empty()) {
    const SendRec& f = sendlog_.front();
    Chunk* ch = tsn_lt(f.tsn, head) ? nullptr : at(f.tsn);
    const bool live = ch && ch->tx == f.tx && !ch->acked && !ch->retransmit;
    if (live) {
      if (!rack_sent || f.sent_us + reo >= rack_sent) break;
      stats_.rack_marks++;
      mark(ch);
    }
    sendlog_.pop_front();
  }
  if (cum_advanced) assoc_errors_ = 0;
  dr_on_sack(cum, newly_acked, flight_before + cfg_.mtu >= cwnd_, now);
  queue_bound(cum, rtt_sample);
  // Congestion control (RFC 9260 §7.2.1-7.2.2).
  const bool long_path = min_rtt_us_ >= kLongPathUs;
  // HyStart judges only rounds that fill cwnd, from kHsLowWindow packets on
  // (RFC 9406's low window): an app-limited sender's RTT says nothing about a
  // queue of its own. Small requests whose SACKs came back behind a download
  // queued the other way ended slow start at the initial window, and the next
  // upload then grew by a packet per round trip (profiles/r06/b14).
  const bool cwnd_limited = flight_before + cfg_.mtu >= cwnd_;
  if (cwnd_ <= ssthresh_ && !hs_done_ && long_path && !fast_recovery_ && cwnd_limited &&
      cwnd_ >= size_t(kHsLowWindow) * cfg_.mtu)
    hystart(cum, rtt_sample);
  if (newly_acked && cum_advanced && !fast_recovery_) {
    if (cwnd_ <= ssthresh_) {
      // Byte counting with RFC 3465's limit L = 2 MTUs per SACK on short
      // paths: the peer SACKs once per received batch, so one MTU per SACK
      // would make slow start nearly linear, while unbounded counting
      // overshoots a LAN bottleneck. On a long path a SACK covers a whole
      // burst (a hundred packets at 1 Gbit/s), and L = 2 MTUs took seconds to
      // open a 2.5 MB window (1 Gbit/s x 20 ms at 21 % of the rate over 64 MB):
      // there the whole acknowledged amount counts, and HyStart++ (RFC 9406,
      // hystart()) ends slow start on rising delay before the queue overflows.
      size_t grow = long_path ? newly_acked : std::min(newly_acked, 2 * cfg_.mtu);
      if (hs_css_) grow /= kCssDivisor;
      if (flight_before + cfg_.mtu >= cwnd_) cwnd_ += std::max<size_t>(grow, 1);
    } else {
      partial_acked_ += newly_acked;
      if (partial_acked_ >= cwnd_ && flight_before + cfg_.mtu >= cwnd_) {
        partial_acked_ -= cwnd_;
        // One MTU per round trip (RFC 9260 §7.2.2) while the path shows a
        // queue; with none, cwnd / 64 per round trip (Scalable TCP's rate):
        // after a random loss on a 1 Gbit/s x 20 ms path (2,000 packets of
        // BDP) one MTU per round trip would take 30 s to reopen the window.
        const uint64_t rtt = std::max<uint64_t>(srtt_us_, 1);
        const bool queue = min_rtt_us_ && rtt > min_rtt_us_ + rtt / 8;
        cwnd_ += queue ? cfg_.mtu : std::max(cfg_.mtu, cwnd_ / 64);
      }
    }
  }
  if (new_fast && !fast_recovery_) cwnd_bypass_ = 1;
  if (new_fast && !fast_recovery_) {
    hs_done_ = true;  // HyStart++ covers only the initial slow start
    // Loss response after TCP Veno: the backlog this association keeps in the
    // path's queues is cwnd * (SRTT - min RTT) / SRTT. A loss with (almost) no
    // backlog is taken as random (wireless, lossy WAN) and keeps cwnd (below);
    // a loss with a standing queue is congestion and cuts by 0.3 (CUBIC's
    // beta, RFC 9438) rather than Reno's half.
    uint64_t rtt = std::max<uint64_t>(srtt_us_, 1);
    size_t backlog = min_rtt_us_ && rtt > min_rtt_us_ ? size_t(double(cwnd_) * double(rtt - min_rtt_us_) / double(rtt)) : 0;
    // Random loss also means isolated loss: a policer or a shallow drop-tail
    // queue overrun by cwnd drops a run of packets with no standing queue in
    // front of it, which is congestion all the same.
    // And a window already past what the path has delivered in recent rounds
    // (1.125 x max delivery rate x min RTT) is overrunning a bottleneck whose
    // queue is too shallow to show as delay: congestion too. A random loss
    // leaves delivery rising with cwnd (emulated 20 ms, 40 Mbit/s behind a
    // 6 KiB queue: 3-6 % of packets dropped while such losses kept cwnd).
    const size_t bdp = dr_bdp();
    const bool over_bdp = bdp && cwnd_ > bdp + bdp / 8 + 2 * cfg_.mtu;
    // "Isolated": at most 2 chunks, or 1 % of the window, newly found lost
    // by this SACK (at 0.5 % random loss a 1 Gbit/s x 20 ms window loses
    // several chunks per round trip, and reading that as congestion held bulk
    // near 10 % of the link).
    const size_t isolated = std::max<size_t>(2, flight_before / (100 * cfg_.mtu));
    bool random_loss = backlog < 3 * cfg_.mtu + cwnd_ / 8 && marked_now <= isolated && !over_bdp;
    if (!(random_loss && random_episode_)) loss_response(random_loss, over_bdp, now);
  }
  if (fast_recovery_ && !tsn_lt(cum, fast_recovery_exit_)) fast_recovery_ = false;
  if (random_episode_ && !tsn_lt(cum, random_exit_)) random_episode_ = false;
  if (ep_active_ && !tsn_lt(cum, ep_exit_)) {
    ep_active_ = false;
    ep_rtx_tsns_.clear();
    if (ep_rtx_ == 0 && ep_undo_cwnd_ > cwnd_) {  // nothing it marked was lost: undo the cut
      cwnd_ = ep_undo_cwnd_;
      ssthresh_ = std::max(ssthresh_, ep_undo_ssthresh_);
      fast_recovery_ = false;
      stats_.spurious_undos++;
    }
  }
  peer_rwnd_ = a_rwnd > flight_size_ ? a_rwnd - flight_size_ : 0;
  if (cum_advanced) tlp_count_ = 0;
  if (inflight_.empty()) {
    stop_t3();
    if (tlp_timer_) r_.cancel(tlp_timer_);
    tlp_timer_ = 0;
  } else if (cum_advanced) {
    start_t3();
    arm_tlp();
  }
  maybe_finish_shutdown();
}

// A new loss episode: cwnd and ssthresh after it (handle_sack classified it).
void SctpAssociation::loss_response(bool random_loss, bool over_bdp, uint64_t now) {
  if (random_loss) stats_.random_loss_events++;
  // A random loss (no standing queue) cuts cwnd by a fifth
  // (TUNNEL_SCTP_CC=beta=NN, default 80: Veno's random-loss beta), at
  // most once per round trip; losses with a backlog cut by 0.3 (CUBIC).
  // Measured against a Reno-like flow on one shared bottleneck
  // (bench/bench_fairness.py: 0.5 % loss, 20 ms), keeping cwnd on random loss
  // (round 3's default, with a 0.85 cut every 8th episode in a row) took 3.8x
  // (50 Mbit/s) and 5.1x (200 Mbit/s) the Reno flow's throughput
  // (profiles/r04/fairness/): an AIMD flow that ignores loss is unfair to
  // every flow that does not (RFC 5033). With a cut of b per loss episode and
  // one MTU per round trip of growth, throughput scales as
  // sqrt((2 - b) / (2 b p)) against Reno's sqrt(1.5 / p): b = 0.2 is 1.7x
  // Reno, within the 2x bound; the cost is bulk on paths with genuinely
  // random loss.
  const int random_beta_pct = cfg_.random_beta_pct >= 0 ? std::clamp(cfg_.random_beta_pct, 50, 100)
                                                        : cc_policy().random_beta_pct;
  last_loss_us_ = now;
  size_t keep = cwnd_ * 7 / 10;
  if (random_loss) {
    keep = cwnd_ * size_t(random_beta_pct) / 100;
    if (random_beta_pct < 100) stats_.random_loss_cuts++;
  } else {
    stats_.congestion_cuts++;
    if (over_bdp) stats_.over_bdp_losses++;
  }
  if (!ep_active_) {
    ep_active_ = true;
    ep_undo_cwnd_ = cwnd_;
    ep_undo_ssthresh_ = ssthresh_;
    ep_rtx_ = 0;
    ep_rtx_tsns_.clear();
  }
  ep_exit_ = next_tsn_ - 1;
  ssthresh_ = std::max(keep, 4 * cfg_.mtu);
  cwnd_ = ssthresh_;
  partial_acked_ = 0;
  if (random_loss) {
    // No recovery period: cwnd keeps growing while the losses are repaired
    // (at 0.5 % loss and 1 Gbit/s a new loss comes every few ms, so a
    // recovery period per loss froze cwnd for good). Further losses within
    // this window's round trip are the same episode.
    random_episode_ = true;
    random_exit_ = next_tsn_ - 1;
  } else {
    fast_recovery_ = true;
    fast_recovery_exit_ = next_tsn_ - 1;
    random_episode_ = false;
  }
}

// Tail-loss probe (after RFC 8985 TLP): with data outstanding and no SACK for
// ~2 SRTT, retransmit the oldest unacknowledged chunk. The probe's SACK
// either acknowledges it or exposes the gaps for the time-based detection,
// instead of waiting for T3. Up to two probes per episode; no cwnd change.
void SctpAssociation::arm_tlp() {
  if (tlp_timer_) r_.cancel(tlp_timer_);
  tlp_timer_ = 0;
  if (inflight_.empty() || tlp_count_ >= 2 || !srtt_us_) return;
  uint64_t pto = std::max<uint64_t>(2 * srtt_us_ + cfg_.sack_delay_us, 10000);
  if (pto >= rto_us_) return;  // T3 comes first anyway
  std::weak_ptr<SctpAssociation> w = shared_from_this();
  tlp_timer_ = r_.call_later_us(pto, [w] {
    if (auto s = w.lock()) {
      s->tlp_timer_ = 0;
      s->on_tlp();
    }
  });
}

void SctpAssociation::on_tlp() {
  // Holes already known lost but held back by a full cwnd come first: the
  // probe repairs the oldest one, so the cumulative ack moves and frees the
  // window (re-sending a chunk the peer already holds would not).
  if (!rtx_.empty()) {
    const uint32_t k = *rtx_.begin() - (inflight_.empty() ? 0 : inflight_.front()->tsn);
    if (k < inflight_.size()) {
      Chunk* ch = inflight_[k];
      if (ch->retransmit && !ch->acked) {
        ch->fast = true;
        ch->probe = true;
        tlp_count_++;
        stats_.tlp_probes++;
        cwnd_bypass_ = 1;
        start_t3();
        return;
      }
    }
  }
  for (Chunk* ch : inflight_) {
    if (ch->acked || ch->retransmit) continue;
    ch->retransmit = true;
    rtx_.insert(ch->tsn);
    ch->fast = true;  // may go out even when cwnd is full
    ch->probe = true;
    if (ch->in_flight) {
      flight_size_ -= ch->len;
      ch->in_flight = false;
    }
    tlp_count_++;
    stats_.tlp_probes++;
    cwnd_bypass_ = 1;
    // Re-arm T3 from the probe (RFC 8985 §7.3): its acknowledgement, one
    // round trip away, either repairs the tail or exposes the rest of it to
    // RACK. Left running from the last cumulative ack, T3 expired before that
    // ack could arrive whenever cwnd had shrunk to a few packets (2 % loss,
    // bursts behind a token trickle): cwnd to one MTU and RTO doubled for a
    // loss the probe was already repairing.
    start_t3();
    break;  // flush() at the end of this iteration sends it
  }
}

void SctpAssociation::handle_forward_tsn(const uint8_t* c, size_t len) {
  if (len < 4) return;
  uint32_t nc = rd32(c);
  sack_needed_ = true;
  if (!tsn_lt(peer_cum_tsn_, nc)) return;
  for (auto it = ooo_.begin(); it != ooo_.end();) {
    if (tsn_le(it->first, nc)) {
      if (!it->second->delivered) ooo_bytes_ -= it->second->data.size();
      delete it->second;
      it = ooo_.erase(it);
    } else {
      ++it;
    }
  }
  peer_cum_tsn_ = nc;
  for (auto& kv : partial_u_) kv.second.active = false;
  for (auto it = early_ready_.begin(); it != early_ready_.end();) {
    if (!ooo_.count(it->second)) it = early_ready_.erase(it);
    else ++it;
  }
  drain_in_order();  // continue delivery of anything now contiguous
}

void SctpAssociation::handle_reconfig(const uint8_t* c, size_t len) {
  size_t off = 0;
  while (off + 4 <= len) {
    uint16_t pt = rd16(c + off), pl = rd16(c + off + 2);
    if (pl < 4 || off + pl > len) break;
    if (pt == 13 && pl >= 16) {  // Outgoing SSN Reset Request
      uint32_t req_seq = rd32(c + off + 4);
      std::vector<uint16_t> streams;
      for (size_t k = 16; k + 2 <= pl; k += 2) streams.push_back(rd16(c + off + k));
      std::vector<uint8_t> b;
      put16(b, 16);  // Re-configuration Response
      put16(b, 12);
      put32(b, req_seq);
      put32(b, 1);  // Success - Performed
      queue_control(kReconfig, 0, b);
      for (uint16_t s : streams) {
        reset_inbound_stream(s);
        if (on_stream_reset) on_stream_reset(s);
      }
    }
    off += (pl + 3u) & ~3u;
  }
}

// The peer reset its outgoing stream `st` (RFC 6525 §5.2.2): it restarts at
// SSN 0, so every piece of per-stream receive state goes — a partial message
// (ordered or not), the expected SSN, and complete messages held or marked
// early for their turn — or the restarted stream's messages would be dropped
// as already delivered or held forever.
void SctpAssociation::reset_inbound_stream(uint16_t st) {
  partial_.erase(st);
  partial_u_.erase(st);
  next_ssn_in_.erase(st);
  const uint32_t lo = stream_ssn(st, 0), hi = stream_ssn(st, 0xFFFF);
  for (auto it = held_.lower_bound(lo); it != held_.end() && it->first <= hi;) {
    held_bytes_ -= it->second.msg.size();
    for (auto& b : it->second.more) held_bytes_ -= b.size();
    it = held_.erase(it);
  }
  early_ready_.erase(early_ready_.lower_bound(lo), early_ready_.upper_bound(hi));
}

void SctpAssociation::request_stream_reset(uint16_t stream) {
  if (state_ != State::Established) return;
  std::vector<uint8_t> b;
  put16(b, 13);
  put16(b, 18);
  put32(b, reconfig_seq_++);
  put32(b, 0);
  put32(b, next_tsn_ - 1);
  put16(b, stream);
  pad4(b);
  queue_control(kReconfig, 0, b);
  next_ssn_.erase(stream);  // the stream restarts at SSN 0 (RFC 6525 §5.1.2)
}

// ------------------------------------------------------------------ sender

bool SctpAssociation::send(uint16_t stream, uint32_t ppid, const std::vector<Bytes>& pieces, bool unordered) {
  if (closed_fired_ || state_ == State::ShutdownPending || state_ == State::ShutdownSent) return false;
  Msg m;
  m.stream = stream;
  m.ppid = ppid;
  m.unordered = unordered;
  m.len = 0;
  for (auto& p : pieces) m.len += p.size();
  if (m.len == 0) return false;
  // Generic gather list: one contiguous copy unless it is a single piece.
  if (pieces.size() == 1) {
    m.body = pieces[0];
  } else {
    std::vector<uint8_t> v;
    v.reserve(m.len);
    for (auto& p : pieces) v.insert(v.end(), p.begin(), p.end());
    m.body = Bytes::take(std::move(v));
  }
  m.ssn = unordered ? 0 : next_ssn_[stream]++;
  unsent_bytes_ += m.len;
  sendq_.push_back(std::move(m));
  return true;
}

bool SctpAssociation::send_framed(uint16_t stream, uint32_t ppid, const uint8_t* hdr, size_t hlen, const Bytes& payload,
                                  bool unordered, bool priority) {
  if (closed_fired_ || state_ == State::ShutdownPending || state_ == State::ShutdownSent) return false;
  if (hlen > kMsgHdrMax) return send(stream, ppid, {Bytes::copy(hdr, hlen), payload}, unordered);
  Msg m;
  m.stream = stream;
  m.ppid = ppid;
  m.unordered = unordered;
  memcpy(m.hdr, hdr, hlen);
  m.hlen = uint8_t(hlen);
  m.body = payload;
  m.len = hlen + payload.size();
  if (m.len == 0) return false;
  m.ssn = unordered ? 0 : next_ssn_[stream]++;
  unsent_bytes_ += m.len;
  // Priority only for messages of one DATA chunk: a message's fragments must
  // carry consecutive TSNs, so a message is never split around another.
  if (priority && m.len <= cfg_.mtu - kCommonHdr - kDataHdr) sendq_pri_.push_back(std::move(m));
  else sendq_.push_back(std::move(m));
  return true;
}

// HyStart++ (RFC 9406) for the initial slow start on long paths: per round
// (one window's worth of TSNs), the minimum RTT of at least kHsSamples
// samples; once it exceeds the previous round's by clamp(prev / 8, 4 ms,
// 16 ms) the queue is building: growth drops to a quarter (conservative slow
// start) for kCssRounds rounds, then congestion avoidance takes over with
// ssthresh = cwnd. A round whose minimum falls back below the CSS baseline
// was a false alarm and resumes slow start.
void SctpAssociation::dr_on_sack(uint32_t cum, size_t newly_acked, bool cwnd_limited, uint64_t now) {
  if (!dr_active_) {
    if (!newly_acked) return;
    dr_active_ = true;
    dr_end_ = next_tsn_ - 1;
    dr_start_us_ = now;
    dr_bytes_ = 0;
    dr_limited_ = cwnd_limited;
    return;
  }
  dr_bytes_ += newly_acked;
  dr_limited_ = dr_limited_ || cwnd_limited;
  if (tsn_lt(cum, dr_end_)) return;
  // Round over: app-limited rounds (the sender never filled cwnd) say nothing
  // about the path and are not recorded.
  if (dr_limited_ && now > dr_start_us_) {
    dr_rates_[dr_next_] = dr_bytes_ * 1000000 / (now - dr_start_us_);
    dr_next_ = (dr_next_ + 1) % kDrRounds;
  }
  dr_end_ = next_tsn_ - 1;
  dr_start_us_ = now;
  dr_bytes_ = 0;
  dr_limited_ = cwnd_limited;
}

// Short-path queue bound. On a LAN or same-host path nothing limits cwnd but
// the peer's window, so a bulk transfer keeps megabytes standing in the socket
// buffers and crypto lanes, and an SSE token sent behind it waits for all of
// them: on the MI355X host the mixed row's SSE TTFT p50 was 1.0-1.4 ms next to
// bulk (direct 0.13-0.27 ms), the SCTP SRTT 1-2.5 ms over a 50 us path. Per
// round trip the smallest RTT sample, less the base RTT (the smallest sample
// of the last 5-10 s), is the standing queue; above the target it takes cwnd
// down by a quarter (and ends slow start), never below the floor. WAN paths (base RTT >=
// kLongPathUs) keep the loss-based response alone, as do paths whose queue
// stays under the target.
void SctpAssociation::note_interactive() { interactive_until_us_ = Reactor::now_us() + 200000; }

void SctpAssociation::queue_bound(uint32_t cum, uint64_t rtt_sample) {
  if (!cc_policy().queue_bound) return;
  constexpr uint64_t target_bulk = 300, target_inter = 150;
  constexpr size_t floor_bulk = 1024 * 1024, floor_inter = 512 * 1024;
  // Two settings: bulk alone keeps a 300 us / 1 MiB bound (64 x 1 MB echo on
  // the MI355X host unchanged by tighter ones, -15 % in the build container);
  // while interactive frames flow (note_interactive) 150 us / 512 KiB:
  // mixed-row SSE TTFT p99 1.28 -> 0.91 ms jumbo, 1.20 -> 0.91 ms at 1200 MTU,
  // token crossing 205-224 -> 126-132 us p50, for 15-21 % of the bulk next to
  // it (profiles/r03/floor512_ab/).
  const bool inter = Reactor::now_us() < interactive_until_us_;
  const uint64_t target_us = inter ? target_inter : target_bulk;
  const size_t floor_bytes = inter ? floor_inter : floor_bulk;
  if (rtt_sample) {
    qb_min_ = std::min(qb_min_, rtt_sample);
    const uint64_t now = Reactor::now_us();
    if (!qb_base_t0_ || now - qb_base_t0_ > 5000000) {
      qb_base_prev_ = qb_base_cur_;
      qb_base_cur_ = UINT64_MAX;
      qb_base_t0_ = now;
    }
    qb_base_cur_ = std::min(qb_base_cur_, rtt_sample);
  }
  if (!qb_active_) {
    qb_active_ = true;
    qb_end_ = next_tsn_ - 1;
    qb_min_ = UINT64_MAX;
    return;
  }
  if (tsn_lt(cum, qb_end_)) return;
  const uint64_t round_min = qb_min_;
  qb_end_ = next_tsn_ - 1;
  qb_min_ = UINT64_MAX;
  if (round_min == UINT64_MAX) return;
  qb_last_ = round_min;
  const uint64_t base = std::min(qb_base_cur_, qb_base_prev_);
  if (!target_us || base == UINT64_MAX || base >= kLongPathUs) return;
  if (round_min <= base + target_us || cwnd_ <= floor_bytes) return;
  cwnd_ = std::max(floor_bytes, cwnd_ - cwnd_ / 4);
  ssthresh_ = std::min(ssthresh_, cwnd_);
  partial_acked_ = 0;
  stats_.queue_cuts++;
}

size_t SctpAssociation::dr_bdp() const {
  uint64_t mx = 0;
  for (uint64_t r : dr_rates_) mx = std::max(mx, r);
  if (!mx || !min_rtt_us_) return 0;
  return size_t(mx * min_rtt_us_ / 1000000);
}

void SctpAssociation::hystart(uint32_t cum, uint64_t rtt_sample) {
  if (!hs_round_ || !tsn_lt(cum, hs_window_end_)) {  // a round ended
    hs_last_min_ = hs_cur_min_;
    hs_cur_min_ = UINT64_MAX;
    hs_samples_ = 0;
    hs_window_end_ = next_tsn_ - 1;
    hs_round_ = true;
    if (hs_css_ && ++hs_css_rounds_ >= kCssRounds) {
      hs_css_ = false;
      hs_done_ = true;
      ssthresh_ = cwnd_;
      stats_.hystart_exits++;
      return;
    }
  }
  if (rtt_sample) {
    hs_cur_min_ = std::min(hs_cur_min_, rtt_sample);
    hs_samples_++;
  }
  if (hs_samples_ < kHsSamples || hs_cur_min_ == UINT64_MAX || hs_last_min_ == UINT64_MAX) return;
  if (!hs_css_) {
    const uint64_t thresh = std::clamp<uint64_t>(hs_last_min_ / 8, 4000, 16000);
    if (hs_cur_min_ >= hs_last_min_ + thresh) {
      hs_css_ = true;
      hs_css_base_ = hs_cur_min_;
      hs_css_rounds_ = 0;
    }
  } else if (hs_cur_min_ < hs_css_base_) {
    hs_css_ = false;  // spurious: back to slow start
  }
}

void SctpAssociation::start_t3() {
  stop_t3();
  std::weak_ptr<SctpAssociation> w = shared_from_this();
  t3_timer_ = r_.call_later_us(rto_us_, [w] {
    if (auto s = w.lock()) {
      s->t3_timer_ = 0;
      s->on_t3();
    }
  });
}

void SctpAssociation::stop_t3() {
  if (t3_timer_) r_.cancel(t3_timer_);
  t3_timer_ = 0;
}

void SctpAssociation::on_t3() {
  if (inflight_.empty()) return;
  stats_.t3_expirations++;
  ep_active_ = false;  // a timeout is no spurious episode to undo
  if (++assoc_errors_ > cfg_.max_assoc_retrans) {
    abort("SCTP: too many retransmissions");
    return;
  }
  ssthresh_ = std::max(cwnd_ / 2, 4 * cfg_.mtu);
  cwnd_ = cfg_.mtu;
  partial_acked_ = 0;
  fast_recovery_ = false;
  random_episode_ = false;
  hs_done_ = true;
  hs_css_ = false;
  rto_us_ = std::min<uint64_t>(rto_us_ * 2, cfg_.rto_max_ms * 1000);
  for (Chunk* ch : inflight_) {
    if (ch->acked) continue;
    ch->retransmit = true;
    rtx_.insert(ch->tsn);
    ch->fast = false;
    ch->probe = false;
    if (ch->in_flight) {
      flight_size_ -= ch->len;
      ch->in_flight = false;
    }
  }
  LOG_DEBUG(kT, "T3-rtx expired: rto %llu ms, %zu chunks outstanding",
            static_cast<unsigned long long>(rto_us_ / 1000), inflight_.size());
  // flush() runs at the end of this reactor iteration and retransmits.
}

void SctpAssociation::flush() {
  if (closed_fired_) return;
  auto self = shared_from_this();
  bool can_data = state_ == State::Established || state_ == State::ShutdownPending ||
                  state_ == State::ShutdownReceived;
  if (!can_data && ctrl_.empty()) return;
  const size_t mtu = cfg_.mtu;
  size_t max_payload = mtu - kCommonHdr - kDataHdr;
  begin_gather();
  auto flush_pkt = [&] {
    if (pkt_len_ > kCommonHdr) emit_gather();
    begin_gather();
  };
  auto add_raw = [&](const std::vector<uint8_t>& ch) {
    if (pkt_len_ + ch.size() > mtu) flush_pkt();
    pkt_.insert(pkt_.end(), ch.begin(), ch.end());
    pkt_len_ += ch.size();
  };
  // SACK policy: immediate when >= 2 data packets are unacknowledged, on
  // gaps/duplicates, or when DATA goes out now anyway (piggyback); otherwise
  // delayed by sack_delay_us so a lone request frame is acknowledged by the
  // response that follows instead of by a pure SACK (one less wakeup per
  // request on each side). RFC 9260 §6.2 allows up to 500 ms.
  bool data_ready = can_data && (!sendq_.empty() || !sendq_pri_.empty() || !rtx_.empty());
  bool sack_now = sack_needed_ && (sack_urgent_ || data_pkts_unacked_ >= 2 || data_ready || cfg_.sack_delay_us == 0 ||
                                   !ooo_.empty() || !dups_.empty());
  if (sack_needed_ && !sack_now && !sack_timer_) {
    std::weak_ptr<SctpAssociation> w = shared_from_this();
    sack_timer_ = r_.call_later_us(cfg_.sack_delay_us, [w] {
      if (auto s = w.lock()) {
        s->sack_timer_ = 0;
        s->sack_urgent_ = true;  // flushed at the end of this reactor iteration
      }
    });
  }
  if (sack_now && have_peer_tsn_ && peer_vtag_) {
    if (sack_timer_) r_.cancel(sack_timer_);
    sack_timer_ = 0;
    sack_urgent_ = false;
    data_pkts_unacked_ = 0;
    std::vector<uint8_t> b;
    build_sack(b);
    std::vector<uint8_t> ch;
    ch.push_back(kSack);
    ch.push_back(0);
    put16(ch, uint16_t(4 + b.size()));
    ch.insert(ch.end(), b.begin(), b.end());
    add_raw(ch);
    sack_needed_ = false;
    stats_.sacks_sent++;
  }
  for (auto& ch : ctrl_) add_raw(ch);
  ctrl_.clear();
  if (!can_data) {
    flush_pkt();
    return;
  }
  uint64_t now = Reactor::now_us();
  auto add_data = [&](Chunk* ch, bool copy) {
    size_t padded = (ch->len + 3) & ~size_t(3);
    size_t need = kDataHdr + padded;
    if (pkt_len_ + need > mtu) flush_pkt();
    std::vector<uint8_t>& pkt = pkt_;
    uint8_t* h = grow(pkt, kDataHdr);  // one store sequence per header (12 push_backs were a hot spot)
    h[0] = kData;
    h[1] = ch->flags;
    wr16(h + 2, uint16_t(kDataHdr + ch->len));
    wr32(h + 4, ch->tsn);
    wr16(h + 8, ch->stream);
    wr16(h + 10, ch->ssn);
    wr32(h + 12, ch->ppid);
    // Inline header bytes and small pieces are copied into the packet buffer;
    // large pieces are referenced in place (the chunk keeps its slices alive
    // until acknowledged).
    pkt.insert(pkt.end(), ch->inl, ch->inl + ch->ilen);
    if (ch->ref) {
      const uint8_t* pd = ch->ref->body.data() + ch->poff;
      if (ch->plen < kInlineMax) {
        pkt.insert(pkt.end(), pd, pd + ch->plen);
      } else {
        close_run();
        iov_.push_back(iovec{const_cast<uint8_t*>(pd), ch->plen});
        iov_own_.push_back(&ch->ref->body);
      }
    }
    pkt.insert(pkt.end(), padded - ch->len, 0);
    pkt_len_ += need;
    if (copy) {  // redundant copy: bytes on the wire only, no sender state
      ch->copied = true;
      ep_rtx_tsns_.erase(ch->tsn);
      stats_.dup_copies_sent++;
      return;
    }
    ch->sent_us = now;
    ch->tx++;
    sendlog_.push_back(SendRec{ch->tsn, ch->tx, now});
    if (!ch->in_flight) {
      ch->in_flight = true;
      flight_size_ += ch->len;
    }
    stats_.data_chunks_sent++;
    stats_.bytes_sent += ch->len;
  };
  // Retransmissions first. A fast-retransmit burst may exceed cwnd once.
  // A chunk may go out beyond cwnd only once per loss event: the first fast
  // retransmission of a recovery episode (RFC 9260 §7.2.4) or a tail-loss
  // probe — not once per flush, which would overdrive a congested path.
  bool sent_any = false;
  for (auto it = rtx_.begin(); it != rtx_.end();) {
    const uint32_t k = *it - (inflight_.empty() ? 0 : inflight_.front()->tsn);
    Chunk* ch = k < inflight_.size() ? inflight_[k] : nullptr;
    if (!ch || !ch->retransmit || ch->acked) {
      it = rtx_.erase(it);
      continue;
    }
    bool allowed = flight_size_ + ch->len <= cwnd_ || flight_size_ == 0 || (ch->fast && cwnd_bypass_ > 0);
    if (!allowed) break;
    if (ch->fast && flight_size_ + ch->len > cwnd_ && flight_size_ && cwnd_bypass_ > 0) cwnd_bypass_--;
    it = rtx_.erase(it);
    ch->retransmit = false;
    ch->fast = false;
    ch->miss = 0;
    add_data(ch, false);
    stats_.retransmits++;
    // Counted once per TSN; a chunk that also went out as a redundant copy
    // counts but can never be undone (its duplicate may be the copy's).
    if (ep_active_ && (ch->copied || ep_rtx_tsns_.insert(ch->tsn).second)) ep_rtx_++;
    sent_any = true;
  }
  // New data. After each drain the producer (data channel -> frame scheduler)
  // is told the queue emptied and may enqueue more right away; keep sending
  // within this flush while the windows allow, instead of idling until the
  // next SACK wakes the reactor (the producer keeps this queue shallow for
  // fairness, so without this loop a flush would send at most one window).
  // Priority messages (one chunk each) go first whenever the bulk queue is
  // between messages, and may exceed cwnd by a few packets: an SSE token
  // queued behind a bulk transfer would otherwise wait for that transfer's
  // SACKs, up to a round trip on a WAN path. The allowance bounds what this
  // adds to a congested path (interactive traffic is a trickle).
  const size_t pri_allow = 4 * mtu;
  const bool dup = dup_small_enabled();
  // New data per flush is bounded (kFlushQuantumPkts packets' worth):
  // fragmenting a megabyte of bulk into 1200-byte chunks
  // keeps this thread busy for a few hundred microseconds, and a request or
  // SACK that arrived meanwhile waited for all of it. Past the quantum the
  // reactor takes one non-blocking turn (its I/O first) and the next flush
  // continues. Counted in packets, since the work is per chunk: 128 packets
  // are 150 KB at a 1200-byte MTU (MI355X host mixed row: SSE TTFT p50 0.99 ->
  // 0.59 ms at 128 KB) and 2 MB on a same-host jumbo path, where a 128 KB
  // quantum (8 packets) cost bulk throughput for little latency.
  constexpr size_t kFlushQuantumPkts = 128;
  const size_t quantum = kFlushQuantumPkts * max_payload;
  size_t new_bytes = 0;
  bool yielded = false;
  for (int round = 0; round < 256 && !yielded; round++) {
  bool progressed = false;
  while (!sendq_pri_.empty() || !sendq_.empty()) {
    if (quantum && new_bytes >= quantum) {
      yielded = true;
      r_.post([] {});  // keeps the next epoll_wait from blocking; the flush hook resumes
      break;
    }
    bool pri = !sendq_pri_.empty() && (sendq_.empty() || sendq_.front().off == 0);
    Msg& m = pri ? sendq_pri_.front() : sendq_.front();
    size_t left = m.len - m.off;
    size_t take = std::min(left, max_payload);
    size_t window = pri ? cwnd_ + pri_allow : cwnd_;
    if (flight_size_ > 0 && (flight_size_ + take > window || take > peer_rwnd_)) break;
    if (flight_size_ == 0 && peer_rwnd_ == 0 && !inflight_.empty()) break;  // wait for window / T3 probe
    progressed = true;
    Chunk* ch = new_chunk();
    ch->tsn = next_tsn_++;
    ch->stream = m.stream;
    ch->ssn = m.ssn;
    ch->ppid = m.ppid;
    ch->flags = uint8_t((m.off == 0 ? 2 : 0) | (take == left ? 1 : 0) | (m.unordered ? 4 : 0));
    ch->len = take;
    // Slice [off, off+take) out of header + body without copying the body.
    size_t want_lo = m.off, want_hi = m.off + take;
    if (want_lo < m.hlen) {
      size_t e = std::min<size_t>(m.hlen, want_hi);
      memcpy(ch->inl, m.hdr + want_lo, e - want_lo);
      ch->ilen = uint8_t(e - want_lo);
    }
    if (want_hi > m.hlen) {
      size_t a = want_lo > m.hlen ? want_lo - m.hlen : 0, b = want_hi - m.hlen;
      if (!m.ref) m.ref = new_ref(std::move(m.body));  // the Msg's own use, until fully fragmented
      m.ref->refs++;
      ch->ref = m.ref;
      ch->poff = uint32_t(a);
      ch->plen = uint32_t(b - a);
    }
    m.off += take;
    unsent_bytes_ -= take;
    new_bytes += take;
    inflight_.push_back(ch);
    add_data(ch, false);
    if (dup && ch->flags == (ch->flags | 3) && ch->len <= kDupMaxChunk) dup_.push_back(ch);
    peer_rwnd_ = peer_rwnd_ > take ? peer_rwnd_ - take : 0;
    sent_any = true;
    if (m.off == m.len) {
      if (m.ref) unref(m.ref);
      if (pri) sendq_pri_.pop_front();
      else sendq_.pop_front();
    }
  }
  if (yielded || !progressed || !sendq_.empty() || !sendq_pri_.empty() || !on_sent) break;
  size_t before = unsent_bytes_;
  on_sent();  // producer may refill the (now empty) queue
  if (closed_fired_ || unsent_bytes_ == before) break;
  }
  flush_pkt();
  // Redundant copies of this flush's small whole messages (SSE tokens,
  // credit, pings), in packets of their own after the originals: on a path
  // that loses packets at random a token then arrives unless both copies are
  // lost, instead of waiting a loss-recovery round trip (the receiver drops
  // the second copy and reports it as a duplicate).
  if (!dup_.empty()) {
    for (Chunk* ch : dup_) add_data(ch, true);
    dup_.clear();
    flush_pkt();
  }
  if (sent_any && !t3_timer_) start_t3();
  if (sent_any && !tlp_timer_) arm_tlp();
  if (sent_any && on_sent) on_sent();
}

std::string SctpAssociation::debug_state() const {
  size_t rtx = 0, acked = 0, infl = 0;
  for (const Chunk* ch : inflight_) {
    rtx += ch->retransmit && !ch->acked;
    acked += ch->acked;
    infl += ch->in_flight;
  }
  char b[512];
  snprintf(b, sizeof b,
           "sctp{state=%d unsent=%zu sendq=%zu/%zu inflight=%zu(in_flight %zu, rtx %zu, gap-acked %zu) flight=%zu "
           "cwnd=%zu ssthresh=%zu peer_rwnd=%zu t3=%d tlp=%d rto_ms=%llu srtt_us=%llu | rx ooo=%zu/%zuB held=%zuB "
           "partial=%zu sack_needed=%d}",
           int(state_), unsent_bytes_, sendq_.size(), sendq_pri_.size(), inflight_.size(), infl, rtx, acked,
           flight_size_, cwnd_, ssthresh_, peer_rwnd_, t3_timer_ != 0, tlp_timer_ != 0,
           static_cast<unsigned long long>(rto_us_ / 1000), static_cast<unsigned long long>(srtt_us_), ooo_.size(),
           ooo_bytes_, held_bytes_, partial_.size(), int(sack_needed_));
  return b;
}

// Redundant copies of small messages: SctpConfig::dup_small 1 always, 0
// never; by default on once the path has shown random loss (at least 8 loss
// events, more than 1 in 400 data chunks sent). A lossless LAN path never
// pays for it; tokens are ~100-300 bytes, so doubling them costs little.
bool SctpAssociation::dup_small_enabled() const {
  if (cfg_.dup_small >= 0) return cfg_.dup_small != 0;
  const uint64_t losses = stats_.fast_retransmits + stats_.tlp_probes + stats_.t3_expirations;
  return losses >= 8 && losses * 400 > stats_.data_chunks_sent;
}

}  // namespace p2pt::rtc
