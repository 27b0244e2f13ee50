#include "rtc/peer.h"

#include "core/json.h"
#include "core/log.h"
#include "tunnel/metrics.h"

namespace p2pt::rtc {

static const char* kT = "tunnel::rtc";

// DCEP (RFC 8832) and WebRTC PPIDs (RFC 8831 §8).
enum : uint32_t { kPpidDcep = 50, kPpidString = 51, kPpidBinary = 53, kPpidStringEmpty = 56, kPpidBinaryEmpty = 57 };
enum : uint8_t { kDcepAck = 0x02, kDcepOpen = 0x03 };

const char* pc_state_name(PcState s) {
  switch (s) {
    case PcState::New: return "New";
    case PcState::Connecting: return "Connecting";
    case PcState::Connected: return "Connected";
    case PcState::Disconnected: return "Disconnected";
    case PcState::Failed: return "Failed";
    case PcState::Closed: return "Closed";
  }
  return "?";
}

// ---------------------------------------------------------------- DataChannel

constexpr size_t kPrioritySmallFrame = 1024;

// The SCTP priority queue only shortens delivery when the frame rides an SCTP
// stream of its own (negotiated `multistream` lanes): on the one ordered
// stream the receiver holds it until every earlier SSN has arrived, so
// sending it ahead of queued bulk would only push traffic beyond cwnd.
bool DataChannel::send_urgent(const uint8_t* hdr, size_t hlen, const Bytes& payload) {
  return send_impl(hdr, hlen, payload, lanes_ && hlen + payload.size() <= kPrioritySmallFrame);
}

bool DataChannel::send(const uint8_t* hdr, size_t hlen, const Bytes& payload) {
  return send_impl(hdr, hlen, payload, false);
}

void DataChannel::note_interactive() {
  auto pc = pc_.lock();
  if (pc && pc->sctp_) pc->sctp_->note_interactive();
}

// `urgent`: the SCTP priority queue (one-chunk messages only), ahead of bulk
// messages not yet started; the receiver keeps each stream's order (SSN).
SctpAssociation* DataChannel::assoc() const {
  if (assoc_) return assoc_;
  auto pc = pc_.lock();
  if (!pc || pc->closed_ || !pc->sctp_) return nullptr;
  assoc_ = pc->sctp_.get();
  return assoc_;
}

bool DataChannel::send_impl(const uint8_t* hdr, size_t hlen, const Bytes& payload, bool urgent) {
  SctpAssociation* a = is_open() ? assoc() : nullptr;
  if (!a) return false;
  uint16_t st = uint16_t(stream_);
  if (lanes_ && hlen >= 5) {
    uint32_t sid = rd32(hdr + 1);
    if (sid) st = uint16_t(stream_ + 2 * (1 + int(sid % uint32_t(lanes_))));
  }
  // Only urgent frames on a lane take the SCTP priority queue. (Every small
  // frame there — SSE tokens, headers, credit — did not shorten the
  // SSE-next-to-bulk tail on the emulated WAN: a token mostly waits behind a
  // bulk message already being fragmented, which it may not interrupt; and
  // 64 x 1 MB bulk ran ~20 % slower. Removed in round 5.)
  bool ok = a->send_framed(st, kPpidBinary, hdr, hlen, payload, false, urgent);
  if (ok && buffered_amount() > buffered_low_threshold) above_low_ = true;
  return ok;
}

size_t DataChannel::buffered_amount() const {
  SctpAssociation* a = assoc();
  return a ? a->buffered_amount() : 0;
}

void DataChannel::close() {
  if (closed_) return;
  auto pc = pc_.lock();
  if (pc && pc->sctp_ && stream_ >= 0) pc->sctp_->request_stream_reset(uint16_t(stream_));
  closed_ = true;
  on_message = nullptr;
  on_message_chain = nullptr;
  on_open = nullptr;
  on_closed = nullptr;
  on_buffered_low = nullptr;
}

size_t DataChannel::send_window_hint() const {
  SctpAssociation* a = assoc();
  return a ? a->cwnd() : 0;
}

std::string DataChannel::debug_state() const {
  auto pc = pc_.lock();
  std::string s = "dc{buffered=" + std::to_string(buffered_amount()) + " low=" + std::to_string(buffered_low_threshold) +
                  " above_low=" + std::to_string(int(above_low_)) + "} ";
  if (pc && pc->sctp_) s += pc->sctp_->debug_state();
  return s;
}

uint64_t DataChannel::rtt_hint_us() const {
  SctpAssociation* a = assoc();
  return a ? a->min_rtt_us() : 0;
}

uint64_t DataChannel::path_rtt_us() const {
  auto pc = pc_.lock();
  const uint64_t ice = pc && pc->ice_ ? pc->ice_->check_rtt_us() : 0;
  return ice ? ice : rtt_hint_us();
}

// On same-host jumbo paths (16 KiB SCTP packets) body frames are sized to one
// DATA chunk: no fragmentation on send, no reassembly copy on receive, and
// finer interleaving of streams. On network paths (~1200 B packets) the
// reference's 65408 B frames are kept while the congestion window is large;
// once it is small (a lossy WAN), a frame is cut to about an eighth of it
// (whole DATA chunks, at least one): an SCTP message's fragments go out
// back to back, so an SSE token queued behind a 64 KB body frame waited for
// the whole frame, several round trips at a 20-40 KB window (the 150 ms
// SSE-next-to-bulk tail at 50 ms RTT / 2 % loss). Sized when a response
// starts, for that response.
size_t DataChannel::body_chunk() const {
  auto pc = pc_.lock();
  size_t mtu = pc ? pc->mtu_ : 0;
  const size_t per_chunk = mtu > 12 + 16 ? mtu - 12 - 16 : 0;  // SCTP common + DATA chunk headers
  if (mtu >= 8192) return per_chunk - proto::kHeaderLen;       // one chunk, less the frame header
  const size_t cw = pc && pc->sctp_ ? pc->sctp_->cwnd() : 0;
  // Only on a long path: on a LAN a 64 KB frame leaves in microseconds, and a
  // response that started in slow start kept small frames for its whole body
  // (MI355X host, 1200-MTU mixed row: bulk 2125 -> 1543 MB/s, token p99 +2 ms).
  const uint64_t base_rtt = pc && pc->sctp_ ? pc->sctp_->min_rtt_us() : 0;
  if (!per_chunk || cw == 0 || cw >= kSmallCwnd || base_rtt < kLongPathUs) return proto::kMaxBodyChunk;
  const size_t chunks = std::max<size_t>(1, cw / 8 / per_chunk);
  return std::min(proto::kMaxBodyChunk, chunks * per_chunk - proto::kHeaderLen);
}

// Both DTLS certificate fingerprints (ours and the one the remote SDP pinned
// and the handshake verified), normalised and sorted: the same string on both
// peers, different on each leg of a man-in-the-middle.
std::string DataChannel::channel_binding() const {
  auto pc = pc_.lock();
  if (!pc) return "";
  auto norm = [](std::string fp) {
    size_t sp = fp.find(' ');
    if (sp != std::string::npos) fp = fp.substr(sp + 1);
    for (auto& c : fp) c = char(toupper(static_cast<unsigned char>(c)));
    return fp;
  };
  std::string a = norm(DtlsTransport::local_fingerprint()), b = norm(pc->remote_.fingerprint);
  return a < b ? a + "|" + b : b + "|" + a;
}

std::string DataChannel::describe() const {
  auto pc = pc_.lock();
  return "webrtc:" + label_ + (pc ? " " + pc->describe_path() : "");
}

void DataChannel::set_open() {
  if (open_ || closed_) return;
  open_ = true;
  LOG_INFO(kT, "data channel '%s' opened", label_.c_str());
  if (on_open) {
    auto cb = on_open;
    cb();
  }
}

void DataChannel::set_closed(const std::string& why) {
  if (closed_) return;
  closed_ = true;
  open_ = false;
  LOG_INFO(kT, "data channel '%s' closed", label_.c_str());
  auto cb = std::move(on_closed);
  on_closed = nullptr;
  if (cb) cb(why);
}

// ---------------------------------------------------------------- PeerConnection

void PeerConnection::gauge(const char* name, std::function<double()> fn) {
  if (cfg_.gauges) metrics::gauge_fn(name, std::move(fn));
}

std::shared_ptr<PeerConnection> PeerConnection::create(Reactor& r, PcConfig cfg, bool offerer) {
  auto pc = std::shared_ptr<PeerConnection>(new PeerConnection(r, std::move(cfg), offerer));
  std::weak_ptr<PeerConnection> w = pc;
  pc->cfg_.ice.auto_flush = false;
  pc->ice_ = IceAgent::create(r, pc->cfg_.ice, offerer);
  pc->ice_->on_candidate = [w](const Candidate& c) {
    auto s = w.lock();
    if (s && s->on_ice_candidate) s->on_ice_candidate(candidate_json(c, s->ice_->local_ufrag()));
  };
  pc->ice_->on_gathering_done = [w] {
    auto s = w.lock();
    if (s && s->on_gathering_complete) s->on_gathering_complete();
  };
  pc->ice_->on_state = [w](IceState st) {
    if (auto s = w.lock()) s->on_ice_state(st);
  };
  pc->ice_->on_data = [w](std::shared_ptr<const void> owner, uint8_t* p, size_t n) {
    auto s = w.lock();
    if (s && s->dtls_) s->dtls_->on_datagram(std::move(owner), p, n);
  };
  pc->ice_->on_rx_burst_end = [w] {
    auto s = w.lock();
    if (s && s->dtls_) s->dtls_->commit_rx();
  };
  // One flush per reactor batch, in dependency order: SCTP packets ->
  // DTLS records -> ICE datagrams (sendmmsg).
  pc->flush_hook_ = r.add_flush_hook([w] {
    if (auto s = w.lock()) s->flush();
  });
  return pc;
}

PeerConnection::PeerConnection(Reactor& r, PcConfig cfg, bool offerer)
    : r_(r), cfg_(std::move(cfg)), offerer_(offerer), mtu_(cfg_.sctp_mtu) {
  const char* e = getenv("TUNNEL_COALESCE_US");
  coalesce_us_ = cfg_.coalesce_us >= 0 ? uint64_t(cfg_.coalesce_us) : (e && *e ? strtoull(e, nullptr, 10) : 50);
  coalesce_load_ = cfg_.coalesce_load >= 0 ? cfg_.coalesce_load : 0.5;
}

PeerConnection::~PeerConnection() { close(); }

void PeerConnection::flush() {
  if (closed_) return;
  // The selected pair changed under the socket reader (a pair switch or the
  // peer rebinding): give the old socket back to the ICE agent and read the
  // new pair's instead of forwarding everything through the slow path.
  if (rx_reader_ && ice_ && ice_->path_generation() != rx_reader_gen_) restart_rx_reader();
  if (dtls_) dtls_->commit_rx();
  if (rx_reader_ && !rx_engaged_) maybe_engage_rx_reader();
  if (sctp_ && coalesce_us_) {
    // A busy loop with a partial packet queued: let the next pass (or the
    // timer, at most coalesce_us after the previous flush) add to it.
    const uint64_t now = Reactor::now_us();
    const size_t q = sctp_->buffered_amount();
    if (q > 0 && q < mtu_ && now - last_flush_us_ < coalesce_us_ && !sctp_->ack_due() && !sctp_->urgent_pending() &&
        !r_.flushing_soon() && r_.load() >= coalesce_load_) {
      coalesced_flushes_++;
      if (!coalesce_timer_) {
        std::weak_ptr<PeerConnection> w = shared_from_this();
        coalesce_timer_ = r_.call_at(last_flush_us_ + coalesce_us_, [w] {
          if (auto s = w.lock()) s->coalesce_timer_ = 0;  // the flush hook runs after timers
        });
      }
      if (ice_) ice_->flush();
      return;
    }
    last_flush_us_ = now;
  }
  if (sctp_) sctp_->flush();
  if (dtls_) dtls_->commit_tx();
  if (ice_) ice_->flush();
}

void PeerConnection::start_rx_reader() {
  if (rx_reader_ || closed_ || !dtls_ || !ice_ || !dtls_->lanes_enabled()) return;
  const int mode = rx_reader_mode();
  if (mode == kRxReaderOff) return;
  const bool adaptive = mode == kRxReaderAdaptive;
  int fd = -1, si = -1;
  SockAddr remote;
  // Adaptive: the reader starts paused and this thread keeps the socket.
  if (!(adaptive ? ice_->reader_target(&fd, &si, &remote) : ice_->detach_reader(&fd, &si, &remote))) return;
  rx_reader_si_ = si;
  rx_reader_gen_ = ice_->path_generation();
  rx_engaged_ = !adaptive;
  rx_win_start_us_ = Reactor::now_us();
  rx_win_bytes0_ = ice_->rx_bytes();
  std::weak_ptr<PeerConnection> w = shared_from_this();
  Reactor* r = &r_;
  rx_reader_ = std::make_unique<RxReader>(fd, remote, dtls_->record_keys(), [w, r, si](std::unique_ptr<RxReader::Burst> b) {
    b->si = si;
    std::shared_ptr<RxReader::Burst> sb(std::move(b));
    r->post_threadsafe([w, sb] {
      if (auto s = w.lock()) s->on_rx_burst(*sb);
    });
  }, ++rx_reader_ids_, rx_slot_bytes(), adaptive, cfg_.rx_idle_us, cfg_.rx_idle_bytes);
  LOG_DEBUG(kT, "UDP socket reader %s for %s", adaptive ? "ready (engaged under bulk)" : "on", remote.str().c_str());
}

// Adaptive reader: hand the socket over once this thread's receive rate is
// bulk-like. Not while receive bursts are out on the RX lane: their records
// come back through this thread's queue and the reader's first burst could
// overtake them.
void PeerConnection::maybe_engage_rx_reader() {
  const uint64_t now = Reactor::now_us(), rx = ice_->rx_bytes();
  if (rx - rx_win_bytes0_ < cfg_.rx_engage_bytes) {
    if (now - rx_win_start_us_ >= cfg_.rx_engage_window_us) {
      rx_win_start_us_ = now;
      rx_win_bytes0_ = rx;
    }
    return;
  }
  if (dtls_->rx_outstanding()) return;
  int fd = -1, si = -1;
  SockAddr remote;
  if (!ice_->detach_reader(&fd, &si, &remote)) return;
  if (si != rx_reader_si_) {  // not the socket the reader holds (the path generation check restarts it)
    ice_->reattach_reader(si);
    return;
  }
  rx_engaged_ = true;
  rx_reader_->engage();
}

// Receive slot of the socket reader: with UDP GRO a read may hold ~50
// coalesced datagrams (64 KiB); without it one datagram, at most the path's
// packet (several records on a coalescing same-host path) plus the DTLS record
// overhead, rounded up.
size_t PeerConnection::rx_slot_bytes() const {
  if (!ice_ || ice_->gro_enabled()) return 65536;
  const size_t pkt = std::max<size_t>(mtu_, ice_->coalesce_limit()) + 256;
  return std::max<size_t>(2048, (pkt + 1023) & ~size_t(1023));
}

void PeerConnection::restart_rx_reader() {
  LOG_DEBUG(kT, "selected pair changed (generation %llu -> %llu): restarting the UDP socket reader",
            static_cast<unsigned long long>(rx_reader_gen_), static_cast<unsigned long long>(ice_->path_generation()));
  rx_reader_.reset();  // joins; bursts it already posted still arrive (their done() is ignored)
  if (rx_engaged_) ice_->reattach_reader(rx_reader_si_);
  rx_engaged_ = false;
  rx_reader_si_ = -1;
  rx_reader_restarts_++;
  start_rx_reader();
}

// A burst from the socket reader: opened records up the stack (replay check
// in DTLS), the rest through the ICE agent as if it had read them.
void PeerConnection::on_rx_burst(RxReader::Burst& b) {
  const bool current = rx_reader_ && rx_reader_->id() == b.reader;
  if (current) rx_reader_->done();
  if (closed_) return;
  if (b.t_read) trace::set_rx(b.t_kernel, b.t_read, Reactor::now_us());
  if (b.handback) {
    // The reader paused behind its last burst: this thread reads again (and
    // at once, whatever arrived since).
    if (current && rx_engaged_) {
      rx_engaged_ = false;
      rx_win_start_us_ = Reactor::now_us();
      rx_win_bytes0_ = ice_ ? ice_->rx_bytes() : 0;
      if (ice_) ice_->reattach_reader(rx_reader_si_);
    }
    return;
  }
  auto self = shared_from_this();
  if (!b.opened.recs.empty()) {
    if (ice_) ice_->note_rx();
    if (dtls_) dtls_->deliver_opened(b.opened);
  }
  for (auto& raw : b.raw) {
    if (closed_ || !ice_) break;
    ice_->inject(b.si, raw.from, raw.buf, raw.off, raw.len);
  }
}

void PeerConnection::close() {
  if (closed_) return;
  if (sctp_ && sctp_->established()) {
    sctp_->abort("closed");
    flush();
  }
  if (dtls_) {
    dtls_->close();
    if (ice_) ice_->flush();
  }
  closed_ = true;
  if (coalesce_timer_) r_.cancel(coalesce_timer_);
  coalesce_timer_ = 0;
  rx_reader_.reset();  // joins the reader; bursts already posted find closed_ set
  if (flush_hook_) r_.remove_flush_hook(flush_hook_);
  flush_hook_ = 0;
  for (auto& kv : channels_) {
    kv.second->assoc_ = nullptr;  // the association goes with this connection
    kv.second->set_closed("peer connection closed");
  }
  for (auto& dc : pending_) dc->set_closed("peer connection closed");
  if (ice_) {
    ice_->on_state = nullptr;
    ice_->on_data = nullptr;
    ice_->close();
  }
  state_ = PcState::Closed;
}

std::shared_ptr<DataChannel> PeerConnection::create_data_channel(const std::string& label) {
  auto dc = std::make_shared<DataChannel>(weak_from_this(), label);
  pending_.push_back(dc);
  if (sctp_ && sctp_->established()) open_pending_channels();
  return dc;
}

void PeerConnection::start_gathering() { ice_->gather(); }

std::string PeerConnection::local_description() const {
  SessionDesc d;
  d.type = offerer_ ? "offer" : "answer";
  d.ice_ufrag = ice_->local_ufrag();
  d.ice_pwd = ice_->local_pwd();
  d.fingerprint = DtlsTransport::local_fingerprint();
  d.setup = offerer_ ? "actpass" : (dtls_client_ ? "active" : "passive");
  d.mid = have_remote_ ? remote_.mid : "0";
  d.candidates = ice_->local_candidates();
  d.end_of_candidates = ice_->gathering_done();
  if (cfg_.allow_jumbo) d.jumbo = cfg_.jumbo_mtu;
  return d.to_string();
}

bool PeerConnection::set_remote_description(const std::string& sdp, std::string* err) {
  SessionDesc d;
  if (!SessionDesc::parse(sdp, d, err)) return false;
  if (!fingerprint_pinned(d.fingerprint)) {  // fail before ICE/DTLS; re-checked on the certificate
    if (err) *err = "remote fingerprint " + d.fingerprint + " is not pinned (--pin-peer)";
    return false;
  }
  remote_ = d;
  have_remote_ = true;
  // DTLS role (RFC 8842 §5): the answerer picks "active" when offered actpass.
  if (offerer_) dtls_client_ = d.setup == "passive";
  else dtls_client_ = d.setup != "active";
  ice_->set_remote_credentials(d.ice_ufrag, d.ice_pwd);
  for (auto& c : d.candidates) ice_->add_remote_candidate(c);
  if (state_ == PcState::New) set_state(PcState::Connecting);
  return true;
}

std::string PeerConnection::candidate_json(const Candidate& c, const std::string& ufrag) {
  Json j = Json::object();
  j.set("candidate", Json(c.to_sdp()));
  j.set("sdpMid", Json("0"));
  j.set("sdpMLineIndex", Json(0));
  j.set("usernameFragment", Json(ufrag));
  return j.dump();
}

bool PeerConnection::add_ice_candidate(const std::string& cand, std::string* err) {
  std::string line = cand;
  Json j;
  if (!cand.empty() && cand[0] == '{') {
    if (!Json::parse(cand, j, err)) return false;
    const Json* c = j.get("candidate");
    if (!c || !c->is_string()) {
      if (err) *err = "candidate JSON lacks a \"candidate\" string";
      return false;
    }
    line = c->as_string();
  }
  if (line.empty()) return true;  // end-of-candidates marker
  Candidate c;
  if (!Candidate::parse(line, c, err)) return false;
  ice_->add_remote_candidate(c);
  return true;
}

void PeerConnection::set_state(PcState s) {
  if (s == state_ || closed_) return;
  state_ = s;
  LOG_INFO(kT, "peer connection state: %s", pc_state_name(s));
  if (on_state) {
    auto cb = on_state;
    cb(s);
  }
}

void PeerConnection::fail(const std::string& why) {
  if (state_ == PcState::Failed || closed_) return;
  LOG_WARN(kT, "peer connection failed: %s", why.c_str());
  set_state(PcState::Failed);
  for (auto& kv : channels_) kv.second->set_closed(why);
}

void PeerConnection::on_ice_state(IceState s) {
  switch (s) {
    case IceState::Checking:
      set_state(PcState::Connecting);
      break;
    case IceState::Connected:
      if (!dtls_) start_dtls();
      else if (state_ == PcState::Disconnected) set_state(PcState::Connected);
      break;
    case IceState::Disconnected:
      if (state_ == PcState::Connected) set_state(PcState::Disconnected);
      break;
    case IceState::Failed:
      fail("ICE connection failed");
      break;
    default:
      break;
  }
}

void PeerConnection::start_dtls() {
  if (!have_remote_) return;
  LOG_DEBUG(kT, "ICE connected via %s; starting DTLS as %s", ice_->selected_desc().c_str(),
            dtls_client_ ? "client" : "server");
  std::weak_ptr<PeerConnection> w = shared_from_this();
  dtls_ = DtlsTransport::create(r_, dtls_client_, remote_.fingerprint, [w](const uint8_t* p, size_t n) {
    auto s = w.lock();
    if (s && s->ice_) s->ice_->send(p, n);
  });
  // Records are encrypted straight into the datagram ICE is assembling.
  dtls_->set_record_sink(
      [w](size_t max) -> uint8_t* {
        static thread_local std::vector<uint8_t> sink;
        auto s = w.lock();
        if (s && s->ice_) return s->ice_->reserve_append(max);
        sink.resize(max);
        return sink.data();
      },
      [w](size_t used) {
        auto s = w.lock();
        if (s && s->ice_) s->ice_->commit_append(used);
      });
  dtls_->on_connected = [w] {
    if (auto s = w.lock()) s->start_sctp();
  };
  dtls_->on_data = [w](Bytes pkt) {
    auto s = w.lock();
    if (s && s->sctp_) s->sctp_->on_packet(pkt);
  };
  // A receive burst's packets under one reference to this connection (a
  // lock per packet was 10-14 % of the association thread at 1200 MTU).
  dtls_->on_data_batch = [w](Bytes* pkts, size_t n) {
    auto s = w.lock();
    if (!s) return;
    if (s->sctp_ && !s->closed_) s->sctp_->on_packets(pkts, n);
  };
  dtls_->on_closed = [w](const std::string& why) {
    if (auto s = w.lock()) {
      s->fail(why);
    }
  };
  dtls_->start();
}

void PeerConnection::start_sctp() {
  bool jumbo = cfg_.allow_jumbo && remote_.jumbo && ice_->selected_same_host();
  mtu_ = jumbo ? std::min(cfg_.jumbo_mtu, remote_.jumbo) : cfg_.sctp_mtu;
  if (jumbo) dtls_->set_record_limit(mtu_);
  // Same-host jumbo path: several records per datagram (fewer syscalls and
  // kernel packets for bulk bodies); elsewhere one record per datagram.
  ice_->set_coalesce_limit(jumbo ? cfg_.jumbo_datagram : 0);
  SctpConfig sc;
  sc.mtu = mtu_;
  sc.sack_delay_us = cfg_.sack_delay_us;
  sc.remote_port = remote_.sctp_port;
  sc.zero_checksum = true;  // SCTP runs over DTLS (RFC 8261), EDMID 1
  if (jumbo) sc.initial_cwnd = cfg_.jumbo_initial_cwnd;
  std::weak_ptr<PeerConnection> w = shared_from_this();
  // Record crypto and UDP sends of bulk flushes off this thread (rtc/datapath.h).
  dtls_->enable_lanes([w](TxTarget& t) {
    auto s = w.lock();
    if (!s || !s->ice_ || !s->ice_->direct_target(&t.fd, &t.to, &t.coalesce)) return false;
    t.gen = s->ice_->path_generation();
    return true;
  });
  start_rx_reader();
  // Packets straight to the DTLS transport, held strongly (it never refers
  // back to the association): no lock of this connection per packet.
  sctp_ = SctpAssociation::create(r_, sc, [d = dtls_](const iovec* iov, const Bytes* const* owners, int cnt) {
    d->send(iov, owners, cnt);
  });
  sctp_->on_established = [w] {
    auto s = w.lock();
    if (!s) return;
    LOG_DEBUG(kT, "SCTP established (packet size %zu)", s->mtu_);
    s->open_pending_channels();
  };
  sctp_->on_message = [w](uint16_t st, uint32_t ppid, Bytes m) {
    if (auto s = w.lock()) s->on_sctp_message(st, ppid, std::move(m), nullptr);
  };
  // Fragmented messages as chains of packet views (PcConfig::message_chains).
  // Off by default: on the 64 x 1 MB echo one reassembled copy per message
  // measured 1432 vs 1350 req/s (profiles/r04/chain_ab) — the copy is cheaper
  // than walking ~900 small views through the frame decoder and upstream
  // writes — and it raised the 1200-MTU SSE p99 next to bulk (1.04 -> 1.83 ms,
  // profiles/r04/chain29).
  if (cfg_.message_chains)
    sctp_->on_message_chain = [w](uint16_t st, uint32_t ppid, Bytes m, std::vector<Bytes>& more) {
      if (auto s = w.lock()) s->on_sctp_message(st, ppid, std::move(m), &more);
    };
  sctp_->on_stream_reset = [w](uint16_t st) {
    auto s = w.lock();
    if (!s) return;
    auto it = s->channels_.find(st);
    if (it != s->channels_.end()) it->second->set_closed("data channel closed by peer");
  };
  sctp_->on_closed = [w](const std::string& why) {
    auto s = w.lock();
    if (!s) return;
    for (auto& kv : s->channels_) kv.second->set_closed(why);
    s->fail(why);
  };
  sctp_->on_sent = [w] {
    auto s = w.lock();
    if (!s) return;
    for (auto& kv : s->channels_) {
      auto& dc = kv.second;
      if (dc->above_low_ && dc->buffered_amount() <= dc->buffered_low_threshold) {
        dc->above_low_ = false;
        if (dc->on_buffered_low) dc->on_buffered_low();
      }
    }
  };
  gauge("tunnel_sctp_cwnd_bytes", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->cwnd()) : 0.0;
  });
  gauge("tunnel_sctp_srtt_us", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->srtt_us()) : 0.0;
  });
  gauge("tunnel_sctp_min_rtt_us", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->min_rtt_us()) : 0.0;
  });
  gauge("tunnel_sctp_round_min_rtt_us", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->last_round_min_rtt_us()) : 0.0;
  });
  gauge("tunnel_sctp_queue_cuts", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().queue_cuts) : 0.0;
  });
  gauge("tunnel_sctp_retransmits", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().retransmits) : 0.0;
  });
  gauge("tunnel_sctp_fast_retransmits", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().fast_retransmits) : 0.0;
  });
  gauge("tunnel_sctp_t3_expirations", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().t3_expirations) : 0.0;
  });
  gauge("tunnel_sctp_rto_us", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->rto_us()) : 0.0;
  });
  gauge("tunnel_wan_queue_drops", [w] {
    auto s = w.lock();
    return s && s->ice_ ? double(s->ice_->wan_queue_drops_) : 0.0;
  });
  gauge("tunnel_sctp_packets_sent", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().packets_sent) : 0.0;
  });
  gauge("tunnel_sctp_dup_copies", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().dup_copies_sent) : 0.0;
  });
  gauge("tunnel_sctp_tlp_probes", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().tlp_probes) : 0.0;
  });
  gauge("tunnel_sctp_rack_marks", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().rack_marks) : 0.0;
  });
  gauge("tunnel_sctp_spurious_undos", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().spurious_undos) : 0.0;
  });
  gauge("tunnel_sctp_probe_ambiguous", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().probe_ambiguous) : 0.0;
  });
  gauge("tunnel_sctp_dup_tsns_received", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().dup_tsns) : 0.0;
  });
  gauge("tunnel_sctp_late_tsns_received", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().late_tsns) : 0.0;
  });
  gauge("tunnel_sctp_rwnd_drops", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().rwnd_drops) : 0.0;
  });
  gauge("tunnel_dtls_rx_dropped", [w] {
    auto s = w.lock();
    return s && s->dtls_ ? double(s->dtls_->rx_dropped()) : 0.0;
  });
  gauge("tunnel_sctp_hystart_exits", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().hystart_exits) : 0.0;
  });
  gauge("tunnel_sctp_random_loss_cuts", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().random_loss_cuts) : 0.0;
  });
  gauge("tunnel_sctp_congestion_cuts", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().congestion_cuts) : 0.0;
  });
  gauge("tunnel_sctp_over_bdp_losses", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().over_bdp_losses) : 0.0;
  });
  gauge("tunnel_sctp_random_loss_events", [w] {
    auto s = w.lock();
    return s && s->sctp_ ? double(s->sctp_->stats().random_loss_events) : 0.0;
  });
  gauge("tunnel_dtls_lane_tx_batches", [w] {
    auto s = w.lock();
    return s && s->dtls_ ? double(s->dtls_->lane_tx_batches()) : 0.0;
  });
  gauge("tunnel_dtls_inline_tx_batches", [w] {
    auto s = w.lock();
    return s && s->dtls_ ? double(s->dtls_->inline_tx_batches()) : 0.0;
  });
  gauge("tunnel_dtls_lane_rx_batches", [w] {
    auto s = w.lock();
    return s && s->dtls_ ? double(s->dtls_->lane_rx_batches()) : 0.0;
  });
  gauge("tunnel_dtls_lane_datagrams", [w] {
    auto s = w.lock();
    auto* st = s && s->dtls_ ? s->dtls_->tx_lane_state() : nullptr;
    return st ? double(st->datagrams.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_datagrams", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->datagrams.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_bursts", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->bursts.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_raw", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->raw_datagrams.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_waits", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->waits.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_truncated", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->truncated.load()) : 0.0;
  });
  gauge("tunnel_udp_reader_escapes", [w] {
    auto s = w.lock();
    return s && s->rx_reader_ ? double(s->rx_reader_->escapes.load()) : 0.0;
  });
  gauge("tunnel_dtls_lane_gso_msgs", [w] {
    auto s = w.lock();
    auto* st = s && s->dtls_ ? s->dtls_->tx_lane_state() : nullptr;
    return st ? double(st->gso_msgs.load()) : 0.0;
  });
  gauge("tunnel_dtls_lane_send_drops", [w] {
    auto s = w.lock();
    auto* st = s && s->dtls_ ? s->dtls_->tx_lane_state() : nullptr;
    return st ? double(st->send_drops.load()) : 0.0;
  });
  gauge("tunnel_udp_gso_sends", [w] {
    auto s = w.lock();
    return s && s->ice_ ? double(s->ice_->gso_sends_) : 0.0;
  });
  // Loss the stack cannot see otherwise: datagrams the kernel dropped on a
  // full receive buffer (every ICE socket, the reader's included).
  gauge("tunnel_udp_rx_overflow_total", [w] {
    auto s = w.lock();
    if (!s || !s->ice_) return 0.0;
    const uint64_t meminfo = s->ice_->rx_overflow();
    const uint64_t cmsg = s->rx_reader_ ? s->rx_reader_->rxq_ovfl.load() : 0;
    return double(std::max(meminfo, cmsg));
  });
  gauge("tunnel_sctp_coalesced_flushes", [w] {
    auto s = w.lock();
    return s ? double(s->coalesced_flushes_) : 0.0;
  });
  gauge("tunnel_udp_send_drops", [w] {
    auto s = w.lock();
    return s && s->ice_ ? double(s->ice_->send_drops_) : 0.0;
  });
  gauge("tunnel_udp_rcvbuf_bytes", [w] {
    auto s = w.lock();
    return s && s->ice_ ? double(s->ice_->rcvbuf_bytes()) : 0.0;
  });
  gauge("tunnel_dtls_lane_send_waits", [w] {
    auto s = w.lock();
    auto* st = s && s->dtls_ ? s->dtls_->tx_lane_state() : nullptr;
    return st ? double(st->send_waits.load()) : 0.0;
  });
  gauge("tunnel_udp_gro_batches", [w] {
    auto s = w.lock();
    if (!s || !s->ice_) return 0.0;
    return double(s->ice_->gro_batches_ + (s->rx_reader_ ? s->rx_reader_->gro_batches.load() : 0));
  });
  set_state(PcState::Connected);
  sctp_->connect();
}

void PeerConnection::open_pending_channels() {
  if (!sctp_ || !sctp_->established()) return;
  // Stream ids: DTLS client uses even, server odd (RFC 8832 §6).
  for (auto& dc : pending_) {
    uint16_t sid = uint16_t(next_stream_ * 2 + (dtls_client_ ? 0 : 1));
    next_stream_++;
    dc->stream_ = sid;
    channels_[sid] = dc;
    std::vector<uint8_t> open;
    open.push_back(kDcepOpen);
    open.push_back(0x00);  // DATA_CHANNEL_RELIABLE (ordered)
    open.push_back(0);
    open.push_back(0);  // priority
    open.insert(open.end(), 4, 0);  // reliability parameter
    open.push_back(uint8_t(dc->label_.size() >> 8));
    open.push_back(uint8_t(dc->label_.size()));
    open.push_back(0);
    open.push_back(0);  // protocol length
    open.insert(open.end(), dc->label_.begin(), dc->label_.end());
    sctp_->send(sid, kPpidDcep, {Bytes::take(std::move(open))});
    LOG_DEBUG(kT, "sent DCEP OPEN for '%s' on stream %u", dc->label_.c_str(), sid);
  }
  pending_.clear();
}

void PeerConnection::on_sctp_message(uint16_t st, uint32_t ppid, Bytes msg, std::vector<Bytes>* more) {
  if (more && !more->empty() && ppid == kPpidDcep) {  // DCEP in fragments: one piece
    std::vector<uint8_t> v(msg.data(), msg.data() + msg.size());
    for (auto& b : *more) v.insert(v.end(), b.data(), b.data() + b.size());
    msg = Bytes::take(std::move(v));
    more = nullptr;
  }
  if (ppid == kPpidDcep) {
    if (msg.empty()) return;
    if (msg[0] == kDcepOpen && msg.size() >= 12) {
      uint16_t llen = rd16(msg.data() + 8);
      std::string label = msg.size() >= 12u + llen ? std::string(msg.view().substr(12, llen)) : "";
      LOG_INFO(kT, "received data channel: %s", label.c_str());
      auto dc = std::make_shared<DataChannel>(weak_from_this(), label);
      dc->stream_ = st;
      // A repeated OPEN on a stream in use replaces its channel: the old one
      // (still held by the application) is closed here and forgets the
      // association, or its cached pointer would outlive this connection.
      auto old = channels_.find(st);
      if (old != channels_.end() && old->second != dc) {
        old->second->assoc_ = nullptr;
        old->second->set_closed("data channel replaced by a new OPEN on its stream");
      }
      channels_[st] = dc;
      sctp_->send(st, kPpidDcep, {Bytes::copy("\x02", 1)});
      if (on_data_channel) on_data_channel(dc);
      dc->set_open();
    } else if (msg[0] == kDcepAck) {
      auto it = channels_.find(st);
      if (it != channels_.end()) it->second->set_open();
    }
    return;
  }
  auto it = channels_.find(st);
  if (it == channels_.end()) {
    // A lane of a channel ("multistream" extension)?
    for (auto& kv : channels_)
      if (kv.second->owns_lane(st)) {
        it = channels_.find(kv.first);
        break;
      }
    if (it == channels_.end()) return;
  }
  auto dc = it->second;
  if (!dc->is_open()) {
    // Data may follow an OPEN we have not ACKed to ourselves yet: an opener
    // treats the first data from the peer as an implicit ACK (RFC 8832 §6).
    dc->set_open();
  }
  if (ppid == kPpidBinaryEmpty || ppid == kPpidStringEmpty) {
    msg = Bytes();
    more = nullptr;
  }
  dc->deliver(std::move(msg), more);
}

std::string PeerConnection::describe_path() const {
  return ice_ ? ice_->selected_desc() + " mtu=" + std::to_string(mtu_) : "";
}

}  // namespace p2pt::rtc
