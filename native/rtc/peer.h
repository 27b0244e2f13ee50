// PeerConnection: ICE + DTLS + SCTP + DCEP assembled into a data-only
// WebRTC endpoint, and DataChannel (the MessageChannel the tunnel runs on).
//
// Replaces the webrtc-rs RTCPeerConnection/RTCDataChannel usage of the
// reference (tunnel/src/rtc.rs:31-122): one reliable, ordered data channel
// labelled "tunnel" created by the offerer (rtc.rs:133) and received by the
// answerer via on_data_channel (rtc.rs:296-322); trickled ICE candidates as
// JSON strings (rtc.rs:141-159); state changes Connected/Failed
// (rtc.rs:166-174, :349-355).
//
// Bring-up order: ICE pair selected -> DTLS handshake (role from a=setup) ->
// SCTP association (both sides INIT) -> DCEP OPEN/ACK (RFC 8832) -> open.
// Datagrams produced in a reactor batch are flushed together: SCTP bundles,
// DTLS encrypts one record per packet (into ICE's datagram buffers), ICE
// sends them with one sendmmsg.
#pragma once

#include <algorithm>

#include <functional>
#include <map>
#include <memory>
#include <string>

#include "rtc/dtls.h"
#include "rtc/ice.h"
#include "rtc/sctp.h"
#include "rtc/sdp.h"
#include "tunnel/channel.h"

namespace p2pt::rtc {

enum class PcState { New, Connecting, Connected, Disconnected, Failed, Closed };
const char* pc_state_name(PcState s);

struct PcConfig {
  IceConfig ice;
  size_t sctp_mtu = 1200;
  bool allow_jumbo = true;   // advertise/use large SCTP packets on same-host paths
  size_t jumbo_mtu = 16384;       // = max DTLS plaintext record (2^14)
  size_t jumbo_datagram = 65000;  // records packed per same-host datagram (UDP max 65507)
  size_t jumbo_initial_cwnd = 1 << 20;
  // Delayed-SACK window for lone packets. Worth it on the side that usually
  // answers what it receives (serve: a request's SACK rides on its response);
  // 0 on the side that mostly receives streams (proxy).
  uint64_t sack_delay_us = 0;
  // Fragmented messages handed to chain consumers as views of their packets
  // instead of one reassembled copy (the default copies; see start_sctp).
  bool message_chains = false;
  // Flush coalescing on a busy loop: while the association loop is at least
  // `coalesce_load` busy (Reactor::load) and less than one packet of data is
  // queued, the SCTP flush waits up to `coalesce_us` after the previous one,
  // so token-sized frames of many streams share packets (and sendmmsg calls,
  // reader wake-ups and SACKs on the far side). 0 = off; < 0: the
  // environment (TUNNEL_COALESCE_US) or 50 us at
  // 50 %: on the MI355X host's node row (1 serve, 8 upstreams, 1 ms tokens)
  // it cut the serve's packets at 1024 streams from 680-930 k to 255-270 k
  // per 10 s and the added p50 TTFT from 2.25 to 1.04 ms (median of 3,
  // profiles/r04/node14); below the load threshold nothing changes.
  int64_t coalesce_us = -1;
  double coalesce_load = -1;  // < 0: 0.5
  // Adaptive socket reader (rtc/datapath.h RxReader): engaged once the
  // association thread has read `rx_engage_bytes` within `rx_engage_window_us`
  // (128 MB/s: bulk), handed back once it reads less than `rx_idle_bytes` in
  // `rx_idle_us` (12.8 MB/s). Measured defaults (docs/ROUND5.md, item 1);
  // tests lower them so sanitizer builds, several times slower, still cycle
  // through engage and handback (native test rx_reader_engage_handback_cycles).
  uint64_t rx_engage_window_us = 2000;
  size_t rx_engage_bytes = 256 * 1024;
  uint64_t rx_idle_us = RxReader::kIdleUs;
  size_t rx_idle_bytes = RxReader::kIdleBytes;
  // Register this connection's transport gauges (tunnel_sctp_*, tunnel_udp_*)
  // with the metrics endpoint. Off for the "assoc" extension's extra
  // connections: the gauges are read from the metrics thread and name one
  // association (the first), not the last one to start.
  bool gauges = true;
};

class PeerConnection;

class DataChannel : public MessageChannel, public std::enable_shared_from_this<DataChannel> {
 public:
  DataChannel(std::weak_ptr<PeerConnection> pc, std::string label) : pc_(std::move(pc)), label_(std::move(label)) {}
  bool send(const uint8_t* hdr, size_t hlen, const Bytes& payload) override;
  bool send_urgent(const uint8_t* hdr, size_t hlen, const Bytes& payload) override;
  void note_interactive() override;
  size_t buffered_amount() const override;
  bool is_open() const override { return open_ && !closed_; }
  void close() override;
  std::string describe() const override;
  size_t body_chunk() const override;
  size_t send_window_hint() const override;
  uint64_t rtt_hint_us() const override;
  uint64_t path_rtt_us() const override;
  std::string debug_state() const override;
  void set_lanes(int lanes) override { lanes_ = std::clamp(lanes, 0, kMaxLanes); }
  std::string channel_binding() const override;
  static constexpr int kMaxLanes = 64;
  static constexpr size_t kSmallCwnd = 256 * 1024;  // below: body frames follow cwnd (body_chunk) ...
  static constexpr uint64_t kLongPathUs = 5000;      // ... on paths with a base RTT of at least this
  // The channel's lane streams: stream + 2, + 4, ... (same parity as the
  // channel's own stream, as RFC 8832 allocates per DTLS role).
  bool owns_lane(uint16_t st) const {
    return stream_ >= 0 && st > stream_ && (st - stream_) % 2 == 0 && (st - stream_) / 2 <= kMaxLanes;
  }
  const std::string& label() const { return label_; }
  int stream() const { return stream_; }

 private:
  bool send_impl(const uint8_t* hdr, size_t hlen, const Bytes& payload, bool urgent);
  friend class PeerConnection;
  void set_open();
  void set_closed(const std::string& why);
  // The association, without locking pc_ (a scheduler asks for the buffered
  // amount and window several times per frame: 6 % of the serve's association
  // thread at 1024 streams, profiles/r05/b20/nodeprof). Cached once the
  // connection has one, cleared by PeerConnection::close() — which runs before
  // the association is destroyed — so it never dangles. Association thread.
  SctpAssociation* assoc() const;
  mutable SctpAssociation* assoc_ = nullptr;
  std::weak_ptr<PeerConnection> pc_;
  std::string label_;
  int stream_ = -1;
  int lanes_ = 0;
  bool open_ = false;
  bool closed_ = false;
  bool above_low_ = false;
};

class PeerConnection : public std::enable_shared_from_this<PeerConnection> {
 public:
  static std::shared_ptr<PeerConnection> create(Reactor& r, PcConfig cfg, bool offerer);
  ~PeerConnection();

  std::shared_ptr<DataChannel> create_data_channel(const std::string& label);
  void start_gathering();
  bool gathering_complete() const { return ice_ && ice_->gathering_done(); }
  // Current local SDP (type offer for the offerer, answer for the answerer)
  // with every candidate gathered so far.
  std::string local_description() const;
  bool set_remote_description(const std::string& sdp, std::string* err);
  // Candidate from signalling: a JSON RTCIceCandidateInit string (webrtc-rs
  // form) or a bare "candidate:..." line.
  bool add_ice_candidate(const std::string& cand, std::string* err);
  static std::string candidate_json(const Candidate& c, const std::string& ufrag);
  void close();
  PcState state() const { return state_; }
  std::string describe_path() const;
  const SctpStats* sctp_stats() const { return sctp_ ? &sctp_->stats() : nullptr; }
  size_t sctp_mtu() const { return mtu_; }
  uint64_t coalesced_flushes() const { return coalesced_flushes_; }
  const DtlsTransport* dtls() const { return dtls_.get(); }
  IceAgent* ice() const { return ice_.get(); }
  const SctpAssociation* sctp() const { return sctp_.get(); }

  std::function<void(const std::string& candidate_json)> on_ice_candidate;
  std::function<void()> on_gathering_complete;
  std::function<void(PcState)> on_state;
  std::function<void(std::shared_ptr<DataChannel>)> on_data_channel;

 private:
  friend class DataChannel;
  PeerConnection(Reactor& r, PcConfig cfg, bool offerer);
  void on_ice_state(IceState s);
  void start_dtls();
  void start_sctp();
  void on_sctp_message(uint16_t stream, uint32_t ppid, Bytes msg, std::vector<Bytes>* more);
  void open_pending_channels();
  void set_state(PcState s);
  void fail(const std::string& why);
  void flush();
  void gauge(const char* name, std::function<double()> fn);
  void start_rx_reader();
  void on_rx_burst(RxReader::Burst& b);

  Reactor& r_;
  PcConfig cfg_;
  bool offerer_;
  std::shared_ptr<IceAgent> ice_;
  std::shared_ptr<DtlsTransport> dtls_;
  std::shared_ptr<SctpAssociation> sctp_;
  SessionDesc remote_;
  bool have_remote_ = false;
  bool dtls_client_ = false;
  PcState state_ = PcState::New;
  std::vector<std::shared_ptr<DataChannel>> pending_;
  std::map<uint16_t, std::shared_ptr<DataChannel>> channels_;
  uint16_t next_stream_ = 0;
  uint64_t flush_hook_ = 0;
  size_t mtu_ = 1200;
  uint64_t coalesce_us_ = 0;
  double coalesce_load_ = 0.5;
  uint64_t last_flush_us_ = 0;
  uint64_t coalesce_timer_ = 0;
  uint64_t coalesced_flushes_ = 0;  // flushes held back (metrics, tests)
  bool closed_ = false;
  // The selected direct pair's socket read off this thread (rtc/datapath.h):
  // always (TUNNEL_RX_READER=1), or, adaptive, only while the receive rate
  // is bulk-like: engaged once this thread has read cfg_.rx_engage_bytes
  // within cfg_.rx_engage_window_us, until the reader hands the socket back.
  std::unique_ptr<RxReader> rx_reader_;
  int rx_reader_si_ = -1;
  uint64_t rx_reader_gen_ = 0;   // ICE path generation the reader was started for
  uint64_t rx_reader_ids_ = 0;
  bool rx_engaged_ = false;      // the reader (not this thread) reads the socket
  uint64_t rx_win_start_us_ = 0, rx_win_bytes0_ = 0;
  void restart_rx_reader();
  void maybe_engage_rx_reader();
  size_t rx_slot_bytes() const;
 public:
  uint64_t rx_reader_restarts_ = 0;
  const RxReader* rx_reader() const { return rx_reader_.get(); }
  bool rx_reader_engaged() const { return rx_engaged_; }
};

}  // namespace p2pt::rtc
