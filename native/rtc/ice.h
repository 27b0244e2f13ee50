// ICE agent (RFC 8445) over UDP: candidate gathering (host, server-reflexive
// via STUN, relayed via TURN), connectivity checks with STUN short-term
// credentials, nomination, consent/liveness, and the datagram path used by
// DTLS once a pair is selected.
//
// Replaces webrtc-ice 0.11 as configured by the reference (tunnel/src/rtc.rs:31-72):
// STUN server stun:stun.l.google.com:19302 plus an optional TURN server,
// mDNS disabled (host IPs are advertised directly, rtc.rs:38-41).
//
// MI355X-host specifics: datagrams leave in one sendmmsg per reactor batch and
// arrive through recvmmsg; 4 MiB socket buffers; loopback host candidates are
// optional (offline / same-host peers).
#pragma once

#include <sys/socket.h>

#include <deque>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "core/net.h"
#include "core/reactor.h"
#include "rtc/stun.h"

namespace p2pt::rtc {

// TUNNEL_FAULT assoc_down_ms (0: off): extra associations fail this long after
// they come up (tunnel/assoc.cc; fail-over tests).
uint64_t fault_assoc_down_ms();

// Byte vector whose resize() leaves new bytes uninitialised (datagram
// buffers are always fully written before use).
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
using DgVec = std::vector<uint8_t, NoInitAlloc<uint8_t>>;

struct Candidate {
  std::string foundation;
  int component = 1;
  std::string transport = "udp";
  uint32_t priority = 0;
  SockAddr addr;
  std::string type = "host";  // host | srflx | prflx | relay
  SockAddr related;
  bool has_related = false;

  // "candidate:<foundation> 1 udp <prio> <ip> <port> typ <type> [raddr <ip> rport <port>]"
  std::string to_sdp() const;
  // Accepts with or without the "candidate:" / "a=candidate:" prefix. Only UDP.
  static bool parse(const std::string& s, Candidate& out, std::string* err = nullptr);
};

uint32_t candidate_priority(const std::string& type, uint32_t local_pref, int component = 1);

class TurnClient;

struct IceConfig {
  std::vector<std::string> stun_urls;  // "stun:host:port"
  std::string turn_url;                // "turn:host:port[?transport=udp]"
  std::string turn_user, turn_pass;
  bool include_loopback = true;
  bool include_ipv6 = false;
  bool ipv6_only = false;  // host candidates on IPv6 interfaces only (implies include_ipv6)
  // iceTransportPolicy "relay": only TURN-relayed local candidates are
  // advertised and checked (forces the TURN path, e.g. symmetric NATs).
  bool relay_only = false;
  uint64_t stun_timeout_ms = 2000;
  uint64_t disconnected_ms = 5000;
  uint64_t failed_ms = 30000;
  uint64_t keepalive_ms = 2500;
  // Register a reactor flush hook that sends queued datagrams. Owners that
  // must order their own flush before ICE's (PeerConnection) turn this off
  // and call IceAgent::flush() themselves.
  bool auto_flush = true;
};

enum class IceState { New, Checking, Connected, Disconnected, Failed, Closed };
const char* ice_state_name(IceState s);

// TUNNEL_UDP_OFFLOAD: the UDP offloads to use, a comma list of "gso" (send
// segmentation) and "gro" (receive coalescing); unset = both, "none" = neither
// (tests of the plain paths).
bool udp_offload_enabled(const char* which);

class IceAgent : public std::enable_shared_from_this<IceAgent> {
 public:
  static std::shared_ptr<IceAgent> create(Reactor& r, IceConfig cfg, bool controlling);
  ~IceAgent();

  const std::string& local_ufrag() const { return ufrag_; }
  const std::string& local_pwd() const { return pwd_; }
  bool controlling() const { return controlling_; }

  void gather();
  bool gathering_done() const { return gathering_done_; }
  const std::vector<Candidate>& local_candidates() const { return local_cands_; }
  void set_remote_credentials(const std::string& ufrag, const std::string& pwd);
  void add_remote_candidate(const Candidate& c);
  void close();

  // Datagram path (valid once a pair is usable). Queued and flushed with one
  // sendmmsg per reactor iteration.
  void send(const uint8_t* p, size_t n);
  // Zero-copy record assembly on the selected path: space for `max` bytes at
  // the end of the datagram being built (a new one when it would exceed the
  // coalescing limit), then commit how many were written.
  uint8_t* reserve_append(size_t max);
  void commit_append(size_t used);
  // Pack several DTLS records into one datagram up to this size (0 = one per
  // datagram). Only for same-host jumbo paths, where IP never fragments.
  void set_coalesce_limit(size_t n) { coalesce_limit_ = n; }
  bool has_path() const { return sel_local_ >= 0; }
  // The selected pair as a plain UDP path another thread may send on (the
  // DTLS TX lane): false with no pair, a TURN relay, or NAT / WAN / fault
  // emulation, all of which live in this agent's own send path.
  bool direct_target(int* fd, SockAddr* to, size_t* coalesce) const;
  // Bumped whenever the selected pair (local socket or remote address)
  // changes: readers and lanes bound to the old path restart on it.
  uint64_t path_generation() const { return path_gen_; }
  bool gro_enabled() const { return gro_enabled_; }
  size_t coalesce_limit() const { return coalesce_limit_; }
  void test_bump_path_generation() { path_gen_++; }  // tests: as if the pair had switched
  // An outside reader (the DTLS RX reader, rtc/datapath.h) takes over the
  // selected direct pair's socket: its reactor reads stop until reattach().
  // False when direct_target() does not hold.
  bool detach_reader(int* fd, int* si, SockAddr* remote);
  void reattach_reader(int si);
  // Tests: the reactor's readable callback for socket `si`, as an event queued
  // earlier in the same turn would run it (a detached socket is not read).
  void readable_for_test(int si) { on_readable(si); }
  // The socket detach_reader() would hand over, without handing it over (a
  // reader that starts paused and engages only under bulk).
  bool reader_target(int* fd, int* si, SockAddr* remote) const;
  // Bytes this agent's own reads took off its sockets (cumulative): the
  // association thread's receive rate, which decides when a reader engages.
  uint64_t rx_bytes() const { return rx_bytes_; }
  // Round-trip time of the connectivity checks (the smallest answered one;
  // 0 = none yet): the path's RTT without any transport's ack delays.
  uint64_t check_rtt_us() const { return check_rtt_us_; }
  // From that reader, on this agent's thread: a datagram it did not handle
  // (STUN, non-application records, other senders), and proof of life for
  // the ones it did (consent freshness).
  void inject(int si, const SockAddr& from, const RawBufPtr& owner, size_t off, size_t len);
  void note_rx();
  // True when both ends of the selected pair are on this host.
  bool selected_same_host() const;
  std::string selected_desc() const;
  size_t local_candidate_count() const { return locals_.size(); }
  IceState state() const { return state_; }
  // Datagrams the kernel dropped on this agent's sockets because their
  // receive buffer was full (sk_drops, the count SO_RXQ_OVFL reports; read
  // with SO_MEMINFO), and the selected socket's effective receive buffer.
  uint64_t rx_overflow() const;
  size_t rcvbuf_bytes() const;
  // Send every queued datagram (sendmmsg, grouped by socket).
  void flush();

  std::function<void(const Candidate&)> on_candidate;
  std::function<void()> on_gathering_done;
  std::function<void(IceState)> on_state;
  // Non-STUN datagrams (DTLS), in a pooled buffer the receiver may modify in
  // place and keep views into (via `owner`).
  std::function<void(std::shared_ptr<const void> owner, uint8_t*, size_t)> on_data;
  // After a readable socket's datagrams were all handed to on_data.
  std::function<void()> on_rx_burst_end;

 private:
  struct Sock {
    int fd = -1;
    SockAddr addr;  // bound address (with port)
    bool loopback = false;
  };
  struct Local {
    Candidate c;
    int sock;       // index into socks_ (base socket)
    bool relay = false;
  };
  struct Pair {
    int local, remote;
    uint64_t prio = 0;
    enum class St { Waiting, InProgress, Succeeded, Failed } st = St::Waiting;
    std::string tid;
    int tries = 0;
    uint64_t next_tx = 0;
    uint64_t rto = 0;
    bool use_cand = false;
    uint64_t sent_us = 0;  // when the check with `tid` went out
  };

  IceAgent(Reactor& r, IceConfig cfg, bool controlling);
  void open_sockets();
  void on_readable(int si);
  void dispatch_rx(int si, const SockAddr& from, const RawBufPtr& owner, size_t len, size_t off = 0);
  void dispatch_segments(int si, const SockAddr& from, const RawBufPtr& owner, size_t len, size_t seg);
  void enable_gro(int fd);
  static size_t gro_segment(const struct msghdr* mh);
  // Test-only NAT emulation (TUNNEL_NAT=port-restricted|symmetric; SURVEY
  // §4.2, BASELINE config #4 without two real NATs). Every datagram leaves
  // through an emulated external socket: one per host socket (endpoint-
  // independent mapping) or one per destination (symmetric). Inbound traffic
  // is accepted only on external sockets and only from destinations that
  // socket has sent to (address+port-dependent filtering); the private host
  // sockets drop everything. STUN servers therefore see the external address
  // (a real srflx candidate), and peers must hole-punch or relay.
  int nat_fd_for(int si, const SockAddr& to);
  void on_nat_readable(int pi);
  void handle_datagram(int local_idx_hint, int si, const SockAddr& from, const uint8_t* p, size_t n, bool via_relay,
                       const RawBufPtr& owner = nullptr);
  void handle_stun(int si, const SockAddr& from, const uint8_t* p, size_t n, bool via_relay);
  void handle_request(int si, const SockAddr& from, const stun::Message& m, const uint8_t* p, size_t n, bool via_relay);
  void handle_response(const SockAddr& from, const stun::Message& m, const uint8_t* p, size_t n);
  void start_srflx();
  struct SrflxWindow;
  void srflx_window_done(const std::shared_ptr<SrflxWindow>& win);
  void start_relay();
  void maybe_gathering_done();
  void add_local(Candidate c, int sock, bool relay);
  void pair_up(int local, int remote);
  int add_pair(int local, int remote);  // index of the (new or existing) pair
  uint64_t pair_priority(const Local& l, const Candidate& r) const;
  void tick();
  void kick();
  void send_check(Pair& p);
  void send_raw(int local_idx, const SockAddr& to, const uint8_t* p, size_t n);
  void select_pair(int pair_idx);
  void set_state(IceState s);
  int find_remote(const SockAddr& a) const;
  int local_for_socket(int si, bool relay) const;

  Reactor& r_;
  IceConfig cfg_;
  bool controlling_;
  uint64_t tiebreaker_;
  std::string ufrag_, pwd_;
  std::string remote_ufrag_, remote_pwd_;
  std::vector<Sock> socks_;
  std::vector<Local> locals_;
  std::vector<Candidate> local_cands_;
  std::vector<Candidate> remotes_;
  std::vector<Pair> pairs_;
  std::map<std::string, int> tx_pairs_;  // STUN tid -> pair index
  uint64_t check_rtt_us_ = 0;
  struct SrflxWindow {  // one STUN server's gathering window
    bool done = false;
    int outstanding = 0;
  };
  struct SrflxReq {
    int sock;
    SockAddr server;
    std::string tid;
    int tries = 0;
    std::shared_ptr<SrflxWindow> win;
  };
  std::vector<SrflxReq> srflx_;
  int pending_gather_ = 0;
  bool gathering_done_ = false;
  bool gather_started_ = false;
  std::shared_ptr<TurnClient> turn_;
  int sel_local_ = -1;
  SockAddr sel_remote_;
  int sel_pair_ = -1;
  IceState state_ = IceState::New;
  uint64_t tick_timer_ = 0;
  uint64_t checking_since_ = 0;
  uint64_t last_rx_ = 0;
  uint64_t last_keepalive_ = 0;
  uint64_t flush_hook_ = 0;
  bool closed_ = false;
  int detached_ = -1;  // socket index read by an outside reader
  uint64_t path_gen_ = 0;
  // Outgoing datagrams for the current batch.
  struct Out {
    int local;
    SockAddr to;
    DgVec data;
    bool faulted = false;  // already passed the fault injector
    bool coalesce = false; // more records may be appended
  };
  std::vector<Out> outq_;
  // WAN emulation (TUNNEL_FAULT rtt_ms / rate_mbps): datagrams waiting for
  // their release time, in order.
  std::deque<std::pair<uint64_t, Out>> delayq_;
  uint64_t link_free_us_ = 0;
  uint64_t delay_timer_ = 0;
  void arm_delay_timer();
 public:
  uint64_t wan_queue_drops_ = 0;
 private:
  struct NatPort {
    int fd = -1;
    int si = -1;                   // host socket it translates for
    SockAddr ext;                  // external (mapped) address
    std::set<std::string> sent;    // destinations sent to (filter)
  };
  int nat_mode_ = 0;               // 0 off, 1 port-restricted cone, 2 symmetric
  std::vector<NatPort> nat_ports_;
  std::map<std::string, int> nat_map_;  // "si|dest" (symmetric) or "si" -> nat_ports_ index
  uint64_t nat_dropped_ = 0;
  std::vector<DgVec> spare_;        // recycled datagram buffers
  size_t coalesce_limit_ = 0;
  size_t append_at_ = 0;
  std::vector<RawBufPtr> rxpool_;   // recvmmsg slots, filled from rxbufs_ each round
  BufPool rxbufs_{65536};
  // UDP GSO/GRO (Linux): runs of equal-size datagrams leave as one message and
  // arrive coalesced. Falls back to one datagram per send if the kernel refuses.
  static constexpr int kGsoMaxSegs = 64;
  static constexpr size_t kGsoMaxBytes = 60000;
  bool gso_ok_ = udp_offload_enabled("gso");
  bool gro_enabled_ = false;
 public:
  uint64_t gso_sends_ = 0, gro_batches_ = 0;  // counters (metrics, tests)
  uint64_t rx_bytes_ = 0;
  uint64_t send_drops_ = 0;  // messages flush() dropped (EAGAIN / unreachable)
 private:
  DgVec drop_;                      // reserve_append target with no path
  friend class TurnClient;
};

}  // namespace p2pt::rtc
