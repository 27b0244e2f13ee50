// DTLS 1.2 transport on OpenSSL 3 (RFC 8842 usage for WebRTC data channels).
//
// Replaces webrtc-dtls 0.10 in the reference stack. Each peer uses an
// ephemeral ECDSA P-256 self-signed certificate whose SHA-256 fingerprint is
// advertised in SDP (a=fingerprint); the handshake verifies the peer's
// certificate against the fingerprint from the remote SDP. OpenSSL runs the
// handshake through a custom datagram BIO (one BIO read == one record) wired
// to the ICE agent's batched send path, and its retransmission timer is
// driven by the reactor.
//
// Application data takes a zero-copy record layer of our own once the
// handshake is done and the suite is AES-GCM (what every WebRTC stack
// negotiates first):
//   - keys come from the session's master secret through the TLS 1.2 PRF
//     ("key expansion", RFC 5246 §6.3) and are checked against a probe record
//     OpenSSL itself encrypts before the switch;
//   - send: the SCTP packet arrives as an iovec gather list (headers plus
//     slices of the frames) and is encrypted straight into the outgoing
//     datagram buffer — no plaintext copy, several records per datagram on
//     same-host jumbo paths;
//   - receive: records are authenticated and decrypted in place inside the
//     pooled receive buffer and handed up as Bytes views into it;
//   - RFC 6347 §4.1.2.6 anti-replay window.
// Records from OpenSSL and ours never share a sequence number: our send side
// starts after the highest epoch-1 sequence OpenSSL wrote, and only once the
// peer has proven it finished the handshake (its first application record
// decrypted), after which OpenSSL never writes again.
#pragma once

#include <sys/uio.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/aesgcm.h"
#include "core/buf.h"
#include "core/reactor.h"
#include "rtc/datapath.h"

typedef struct ssl_st SSL;
typedef struct bio_st BIO;
typedef struct evp_cipher_ctx_st EVP_CIPHER_CTX;

namespace p2pt::rtc {

// Process-wide DTLS identity and peer pinning, set before the first session
// (reference README "Future options": certificate pinning via the DTLS
// fingerprints). Without an identity file every process start has a fresh
// ephemeral certificate.
//   set_identity_file: load a PEM key + certificate, creating it (0600, fresh
//     P-256 key, 10-year self-signed certificate) if missing.
//   set_pinned_fingerprints: only peers whose certificate SHA-256 is listed are
//     accepted (checked against the SDP offer/answer and again after the DTLS
//     handshake). Accepts "sha-256 AB:CD:..", "AB:CD:.." or bare hex; false
//     (with *bad set) on a malformed entry.
bool set_identity_file(const std::string& path, std::string* err);
bool set_pinned_fingerprints(const std::vector<std::string>& fps, std::string* bad = nullptr);
bool fingerprint_pinned(const std::string& fp);  // true when nothing is pinned

class DtlsTransport : public std::enable_shared_from_this<DtlsTransport> {
 public:
  using WriteFn = std::function<void(const uint8_t*, size_t)>;
  // Space for one record appended to the datagram being assembled
  // (reserve(max) -> pointer, commit(used)). Optional: without it records are
  // built in a scratch buffer and handed to WriteFn.
  using ReserveFn = std::function<uint8_t*(size_t)>;
  using CommitFn = std::function<void(size_t)>;

  static std::shared_ptr<DtlsTransport> create(Reactor& r, bool is_client, std::string remote_fingerprint,
                                               WriteFn write_datagram);
  ~DtlsTransport();

  // "sha-256 AB:CD:..." value for a=fingerprint (process-wide certificate).
  static const std::string& local_fingerprint();

  void set_record_sink(ReserveFn reserve, CommitFn commit) {
    reserve_ = std::move(reserve);
    commit_ = std::move(commit);
  }
  void start();
  // One received datagram (may hold several records). The buffer is owned by
  // `owner` and is decrypted in place; plaintext is handed up as views into it.
  void on_datagram(std::shared_ptr<const void> owner, uint8_t* p, size_t n);
  void on_datagram(const uint8_t* p, size_t n);  // copies first
  // Encrypt and send one application record (one SCTP packet) given as a
  // gather list. owners[i] (optional, may be null) keeps iov[i] alive: with
  // the crypto lanes on, such pieces are sealed later on the TX lane without
  // a copy; pieces without an owner are copied.
  bool send(const iovec* iov, const Bytes* const* owners, int cnt);
  bool send(const iovec* iov, int cnt) { return send(iov, nullptr, cnt); }
  bool send(const uint8_t* p, size_t n);

  // Crypto/IO lanes (rtc/datapath.h). Possible once the own record layer runs
  // on the vector AES-GCM; `target` says where the TX lane may send directly
  // (false: through the ICE agent, sealed inline).
  bool lanes_possible() const { return keys_ && keys_->w && keys_->r; }
  void enable_lanes(std::function<bool(TxTarget&)> target);
  bool lanes_enabled() const { return tx_lane_ != nullptr; }
  // End of a flush: seal this flush's records inline or hand them to the TX
  // lane. End of a receive burst: open its records inline or on the RX lane.
  void commit_tx();
  void commit_rx();
  // Records opened by the socket reader (RxReader), on this thread, in
  // receive order: replay check, then up the stack as received records are.
  void deliver_opened(RxBatch& b);
  std::shared_ptr<const RecordKeys> record_keys() const { return keys_; }
  const TxLaneState* tx_lane_state() const { return tx_state_.get(); }
  uint64_t lane_tx_batches() const { return lane_tx_batches_; }
  uint64_t lane_rx_batches() const { return lane_rx_batches_; }
  // Receive bursts on the RX lane not yet back on this thread (a socket
  // reader engaging now could overtake them).
  int rx_outstanding() const { return rx_outstanding_ + (rx_pend_.recs.empty() ? 0 : 1); }
  // Records dropped on receive (failed authentication, replayed or older than
  // the 64-record replay window): loss the SCTP layer sees as a hole.
  uint64_t rx_dropped() const { return rx_dropped_; }
  uint64_t inline_tx_batches() const { return inline_tx_batches_; }
  void close();
  bool connected() const { return connected_; }
  bool fast_path() const { return fast_tx_; }  // own record layer carries sends
  // Largest application record (plaintext) after the handshake.
  void set_record_limit(size_t n);
  std::string cipher() const;

  std::function<void()> on_connected;
  std::function<void(Bytes)> on_data;
  // Records of one receive burst together (set: used for bursts; on_data for
  // single datagrams). The views may be moved from.
  std::function<void(Bytes*, size_t)> on_data_batch;
  std::function<void(const std::string&)> on_closed;

 private:
  DtlsTransport(Reactor& r) : r_(r) {}
  void drive();
  void arm_timer();
  void fail(const std::string& why);
  bool verify_peer();
  void setup_fast_path();
  bool fast_decrypt(uint8_t* rec, size_t len, uint8_t type, uint64_t seq48, uint8_t** pt, size_t* pt_len);
  bool fast_encrypt_into(uint8_t* out, uint8_t type, const iovec* iov, int cnt, size_t total);
  bool replay_seen(uint64_t seq) const;
  void replay_mark(uint64_t seq);
  // An authenticated application/alert record: alerts may end the transport
  // (false), data goes up.
  bool deliver_plain(const std::shared_ptr<const void>& owner, uint8_t type, uint8_t* pt, size_t ptl);
  bool deliver_plain_take(std::shared_ptr<const void>& owner, uint8_t type, uint8_t* pt, size_t ptl);
  void flush_batch();
  bool batching_ = false;
  std::vector<Bytes> batch_;
  void seal_inline(const TxBatch& b);
  void rx_done(RxBatch& b);
  void feed_openssl(const uint8_t* p, size_t n);
  void bio_wrote(const uint8_t* p, size_t n);

  Reactor& r_;
  SSL* ssl_ = nullptr;
  BIO* bio_ = nullptr;
  bool client_ = false;
  bool connected_ = false;
  bool closed_ = false;
  std::string remote_fp_;
  WriteFn write_;
  ReserveFn reserve_;
  CommitFn commit_;
  uint64_t timer_ = 0;
  // current inbound record (read by the BIO)
  const uint8_t* in_ = nullptr;
  size_t in_len_ = 0;
  size_t mtu_ = 1200;

  // --- own record layer
  bool fast_rx_ = false;   // decrypt epoch-1 application records ourselves
  bool fast_tx_ = false;   // encrypt ourselves; OpenSSL is muted from here on
  bool capture_ = false;   // BIO writes are captured (probe record), not sent
  std::string captured_;
  EVP_CIPHER_CTX* wctx_ = nullptr;
  EVP_CIPHER_CTX* rctx_ = nullptr;
  // VAES/VPCLMULQDQ AES-GCM (core/aesgcm.h) when the CPU has it (keys_->w,
  // keys_->r, shared with the lanes); EVP otherwise.
  std::shared_ptr<RecordKeys> keys_;
  uint8_t wiv_[4] = {}, riv_[4] = {};
  // --- crypto/IO lanes
  // Declared before the seal lane so it is destroyed after it: the seal
  // lane's last jobs still hand their batches to the send lane.
  std::unique_ptr<Lane> tx_send_lane_;
  std::unique_ptr<Lane> tx_lane_, rx_lane_;  // tx_lane_: the seal stage
  std::shared_ptr<TxLaneState> tx_state_;
  std::shared_ptr<LaneFd> lane_fd_;
  uint64_t rx_dropped_ = 0;
  std::function<bool(TxTarget&)> tx_target_;
  std::shared_ptr<TxBatch> tx_pend_;
  std::shared_ptr<TxBatchPool> tx_pool_;
  RxBatch rx_pend_;
  int rx_outstanding_ = 0;
  uint64_t lane_tx_batches_ = 0, lane_rx_batches_ = 0, inline_tx_batches_ = 0;
  uint64_t wseq_ = 0;              // next epoch-1 sequence number we send
  uint64_t ossl_max_wseq_ = 0;     // highest epoch-1 sequence OpenSSL wrote
  uint64_t rx_max_ = 0;            // anti-replay: highest authenticated seq
  uint64_t rx_bitmap_ = 0;         // bit i = rx_max_ - i seen
  bool rx_any_ = false;
  std::vector<uint8_t> scratch_;
  friend struct DtlsBio;
};

}  // namespace p2pt::rtc
