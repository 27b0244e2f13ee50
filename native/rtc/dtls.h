// DTLS 1.2 transport on OpenSSL 3 (RFC 8842 usage for WebRTC data channels).
//
// Replaces webrtc-dtls 0.10 in the reference stack. Each peer uses an
// ephemeral ECDSA P-256 self-signed certificate whose SHA-256 fingerprint is
// advertised in SDP (a=fingerprint); the handshake verifies the peer's
// certificate against the fingerprint from the remote SDP. I/O goes through a
// custom datagram BIO (one BIO write == one UDP datagram) wired to the ICE
// agent's batched send path, and OpenSSL's retransmission timer is driven by
// the reactor.
#pragma once

#include <functional>
#include <memory>
#include <string>

#include "core/reactor.h"

typedef struct ssl_st SSL;
typedef struct bio_st BIO;

namespace p2pt::rtc {

class DtlsTransport : public std::enable_shared_from_this<DtlsTransport> {
 public:
  using WriteFn = std::function<void(const uint8_t*, size_t)>;
  static std::shared_ptr<DtlsTransport> create(Reactor& r, bool is_client, std::string remote_fingerprint,
                                               WriteFn write_datagram);
  ~DtlsTransport();

  // "sha-256 AB:CD:..." value for a=fingerprint (process-wide certificate).
  static const std::string& local_fingerprint();

  void start();
  void on_datagram(const uint8_t* p, size_t n);
  // Encrypt and send one application record (one SCTP packet).
  bool send(const uint8_t* p, size_t n);
  void close();
  bool connected() const { return connected_; }
  // Largest application record (plaintext) after the handshake.
  void set_record_limit(size_t n);
  std::string cipher() const;

  std::function<void()> on_connected;
  std::function<void(const uint8_t*, size_t)> on_data;
  std::function<void(const std::string&)> on_closed;

 private:
  DtlsTransport(Reactor& r) : r_(r) {}
  void drive();
  void arm_timer();
  void fail(const std::string& why);
  bool verify_peer();

  Reactor& r_;
  SSL* ssl_ = nullptr;
  BIO* bio_ = nullptr;
  bool client_ = false;
  bool connected_ = false;
  bool closed_ = false;
  std::string remote_fp_;
  WriteFn write_;
  uint64_t timer_ = 0;
  // current inbound datagram (read by the BIO)
  const uint8_t* in_ = nullptr;
  size_t in_len_ = 0;
  size_t mtu_ = 1200;
  friend struct DtlsBio;
};

}  // namespace p2pt::rtc
