#include "rtc/dtls.h"

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>

#include <cstring>
#include <mutex>

#include "core/crypto.h"
#include "core/log.h"

namespace p2pt::rtc {

static const char* kT = "tunnel::dtls";

namespace {

struct Identity {
  EVP_PKEY* key = nullptr;
  X509* cert = nullptr;
  std::string fingerprint;  // "sha-256 AB:CD:..."
  SSL_CTX* ctx = nullptr;
};

std::string fp_of(X509* cert) {
  unsigned char* der = nullptr;
  int len = i2d_X509(cert, &der);
  if (len <= 0) return "";
  auto d = sha256(der, size_t(len));
  OPENSSL_free(der);
  return hex_encode(d.data(), d.size(), true, ':');
}

int verify_any(int, X509_STORE_CTX*) { return 1; }  // self-signed: checked against the SDP fingerprint

Identity& identity() {
  static Identity id;
  static std::once_flag once;
  std::call_once(once, [] {
    id.key = EVP_EC_gen("P-256");
    id.cert = X509_new();
    X509_set_version(id.cert, 2);
    ASN1_INTEGER_set(X509_get_serialNumber(id.cert), long(random_u32() & 0x7fffffff));
    X509_gmtime_adj(X509_getm_notBefore(id.cert), -86400);
    X509_gmtime_adj(X509_getm_notAfter(id.cert), 30L * 86400);
    X509_set_pubkey(id.cert, id.key);
    X509_NAME* name = X509_get_subject_name(id.cert);
    X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("WebRTC"), -1, -1, 0);
    X509_set_issuer_name(id.cert, name);
    X509_sign(id.cert, id.key, EVP_sha256());
    id.fingerprint = "sha-256 " + fp_of(id.cert);

    SSL_CTX* ctx = SSL_CTX_new(DTLS_method());
    SSL_CTX_set_min_proto_version(ctx, DTLS1_2_VERSION);
    SSL_CTX_set_max_proto_version(ctx, DTLS1_2_VERSION);
    SSL_CTX_use_certificate(ctx, id.cert);
    SSL_CTX_use_PrivateKey(ctx, id.key);
    // WebRTC peers (browsers, webrtc-rs) offer ECDHE-ECDSA AEAD suites.
    SSL_CTX_set_cipher_list(ctx,
                            "ECDHE-ECDSA-AES128-GCM-SHA256:ECDHE-ECDSA-AES256-GCM-SHA384:"
                            "ECDHE-ECDSA-CHACHA20-POLY1305:ECDHE-ECDSA-AES256-SHA:ECDHE-ECDSA-AES128-SHA");
    SSL_CTX_set1_groups_list(ctx, "X25519:P-256:P-384");
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, verify_any);
    SSL_CTX_set_read_ahead(ctx, 1);
    SSL_CTX_set_options(ctx, SSL_OP_NO_QUERY_MTU | SSL_OP_NO_TICKET);
    id.ctx = ctx;
  });
  return id;
}

}  // namespace

// Datagram BIO bridging OpenSSL to the ICE agent: every write is one UDP
// datagram; reads return the datagram currently being processed.
struct DtlsBio {
  static BIO_METHOD* method() {
    static BIO_METHOD* m = [] {
      BIO_METHOD* bm = BIO_meth_new(BIO_get_new_index() | BIO_TYPE_SOURCE_SINK, "p2pt-dgram");
      BIO_meth_set_write(bm, write);
      BIO_meth_set_read(bm, read);
      BIO_meth_set_ctrl(bm, ctrl);
      BIO_meth_set_create(bm, [](BIO* b) {
        BIO_set_init(b, 1);
        return 1;
      });
      return bm;
    }();
    return m;
  }
  static int write(BIO* b, const char* data, int len) {
    auto* t = static_cast<DtlsTransport*>(BIO_get_data(b));
    if (!t || t->closed_ || !t->write_) return len;
    t->write_(reinterpret_cast<const uint8_t*>(data), size_t(len));
    return len;
  }
  static int read(BIO* b, char* out, int len) {
    auto* t = static_cast<DtlsTransport*>(BIO_get_data(b));
    BIO_clear_retry_flags(b);
    if (!t || !t->in_ || t->in_len_ == 0) {
      BIO_set_retry_read(b);
      return -1;
    }
    int n = int(t->in_len_) < len ? int(t->in_len_) : len;
    memcpy(out, t->in_, size_t(n));
    t->in_ = nullptr;
    t->in_len_ = 0;
    return n;
  }
  static long ctrl(BIO* b, int cmd, long num, void*) {
    auto* t = static_cast<DtlsTransport*>(BIO_get_data(b));
    switch (cmd) {
      case BIO_CTRL_FLUSH: return 1;
      case BIO_CTRL_DGRAM_QUERY_MTU:
      case BIO_CTRL_DGRAM_GET_FALLBACK_MTU: return t ? long(t->mtu_) : 1200;
      case BIO_CTRL_WPENDING: return 0;
      case BIO_CTRL_PENDING: return t ? long(t->in_len_) : 0;
      case BIO_CTRL_DGRAM_GET_MTU_OVERHEAD: return 0;
      case BIO_CTRL_DGRAM_SET_NEXT_TIMEOUT: return 0;
      case BIO_CTRL_DGRAM_MTU_EXCEEDED: return 0;
      default: (void)num; return 0;
    }
  }
};

const std::string& DtlsTransport::local_fingerprint() { return identity().fingerprint; }

std::shared_ptr<DtlsTransport> DtlsTransport::create(Reactor& r, bool is_client, std::string remote_fp,
                                                     WriteFn write) {
  auto t = std::shared_ptr<DtlsTransport>(new DtlsTransport(r));
  t->client_ = is_client;
  // Normalise "sha-256 ab:cd" -> "AB:CD".
  size_t sp = remote_fp.find(' ');
  std::string fp = sp == std::string::npos ? remote_fp : remote_fp.substr(sp + 1);
  for (auto& c : fp) c = char(toupper(c));
  t->remote_fp_ = fp;
  t->write_ = std::move(write);
  t->ssl_ = SSL_new(identity().ctx);
  t->bio_ = BIO_new(DtlsBio::method());
  BIO_set_data(t->bio_, t.get());
  SSL_set_bio(t->ssl_, t->bio_, t->bio_);
  SSL_set_mtu(t->ssl_, long(t->mtu_));
  DTLS_set_link_mtu(t->ssl_, long(t->mtu_));
  if (is_client) SSL_set_connect_state(t->ssl_);
  else SSL_set_accept_state(t->ssl_);
  return t;
}

DtlsTransport::~DtlsTransport() {
  if (timer_) r_.cancel(timer_);
  if (ssl_) {
    BIO_set_data(bio_, nullptr);
    SSL_free(ssl_);  // frees the BIO
  }
}

void DtlsTransport::start() {
  if (client_) drive();
}

void DtlsTransport::fail(const std::string& why) {
  if (closed_) return;
  closed_ = true;
  if (timer_) r_.cancel(timer_);
  timer_ = 0;
  auto cb = std::move(on_closed);
  on_closed = nullptr;
  if (cb) cb(why);
}

static std::string ssl_errors() {
  std::string s;
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof buf);
    if (!s.empty()) s += "; ";
    s += buf;
  }
  return s.empty() ? "unknown error" : s;
}

bool DtlsTransport::verify_peer() {
  X509* peer = SSL_get1_peer_certificate(ssl_);
  if (!peer) return false;
  std::string fp = fp_of(peer);
  X509_free(peer);
  if (fp != remote_fp_) {
    LOG_ERROR(kT, "DTLS fingerprint mismatch: got %s, SDP says %s", fp.c_str(), remote_fp_.c_str());
    return false;
  }
  return true;
}

void DtlsTransport::drive() {
  if (closed_) return;
  auto self = shared_from_this();
  if (!connected_) {
    ERR_clear_error();
    int rc = SSL_do_handshake(ssl_);
    if (rc == 1) {
      if (!verify_peer()) {
        fail("DTLS peer certificate does not match the SDP fingerprint");
        return;
      }
      connected_ = true;
      if (timer_) r_.cancel(timer_);
      timer_ = 0;
      LOG_DEBUG(kT, "DTLS handshake complete (%s, %s)", client_ ? "client" : "server", cipher().c_str());
      if (on_connected) on_connected();
      if (closed_) return;
    } else {
      int e = SSL_get_error(ssl_, rc);
      if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) {
        fail("DTLS handshake failed: " + ssl_errors());
        return;
      }
      arm_timer();
      return;
    }
  }
  // Application data: one record per SSL_read.
  uint8_t buf[17 * 1024];
  while (!closed_) {
    ERR_clear_error();
    int n = SSL_read(ssl_, buf, sizeof buf);
    if (n > 0) {
      if (on_data) on_data(buf, size_t(n));
      continue;
    }
    int e = SSL_get_error(ssl_, n);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
    if (e == SSL_ERROR_ZERO_RETURN) {
      fail("DTLS close_notify received");
      return;
    }
    // Corrupt/unexpected records are dropped by DTLS; only fatal alerts end us.
    std::string err = ssl_errors();
    if (SSL_get_shutdown(ssl_) & SSL_RECEIVED_SHUTDOWN) {
      fail("DTLS connection closed: " + err);
      return;
    }
    LOG_DEBUG(kT, "DTLS read error (ignored): %s", err.c_str());
    break;
  }
}

void DtlsTransport::arm_timer() {
  if (timer_) r_.cancel(timer_);
  timer_ = 0;
  timeval tv{};
  if (DTLSv1_get_timeout(ssl_, &tv) != 1) return;
  uint64_t us = uint64_t(tv.tv_sec) * 1000000u + uint64_t(tv.tv_usec);
  std::weak_ptr<DtlsTransport> w = shared_from_this();
  timer_ = r_.call_later_us(us ? us : 1, [w] {
    auto s = w.lock();
    if (!s || s->closed_) return;
    s->timer_ = 0;
    if (DTLSv1_handle_timeout(s->ssl_) < 0) {
      s->fail("DTLS handshake timed out");
      return;
    }
    s->drive();
  });
}

void DtlsTransport::on_datagram(const uint8_t* p, size_t n) {
  if (closed_) return;
  in_ = p;
  in_len_ = n;
  drive();
  in_ = nullptr;
  in_len_ = 0;
}

bool DtlsTransport::send(const uint8_t* p, size_t n) {
  if (!connected_ || closed_) return false;
  ERR_clear_error();
  int rc = SSL_write(ssl_, p, int(n));
  if (rc <= 0) {
    LOG_DEBUG(kT, "DTLS write failed: %s", ssl_errors().c_str());
    return false;
  }
  return true;
}

void DtlsTransport::set_record_limit(size_t n) {
  mtu_ = n + 64;
  if (ssl_) {
    SSL_set_mtu(ssl_, long(mtu_));
    DTLS_set_link_mtu(ssl_, long(mtu_));
  }
}

std::string DtlsTransport::cipher() const {
  const char* c = ssl_ ? SSL_get_cipher_name(ssl_) : nullptr;
  return c ? c : "";
}

void DtlsTransport::close() {
  if (closed_) return;
  if (ssl_ && connected_) SSL_shutdown(ssl_);
  closed_ = true;
  if (timer_) r_.cancel(timer_);
  timer_ = 0;
}

}  // namespace p2pt::rtc
