#include "rtc/dtls.h"

#include <cstdlib>

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/kdf.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
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

// Process-wide settings, fixed before the first session (set_identity_file,
// set_pinned_fingerprints; see dtls.h).
std::string g_identity_path;
std::vector<std::string> g_pins;

void make_cert(Identity& id, long days) {
  id.key = EVP_EC_gen("P-256");
  id.cert = X509_new();
  X509_set_version(id.cert, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(id.cert), long(random_u32() & 0x7fffffff));
  X509_gmtime_adj(X509_getm_notBefore(id.cert), -86400);
  X509_gmtime_adj(X509_getm_notAfter(id.cert), days * 86400);
  X509_set_pubkey(id.cert, id.key);
  X509_NAME* name = X509_get_subject_name(id.cert);
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("WebRTC"), -1, -1, 0);
  X509_set_issuer_name(id.cert, name);
  X509_sign(id.cert, id.key, EVP_sha256());
}

// PEM private key + certificate. A missing file is created (mode 0600) with a
// fresh long-lived key pair, so the fingerprint stays stable across restarts
// and the peer can pin it.
bool load_or_create(const std::string& path, Identity& id, std::string* err) {
  if (FILE* f = fopen(path.c_str(), "r")) {
    id.key = PEM_read_PrivateKey(f, nullptr, nullptr, nullptr);
    id.cert = id.key ? PEM_read_X509(f, nullptr, nullptr, nullptr) : nullptr;
    fclose(f);
    if (!id.key || !id.cert || X509_check_private_key(id.cert, id.key) != 1) {
      *err = "not a PEM private key followed by its certificate";
      return false;
    }
    return true;
  }
  if (errno != ENOENT) {
    *err = strerror(errno);
    return false;
  }
  make_cert(id, 3650);
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0600);
  FILE* f = fd >= 0 ? fdopen(fd, "w") : nullptr;
  if (!f) {
    *err = std::string("cannot create: ") + strerror(errno);
    if (fd >= 0) ::close(fd);
    return false;
  }
  bool ok = PEM_write_PrivateKey(f, id.key, nullptr, nullptr, 0, nullptr, nullptr) == 1 &&
            PEM_write_X509(f, id.cert) == 1;
  ok = fclose(f) == 0 && ok;
  if (!ok) *err = "write failed";
  return ok;
}

// "sha-256 ab:cd..." / "AB:CD..." / "abcd..." -> "AB:CD:..." (empty if not a
// SHA-256 fingerprint).
std::string normalize_fp(std::string s) {
  size_t sp = s.find_last_of(' ');
  if (sp != std::string::npos) s = s.substr(sp + 1);
  std::string hex;
  for (char c : s)
    if (c != ':') hex += char(toupper(static_cast<unsigned char>(c)));
  if (hex.size() != 64 || hex.find_first_not_of("0123456789ABCDEF") != std::string::npos) return "";
  std::string out;
  for (size_t i = 0; i < hex.size(); i += 2) {
    if (i) out += ':';
    out += hex.substr(i, 2);
  }
  return out;
}

Identity& identity() {
  static Identity id;
  static std::once_flag once;
  std::call_once(once, [] {
    std::string err;
    if (!g_identity_path.empty() && !load_or_create(g_identity_path, id, &err)) {
      // set_identity_file() validated the file already; reaching this means
      // it changed underneath us. Never fall back to a different identity
      // silently: pinned peers would reject it anyway.
      LOG_ERROR(kT, "DTLS identity %s: %s", g_identity_path.c_str(), err.c_str());
      abort();
    }
    if (g_identity_path.empty()) make_cert(id, 30);
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
    SSL_CTX_set_options(ctx, SSL_OP_NO_QUERY_MTU | SSL_OP_NO_TICKET | SSL_OP_NO_RENEGOTIATION);
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
    if (t) t->bio_wrote(reinterpret_cast<const uint8_t*>(data), size_t(len));
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

bool set_identity_file(const std::string& path, std::string* err) {
  Identity probe;  // validate (or create) now, so a bad file fails at startup
  bool ok = load_or_create(path, probe, err);
  EVP_PKEY_free(probe.key);
  X509_free(probe.cert);
  if (ok) g_identity_path = path;
  return ok;
}

bool set_pinned_fingerprints(const std::vector<std::string>& fps, std::string* bad) {
  std::vector<std::string> pins;
  for (auto& f : fps) {
    std::string n = normalize_fp(f);
    if (n.empty()) {
      if (bad) *bad = f;
      return false;
    }
    pins.push_back(n);
  }
  g_pins = std::move(pins);
  return true;
}

bool fingerprint_pinned(const std::string& fp) {
  if (g_pins.empty()) return true;
  std::string n = normalize_fp(fp);
  return std::find(g_pins.begin(), g_pins.end(), n) != g_pins.end();
}

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
  if (wctx_) EVP_CIPHER_CTX_free(wctx_);
  if (rctx_) EVP_CIPHER_CTX_free(rctx_);
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
  if (!fingerprint_pinned(fp)) {
    LOG_ERROR(kT, "DTLS peer certificate sha-256 %s is not pinned (--pin-peer)", fp.c_str());
    return false;
  }
  return true;
}

namespace {
constexpr uint8_t kAppData = 23, kAlert = 21;

uint64_t rd48(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 6; i++) v = v << 8 | p[i];
  return v;
}
void wr48(uint8_t* p, uint64_t v) {
  for (int i = 5; i >= 0; i--) {
    p[i] = uint8_t(v);
    v >>= 8;
  }
}
}  // namespace

// Every datagram OpenSSL emits passes here: remember the highest epoch-1
// sequence number it used (our record layer continues after it), capture the
// probe record, and mute OpenSSL once our layer owns the epoch.
void DtlsTransport::bio_wrote(const uint8_t* p, size_t n) {
  for (size_t off = 0; off + kRecHdr <= n;) {
    size_t len = rd16(p + off + 11);
    if (rd16(p + off + 3) == 1) ossl_max_wseq_ = std::max(ossl_max_wseq_, rd48(p + off + 5));
    off += kRecHdr + len;
  }
  if (capture_) {
    captured_.append(reinterpret_cast<const char*>(p), n);
    return;
  }
  if (closed_ || fast_tx_ || !write_) return;
  write_(p, n);
}

// TLS 1.2 key block for the AES-GCM suites (RFC 5246 §6.3, RFC 5288 §3):
// client_write_key | server_write_key | client_write_IV[4] | server_write_IV[4].
// TUNNEL_DTLS_RECORDS: the record layer after the handshake. Unset: this
// build's own (vector AES-GCM where the CPU has VAES, OpenSSL's EVP cipher
// otherwise); "evp": own records, EVP cipher; "openssl": OpenSSL's record
// layer throughout (a standard DTLS 1.2 stack on the wire, for interop tests).
static std::string record_layer() {
  static const std::string v = [] {
    const char* e = getenv("TUNNEL_DTLS_RECORDS");
    return std::string(e ? e : "");
  }();
  return v;
}

void DtlsTransport::setup_fast_path() {
  if (record_layer() == "openssl") return;  // diagnostics: keep OpenSSL's record layer
  const SSL_CIPHER* c = SSL_get_current_cipher(ssl_);
  if (!c) return;
  uint16_t id = SSL_CIPHER_get_protocol_id(c);
  const EVP_CIPHER* ciph;
  const char* md;
  size_t klen;
  if (id == 0xC02B) {  // ECDHE-ECDSA-AES128-GCM-SHA256
    ciph = EVP_aes_128_gcm();
    md = "SHA256";
    klen = 16;
  } else if (id == 0xC02C) {  // ECDHE-ECDSA-AES256-GCM-SHA384
    ciph = EVP_aes_256_gcm();
    md = "SHA384";
    klen = 32;
  } else {
    LOG_DEBUG(kT, "DTLS suite %s: OpenSSL record layer", cipher().c_str());
    return;
  }
  uint8_t master[48], cr[32], sr[32];
  size_t mlen = SSL_SESSION_get_master_key(SSL_get_session(ssl_), master, sizeof master);
  if (mlen != 48 || SSL_get_client_random(ssl_, cr, 32) != 32 || SSL_get_server_random(ssl_, sr, 32) != 32) return;
  uint8_t seed[13 + 64];
  memcpy(seed, "key expansion", 13);
  memcpy(seed + 13, sr, 32);
  memcpy(seed + 45, cr, 32);
  uint8_t kb[2 * 32 + 2 * 4];
  size_t kblen = 2 * klen + 8;
  EVP_KDF* kdf = EVP_KDF_fetch(nullptr, "TLS1-PRF", nullptr);
  EVP_KDF_CTX* kctx = kdf ? EVP_KDF_CTX_new(kdf) : nullptr;
  OSSL_PARAM params[] = {
      OSSL_PARAM_construct_utf8_string(OSSL_KDF_PARAM_DIGEST, const_cast<char*>(md), 0),
      OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_SECRET, master, mlen),
      OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_SEED, seed, sizeof seed),
      OSSL_PARAM_construct_end()};
  bool ok = kctx && EVP_KDF_derive(kctx, kb, kblen, params) == 1;
  EVP_KDF_CTX_free(kctx);
  EVP_KDF_free(kdf);
  OPENSSL_cleanse(master, sizeof master);
  if (!ok) return;
  const uint8_t* ckey = kb;
  const uint8_t* skey = kb + klen;
  const uint8_t* civ = kb + 2 * klen;
  const uint8_t* siv = civ + 4;
  const uint8_t* wkey = client_ ? ckey : skey;
  const uint8_t* rkey = client_ ? skey : ckey;
  memcpy(wiv_, client_ ? civ : siv, 4);
  memcpy(riv_, client_ ? siv : civ, 4);
  wctx_ = EVP_CIPHER_CTX_new();
  rctx_ = EVP_CIPHER_CTX_new();
  EVP_EncryptInit_ex(wctx_, ciph, nullptr, wkey, nullptr);
  EVP_DecryptInit_ex(rctx_, ciph, nullptr, rkey, nullptr);
  // Known-answer check of the derivation: OpenSSL encrypts a probe record
  // (captured, never sent); our write key must open it.
  static const char kProbe[] = "p2pt-record-probe";
  capture_ = true;
  captured_.clear();
  ERR_clear_error();
  int rc = SSL_write(ssl_, kProbe, int(sizeof kProbe - 1));
  capture_ = false;
  bool probe_ok = false;
  if (rc > 0 && captured_.size() >= kRecHdr + kExplicit + kTag) {
    auto* rec = reinterpret_cast<uint8_t*>(captured_.data());
    size_t ctlen = captured_.size() - kRecHdr - kExplicit - kTag;
    EVP_CIPHER_CTX* t = EVP_CIPHER_CTX_new();
    uint8_t nonce[12], aad[13], out[64];
    memcpy(nonce, wiv_, 4);
    memcpy(nonce + 4, rec + kRecHdr, 8);
    memcpy(aad, rec + 3, 8);
    aad[8] = rec[0];
    aad[9] = rec[1];
    aad[10] = rec[2];
    wr16(aad + 11, uint16_t(ctlen));
    int l = 0, l2 = 0;
    probe_ok = ctlen == sizeof kProbe - 1 && EVP_DecryptInit_ex(t, ciph, nullptr, wkey, nonce) == 1 &&
               EVP_DecryptUpdate(t, nullptr, &l, aad, 13) == 1 &&
               EVP_DecryptUpdate(t, out, &l, rec + kRecHdr + kExplicit, int(ctlen)) == 1 &&
               EVP_CIPHER_CTX_ctrl(t, EVP_CTRL_GCM_SET_TAG, 16, rec + kRecHdr + kExplicit + ctlen) == 1 &&
               EVP_DecryptFinal_ex(t, out + l, &l2) == 1 && memcmp(out, kProbe, ctlen) == 0;
    EVP_CIPHER_CTX_free(t);
    // The vector AES-GCM must open OpenSSL's probe too, or it stays unused.
    keys_ = std::make_shared<RecordKeys>();
    memcpy(keys_->wiv, wiv_, 4);
    memcpy(keys_->riv, riv_, 4);
    if (probe_ok && AesGcm::supported() && record_layer() != "evp") {
      auto w = std::make_shared<AesGcm>(), r = std::make_shared<AesGcm>();
      uint8_t ct[sizeof kProbe];
      if (w->init(wkey, klen) && r->init(rkey, klen) &&
          w->open(nonce, aad, 13, rec + kRecHdr + kExplicit, ct, ctlen, rec + kRecHdr + kExplicit + ctlen) &&
          memcmp(ct, kProbe, ctlen) == 0) {
        keys_->w = std::move(w);
        keys_->r = std::move(r);
      } else {
        LOG_WARN(kT, "vector AES-GCM self-check failed; using OpenSSL's EVP for records");
      }
    }
  }
  OPENSSL_cleanse(kb, sizeof kb);
  if (!probe_ok) {
    LOG_WARN(kT, "DTLS key derivation self-check failed; staying on OpenSSL's record layer");
    return;
  }
  fast_rx_ = true;
  LOG_DEBUG(kT, "DTLS own record layer armed (%s, %s)", cipher().c_str(), lanes_possible() ? "VAES AES-GCM" : "EVP AES-GCM");
}

bool DtlsTransport::replay_seen(uint64_t seq) const {
  if (!rx_any_ || seq > rx_max_) return false;
  uint64_t d = rx_max_ - seq;
  return d >= 64 || (rx_bitmap_ >> d) & 1;  // replayed or too old
}

void DtlsTransport::replay_mark(uint64_t seq) {
  if (!rx_any_ || seq > rx_max_) {
    uint64_t sh = rx_any_ ? seq - rx_max_ : 64;
    rx_bitmap_ = sh >= 64 ? 1 : (rx_bitmap_ << sh) | 1;
    rx_max_ = seq;
    rx_any_ = true;
  } else {
    rx_bitmap_ |= uint64_t(1) << (rx_max_ - seq);
  }
}

bool DtlsTransport::fast_decrypt(uint8_t* rec, size_t len, uint8_t type, uint64_t seq, uint8_t** pt, size_t* pt_len) {
  if (len < kRecHdr + kExplicit + kTag) return false;
  if (replay_seen(seq)) return false;
  if (keys_ && keys_->r) {
    if (!open_record(*keys_->r, riv_, rec, len, pt, pt_len)) return false;
    replay_mark(seq);
    return true;
  }
  size_t ctlen = len - kRecHdr - kExplicit - kTag;
  uint8_t* ct = rec + kRecHdr + kExplicit;
  uint8_t nonce[12], aad[13];
  memcpy(nonce, riv_, 4);
  memcpy(nonce + 4, rec + kRecHdr, 8);
  memcpy(aad, rec + 3, 8);
  aad[8] = type;
  aad[9] = rec[1];
  aad[10] = rec[2];
  wr16(aad + 11, uint16_t(ctlen));
  int l = 0, l2 = 0;
  if (EVP_DecryptInit_ex(rctx_, nullptr, nullptr, nullptr, nonce) != 1 ||
      EVP_DecryptUpdate(rctx_, nullptr, &l, aad, 13) != 1 || EVP_DecryptUpdate(rctx_, ct, &l, ct, int(ctlen)) != 1 ||
      EVP_CIPHER_CTX_ctrl(rctx_, EVP_CTRL_GCM_SET_TAG, 16, ct + ctlen) != 1 ||
      EVP_DecryptFinal_ex(rctx_, ct + l, &l2) != 1)
    return false;
  replay_mark(seq);
  *pt = ct;
  *pt_len = ctlen;
  return true;
}

bool DtlsTransport::fast_encrypt_into(uint8_t* out, uint8_t type, const iovec* iov, int cnt, size_t total) {
  out[0] = type;
  out[1] = 0xFE;  // DTLS 1.2
  out[2] = 0xFD;
  wr16(out + 3, 1);  // epoch
  wr48(out + 5, wseq_++);
  wr16(out + 11, uint16_t(kExplicit + total + kTag));
  memcpy(out + kRecHdr, out + 3, 8);  // explicit nonce = epoch || seq (as OpenSSL does)
  uint8_t nonce[12], aad[13];
  memcpy(nonce, wiv_, 4);
  memcpy(nonce + 4, out + 3, 8);
  memcpy(aad, out + 3, 8);
  aad[8] = type;
  aad[9] = 0xFE;
  aad[10] = 0xFD;
  wr16(aad + 11, uint16_t(total));
  if (keys_ && keys_->w) {  // straight from the gather list into the datagram
    uint8_t* o = out + kRecHdr + kExplicit;
    keys_->w->seal_gather(nonce, aad, 13, iov, cnt, o, total, o + total);
    return true;
  }
  int l = 0;
  if (EVP_EncryptInit_ex(wctx_, nullptr, nullptr, nullptr, nonce) != 1 ||
      EVP_EncryptUpdate(wctx_, nullptr, &l, aad, 13) != 1)
    return false;
  uint8_t* o = out + kRecHdr + kExplicit;
  for (int i = 0; i < cnt; i++) {
    if (!iov[i].iov_len) continue;
    if (EVP_EncryptUpdate(wctx_, o, &l, static_cast<const uint8_t*>(iov[i].iov_base), int(iov[i].iov_len)) != 1)
      return false;
    o += l;
  }
  if (EVP_EncryptFinal_ex(wctx_, o, &l) != 1) return false;
  o += l;
  return EVP_CIPHER_CTX_ctrl(wctx_, EVP_CTRL_GCM_GET_TAG, 16, o) == 1;
}

void DtlsTransport::drive() {
  if (closed_ || fast_tx_) return;
  auto self = shared_from_this();
  if (!connected_) {
    ERR_clear_error();
    int rc = SSL_do_handshake(ssl_);
    if (rc == 1) {
      if (!verify_peer()) {
        fail("DTLS peer certificate rejected (SDP fingerprint mismatch or not pinned)");
        return;
      }
      connected_ = true;
      if (timer_) r_.cancel(timer_);
      timer_ = 0;
      LOG_DEBUG(kT, "DTLS handshake complete (%s, %s)", client_ ? "client" : "server", cipher().c_str());
      setup_fast_path();
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
  // Application data through OpenSSL (before our layer is armed, or for
  // records OpenSSL buffered during the handshake).
  uint8_t buf[17 * 1024];
  while (!closed_) {
    ERR_clear_error();
    int n = SSL_read(ssl_, buf, sizeof buf);
    if (n > 0) {
      if (on_data) on_data(Bytes::copy(buf, size_t(n)));
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
    if (!s || s->closed_ || s->fast_tx_) return;
    s->timer_ = 0;
    if (DTLSv1_handle_timeout(s->ssl_) < 0) {
      s->fail("DTLS handshake timed out");
      return;
    }
    s->drive();
  });
}

void DtlsTransport::feed_openssl(const uint8_t* p, size_t n) {
  in_ = p;
  in_len_ = n;
  drive();
  in_ = nullptr;
  in_len_ = 0;
}

void DtlsTransport::on_datagram(const uint8_t* p, size_t n) {
  auto buf = std::make_shared<RawBuf>(n ? n : 1);
  memcpy(buf->data.get(), p, n);
  uint8_t* d = buf->data.get();
  on_datagram(std::move(buf), d, n);
}

void DtlsTransport::on_datagram(std::shared_ptr<const void> owner, uint8_t* p, size_t n) {
  if (closed_) return;
  auto self = shared_from_this();
  size_t off = 0;
  while (off + kRecHdr <= n && !closed_) {
    uint8_t* rec = p + off;
    uint8_t type = rec[0];
    uint16_t epoch = rd16(rec + 3);
    size_t len = kRecHdr + rd16(rec + 11);
    if (off + len > n) break;  // truncated record: drop the rest
    off += len;
    if (fast_rx_ && epoch == 1 && (type == kAppData || type == kAlert)) {
      if (rx_lane_ && fast_tx_) {  // opened at the end of the receive burst (commit_rx)
        RxBatch::Rec r;
        r.rec = rec;
        r.len = uint32_t(len);
        r.type = type;
        r.seq = rd48(rec + 5);
        r.owner = owner;
        rx_pend_.recs.push_back(std::move(r));
        rx_pend_.bytes += len;
        continue;
      }
      uint8_t* pt;
      size_t ptl;
      if (!fast_decrypt(rec, len, type, rd48(rec + 5), &pt, &ptl)) {
        LOG_TRACE(kT, "dropping DTLS record that fails authentication or replay check");
        rx_dropped_++;
        continue;
      }
      if (!deliver_plain(owner, type, pt, ptl)) return;
      continue;
    }
    if (fast_tx_) continue;  // stale handshake retransmissions: OpenSSL is retired
    feed_openssl(rec, len);
  }
}

bool DtlsTransport::deliver_plain(const std::shared_ptr<const void>& owner, uint8_t type, uint8_t* pt, size_t ptl) {
  std::shared_ptr<const void> o = owner;
  return deliver_plain_take(o, type, pt, ptl);
}

// `owner` is moved into the record's view (no reference count traffic), and
// with a batch open (deliver_opened) the view is collected for on_data_batch.
bool DtlsTransport::deliver_plain_take(std::shared_ptr<const void>& owner, uint8_t type, uint8_t* pt, size_t ptl) {
  if (type == kAlert) {
    if (ptl >= 2 && (pt[0] == 2 || pt[1] == 0)) {
      flush_batch();  // what came before the alert goes up first
      if (closed_) return false;
      fail(pt[1] == 0 ? "DTLS close_notify received" : "DTLS fatal alert received");
      return false;
    }
    return true;
  }
  if (!fast_tx_) {
    // The peer finished its handshake: OpenSSL has nothing left to send.
    fast_tx_ = true;
    wseq_ = ossl_max_wseq_ + 1;
    if (timer_) r_.cancel(timer_);
    timer_ = 0;
  }
  if (batching_ && on_data_batch) {
    batch_.push_back(Bytes::adopt(std::move(owner), pt, ptl));
    return true;
  }
  if (on_data) on_data(Bytes::adopt(std::move(owner), pt, ptl));
  return !closed_;
}

void DtlsTransport::flush_batch() {
  if (batch_.empty()) return;
  std::vector<Bytes> b;
  b.swap(batch_);
  if (on_data_batch && !closed_) on_data_batch(b.data(), b.size());
  b.clear();
  if (batch_.empty()) batch_.swap(b);  // keep the capacity
}

void DtlsTransport::enable_lanes(std::function<bool(TxTarget&)> target) {
  if (tx_lane_ || !lanes_possible()) return;
  tx_target_ = std::move(target);
  tx_state_ = std::make_shared<TxLaneState>();
  tx_pool_ = std::make_shared<TxBatchPool>();
  tx_pend_ = tx_pool_->get();
  tx_send_lane_ = std::make_unique<Lane>("p2pt-dtls-txsend");
  tx_lane_ = std::make_unique<Lane>("p2pt-dtls-tx");
  rx_lane_ = std::make_unique<Lane>("p2pt-dtls-rx");
  LOG_DEBUG(kT, "DTLS crypto lanes on (inline below %zu bytes)", datapath_inline_bytes());
}

void DtlsTransport::seal_inline(const TxBatch& b) {
  iovec iov[64];
  for (auto& r : b.recs) {
    const int cnt = b.gather(r, iov, 64);
    const size_t rec = record_size(r.total);
    if (reserve_) {
      uint8_t* o = reserve_(rec);
      seal_record(*keys_->w, wiv_, o, r.type, r.seq, iov, cnt, r.total);
      commit_(rec);
    } else {
      if (scratch_.size() < rec) scratch_.resize(rec);
      seal_record(*keys_->w, wiv_, scratch_.data(), r.type, r.seq, iov, cnt, r.total);
      if (write_) write_(scratch_.data(), rec);
    }
  }
}

void DtlsTransport::commit_tx() {
  if (!tx_pend_ || tx_pend_->recs.empty()) return;
  if (closed_) {
    tx_pend_->clear();
    return;
  }
  TxTarget t;
  const bool direct = tx_target_ && tx_target_(t) && t.fd >= 0;
  if (!direct || (tx_pend_->bytes < datapath_inline_bytes() && tx_lane_->idle() && tx_send_lane_->idle())) {
    // A small flush with nothing ahead of it on the lane (or no direct path):
    // sealed here, sent by the ICE agent's flush — no thread hop on the
    // latency path of a token. (Handing small flushes to the lanes off a
    // >= 50 %-busy loop cost the 64 x 1 MB echo 4-14 % on the MI355X host,
    // profiles/r04/inl_ab: removed in round 5.)
    seal_inline(*tx_pend_);
    tx_pend_->clear();
    inline_tx_batches_++;
    return;
  }
  if (!lane_fd_ || lane_fd_->src != t.fd || lane_fd_->gen != t.gen) lane_fd_ = std::make_shared<LaneFd>(t.fd, t.gen);
  auto b = std::move(tx_pend_);
  tx_pend_ = tx_pool_->get();
  lane_tx_batches_++;
  // Seal stage, then the send stage on its own thread: while one batch is
  // in sendmmsg the next is being encrypted (wire order is the batch order).
  // (Both stages on one thread lost: 0.633 against 0.729 of direct on the
  // 1200-MTU 64 x 1 MB echo, profiles/r04/pipe_ab.)
  Lane* send_lane = tx_send_lane_.get();
  tx_lane_->submit([b = std::move(b), st = tx_state_, k = keys_, fd = lane_fd_, to = t.to, co = t.coalesce,
                    pool = tx_pool_, send_lane]() mutable {
    auto sb = st->get_sealed();
    st->seal(*b, *k, co, *sb);
    b->clear();  // the body references go here, once the records are sealed
    pool->put(std::move(b));
    send_lane->submit([sb = std::move(sb), st, fd = std::move(fd), to]() mutable {
      st->send(*sb, fd->fd, to);
      st->put_sealed(std::move(sb));
    });
  });
}

void DtlsTransport::commit_rx() {
  if (rx_pend_.recs.empty()) return;
  if (closed_) {
    rx_pend_ = RxBatch();
    return;
  }
  auto self = shared_from_this();
  if (rx_outstanding_ == 0 && rx_pend_.bytes < datapath_inline_bytes()) {
    RxBatch b = std::move(rx_pend_);
    rx_pend_ = RxBatch();
    batching_ = true;
    for (auto& r : b.recs) {
      uint8_t* pt;
      size_t ptl;
      if (!fast_decrypt(r.rec, r.len, r.type, r.seq, &pt, &ptl)) continue;
      if (!deliver_plain_take(r.owner, r.type, pt, ptl)) break;
    }
    batching_ = false;
    flush_batch();
    return;
  }
  auto b = std::make_shared<RxBatch>(std::move(rx_pend_));
  rx_pend_ = RxBatch();
  rx_outstanding_++;
  lane_rx_batches_++;
  std::weak_ptr<DtlsTransport> w = self;
  Reactor* r = &r_;
  rx_lane_->submit([b, k = keys_, w, r] {
    for (auto& x : b->recs) {
      size_t ptl = 0;
      x.ok = open_record(*k->r, k->riv, x.rec, x.len, &x.pt, &ptl);
      x.ptl = uint32_t(ptl);
    }
    r->post_threadsafe([b, w] {
      if (auto s = w.lock()) s->rx_done(*b);
    });
  });
}

// Opened records back on the association thread, in receive order: the
// replay window (only authenticated records move it), then up the stack.
void DtlsTransport::rx_done(RxBatch& b) {
  rx_outstanding_--;
  deliver_opened(b);
}

// A burst's records go up as one batch (on_data_batch): the receiver takes
// its references once per burst instead of once per record.
void DtlsTransport::deliver_opened(RxBatch& b) {
  if (closed_) return;
  auto self = shared_from_this();
  batching_ = true;
  for (auto& x : b.recs) {
    if (!x.ok || replay_seen(x.seq)) {
      LOG_TRACE(kT, "dropping DTLS record that fails authentication or replay check");
      rx_dropped_++;
      continue;
    }
    replay_mark(x.seq);
    if (!deliver_plain_take(x.owner, x.type, x.pt, x.ptl)) break;
  }
  batching_ = false;
  flush_batch();
}

bool DtlsTransport::send(const uint8_t* p, size_t n) {
  iovec v{const_cast<uint8_t*>(p), n};
  return send(&v, nullptr, 1);
}

bool DtlsTransport::send(const iovec* iov, const Bytes* const* owners, int cnt) {
  if (!connected_ || closed_) return false;
  if (fast_tx_ && tx_pend_) {  // lanes: sealed at commit_tx (end of this flush)
    tx_pend_->add(wseq_++, kAppData, iov, owners, cnt);
    return true;
  }
  size_t total = 0;
  for (int i = 0; i < cnt; i++) total += iov[i].iov_len;
  if (fast_tx_) {
    size_t rec = kRecHdr + kExplicit + total + kTag;
    if (reserve_) {
      uint8_t* o = reserve_(rec);
      if (!fast_encrypt_into(o, kAppData, iov, cnt, total)) return false;
      commit_(rec);
    } else {
      if (scratch_.size() < rec) scratch_.resize(rec);
      if (!fast_encrypt_into(scratch_.data(), kAppData, iov, cnt, total)) return false;
      if (write_) write_(scratch_.data(), rec);
    }
    return true;
  }
  const void* p = iov[0].iov_base;
  if (cnt > 1) {
    scratch_.resize(total);
    size_t o = 0;
    for (int i = 0; i < cnt; i++) {
      memcpy(scratch_.data() + o, iov[i].iov_base, iov[i].iov_len);
      o += iov[i].iov_len;
    }
    p = scratch_.data();
  }
  ERR_clear_error();
  int rc = SSL_write(ssl_, p, int(total));
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
  commit_tx();  // records of this flush go before the close_notify
  if (fast_tx_ && connected_) {
    static const uint8_t kCloseNotify[2] = {1, 0};
    iovec v{const_cast<uint8_t*>(kCloseNotify), 2};
    uint8_t rec[kRecHdr + kExplicit + 2 + kTag];
    if (fast_encrypt_into(rec, kAlert, &v, 1, 2) && write_) write_(rec, sizeof rec);
  } else if (ssl_ && connected_) {
    SSL_shutdown(ssl_);
  }
  closed_ = true;
  if (timer_) r_.cancel(timer_);
  timer_ = 0;
}

}  // namespace p2pt::rtc
