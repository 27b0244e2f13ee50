#include "core/crypto.h"

#include <nmmintrin.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>

#include <cstring>
#include <stdexcept>

namespace p2pt {

namespace {
template <size_t N>
std::array<uint8_t, N> digest(const EVP_MD* md, const void* p, size_t n) {
  std::array<uint8_t, N> out{};
  unsigned int len = 0;
  EVP_Digest(p, n, out.data(), &len, md, nullptr);
  return out;
}
}  // namespace

std::array<uint8_t, 20> sha1(const void* p, size_t n) { return digest<20>(EVP_sha1(), p, n); }
std::array<uint8_t, 32> sha256(const void* p, size_t n) { return digest<32>(EVP_sha256(), p, n); }
std::array<uint8_t, 16> md5(const void* p, size_t n) { return digest<16>(EVP_md5(), p, n); }

std::array<uint8_t, 20> hmac_sha1(const void* key, size_t klen, const void* p, size_t n) {
  std::array<uint8_t, 20> out{};
  unsigned int len = 0;
  HMAC(EVP_sha1(), key, int(klen), static_cast<const uint8_t*>(p), n, out.data(), &len);
  return out;
}

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  std::string out;
  out.reserve((n + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = uint32_t(p[i]) << 16 | uint32_t(p[i + 1]) << 8 | p[i + 2];
    out.push_back(kB64[v >> 18]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(kB64[(v >> 6) & 63]);
    out.push_back(kB64[v & 63]);
  }
  if (n - i == 1) {
    uint32_t v = uint32_t(p[i]) << 16;
    out.push_back(kB64[v >> 18]);
    out.push_back(kB64[(v >> 12) & 63]);
    out += "==";
  } else if (n - i == 2) {
    uint32_t v = uint32_t(p[i]) << 16 | uint32_t(p[i + 1]) << 8;
    out.push_back(kB64[v >> 18]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(kB64[(v >> 6) & 63]);
    out.push_back('=');
  }
  return out;
}

bool base64_decode(std::string_view s, std::vector<uint8_t>& out) {
  int8_t map[256];
  memset(map, -1, sizeof map);
  for (int i = 0; i < 64; i++) map[uint8_t(kB64[i])] = int8_t(i);
  uint32_t acc = 0;
  int bits = 0;
  size_t pad = 0;
  for (char c : s) {
    if (c == '=') {
      pad++;
      continue;
    }
    if (pad) return false;
    int8_t v = map[uint8_t(c)];
    if (v < 0) return false;
    acc = (acc << 6) | uint32_t(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(uint8_t(acc >> bits));
    }
  }
  return pad <= 2;
}

std::string hex_encode(const void* data, size_t n, bool upper, char sep) {
  const char* d = upper ? "0123456789ABCDEF" : "0123456789abcdef";
  const uint8_t* p = static_cast<const uint8_t*>(data);
  std::string out;
  for (size_t i = 0; i < n; i++) {
    if (sep && i) out.push_back(sep);
    out.push_back(d[p[i] >> 4]);
    out.push_back(d[p[i] & 15]);
  }
  return out;
}

void random_bytes(void* p, size_t n) {
  if (RAND_bytes(static_cast<unsigned char*>(p), int(n)) != 1) throw std::runtime_error("RAND_bytes failed");
}
uint32_t random_u32() {
  uint32_t v;
  random_bytes(&v, sizeof v);
  return v;
}
uint64_t random_u64() {
  uint64_t v;
  random_bytes(&v, sizeof v);
  return v;
}

std::string random_ice_chars(size_t n) {
  std::string s(n, 'a');
  std::vector<uint8_t> r(n);
  random_bytes(r.data(), n);
  for (size_t i = 0; i < n; i++) s[i] = kB64[r[i] & 63];
  return s;
}

std::string uuid4() {
  uint8_t b[16];
  random_bytes(b, 16);
  b[6] = uint8_t((b[6] & 0x0F) | 0x40);
  b[8] = uint8_t((b[8] & 0x3F) | 0x80);
  std::string h = hex_encode(b, 16);
  return h.substr(0, 8) + "-" + h.substr(8, 4) + "-" + h.substr(12, 4) + "-" + h.substr(16, 4) + "-" +
         h.substr(20);
}

namespace {
struct Crc32Table {
  uint32_t t[256];
  Crc32Table() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[i] = c;
    }
  }
};
}  // namespace

uint32_t crc32_ieee(const void* data, size_t n, uint32_t crc) {
  static const Crc32Table tab;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  crc = ~crc;
  for (size_t i = 0; i < n; i++) crc = tab.t[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

// CRC-32c (Castagnoli) via the SSE4.2 crc32 instruction: 8 bytes/cycle-ish,
// which keeps the SCTP checksum far below the AES-GCM cost per packet.
uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint64_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = _mm_crc32_u8(uint32_t(c), *p++);
    n--;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8(uint32_t(c), *p++);
  return ~uint32_t(c);
}

}  // namespace p2pt
