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

std::array<uint8_t, 32> hmac_sha256(const void* key, size_t klen, const void* p, size_t n) {
  std::array<uint8_t, 32> out{};
  unsigned int len = 0;
  HMAC(EVP_sha256(), key, int(klen), static_cast<const uint8_t*>(p), n, out.data(), &len);
  return out;
}

bool equal_ct(std::string_view a, std::string_view b) {
  return a.size() == b.size() && CRYPTO_memcmp(a.data(), b.data(), a.size()) == 0;
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

// CRC-32c (Castagnoli) via the SSE4.2 crc32 instruction. One crc32q has a
// 3-cycle latency but issues every cycle, so buffers of >= 3 lanes are
// checksummed as three independent chains over adjacent blocks that are then
// merged with a GF(2) multiply by x^(8*len) mod P (the zlib crc32_combine
// identity on raw registers). That is ~3x the single-chain rate and keeps the
// SCTP checksum of 16 KB packets well below the AES-GCM cost.
namespace {
constexpr uint32_t kCrc32cPoly = 0x82F63B78u;  // reflected

uint32_t gf2_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ kCrc32cPoly : b >> 1;
  }
  return p;
}

// x^(8*n) mod P.
uint32_t gf2_x8n(size_t n) {
  uint32_t x2n[32];
  uint32_t p = 1u << 30;  // x^1
  x2n[0] = p;
  for (int k = 1; k < 32; k++) x2n[k] = p = gf2_multmodp(p, p);
  p = 1u << 31;  // x^0
  unsigned k = 3;
  while (n) {
    if (n & 1) p = gf2_multmodp(x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

constexpr size_t kLane = 1024;  // bytes per chain per round
const uint32_t kShift1 = gf2_x8n(kLane);
const uint32_t kShift2 = gf2_x8n(2 * kLane);
}  // namespace

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint64_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = _mm_crc32_u8(uint32_t(c), *p++);
    n--;
  }
  while (n >= 3 * kLane) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t* q = p;
    for (size_t i = 0; i < kLane; i += 8) {
      uint64_t v0, v1, v2;
      memcpy(&v0, q + i, 8);
      memcpy(&v1, q + kLane + i, 8);
      memcpy(&v2, q + 2 * kLane + i, 8);
      c = _mm_crc32_u64(c, v0);
      c1 = _mm_crc32_u64(c1, v1);
      c2 = _mm_crc32_u64(c2, v2);
    }
    c = gf2_multmodp(kShift2, uint32_t(c)) ^ gf2_multmodp(kShift1, uint32_t(c1)) ^ uint32_t(c2);
    p += 3 * kLane;
    n -= 3 * kLane;
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
