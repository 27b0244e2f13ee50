// Hashes, MACs, checksums, encodings and randomness used across the stack.
//   - SHA-1/base64: WebSocket accept key (RFC 6455 §4.2.2)
//   - HMAC-SHA1 + CRC-32: STUN MESSAGE-INTEGRITY / FINGERPRINT (RFC 5389 §15.4-15.5)
//   - SHA-256: DTLS certificate fingerprints in SDP (RFC 8122)
//   - CRC-32c: SCTP packet checksum (RFC 9260 App. B), hardware SSE4.2 path
//   - UUIDv4: signal-server peer ids (reference signal-server/src/index.ts:131)
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace p2pt {

std::array<uint8_t, 20> sha1(const void* p, size_t n);
std::array<uint8_t, 32> sha256(const void* p, size_t n);
std::array<uint8_t, 20> hmac_sha1(const void* key, size_t klen, const void* p, size_t n);
std::array<uint8_t, 32> hmac_sha256(const void* key, size_t klen, const void* p, size_t n);
// Constant-time equality (MAC comparison).
bool equal_ct(std::string_view a, std::string_view b);
std::array<uint8_t, 16> md5(const void* p, size_t n);

std::string base64_encode(const void* p, size_t n);
bool base64_decode(std::string_view s, std::vector<uint8_t>& out);
std::string hex_encode(const void* p, size_t n, bool upper = false, char sep = 0);

void random_bytes(void* p, size_t n);
uint32_t random_u32();
uint64_t random_u64();
// Random string over [A-Za-z0-9+/] (ICE ufrag/pwd alphabet, RFC 8839 §5.4).
std::string random_ice_chars(size_t n);
std::string uuid4();

uint32_t crc32_ieee(const void* p, size_t n, uint32_t crc = 0);
uint32_t crc32c(const void* p, size_t n, uint32_t crc = 0);

}  // namespace p2pt
