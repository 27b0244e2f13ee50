// STUN (RFC 5389/8489) message codec with the ICE (RFC 8445) and TURN
// (RFC 8656) attributes this stack needs.
//
// Replaces the `stun` 0.6 crate used by webrtc-rs in the reference (via
// webrtc-ice; reference tunnel/Cargo.lock). Verified against the RFC 5769
// test vectors in native/tests.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "core/net.h"

namespace p2pt::stun {

constexpr uint32_t kMagic = 0x2112A442;

// Message types (method | class bits).
enum : uint16_t {
  kBindingRequest = 0x0001,
  kBindingSuccess = 0x0101,
  kBindingError = 0x0111,
  kBindingIndication = 0x0011,
  kAllocateRequest = 0x0003,
  kAllocateSuccess = 0x0103,
  kAllocateError = 0x0113,
  kRefreshRequest = 0x0004,
  kRefreshSuccess = 0x0104,
  kRefreshError = 0x0114,
  kSendIndication = 0x0016,
  kDataIndication = 0x0017,
  kCreatePermissionRequest = 0x0008,
  kCreatePermissionSuccess = 0x0108,
  kCreatePermissionError = 0x0118,
  kChannelBindRequest = 0x0009,
  kChannelBindSuccess = 0x0109,
  kChannelBindError = 0x0119,
};

// Attribute types.
enum : uint16_t {
  kMappedAddress = 0x0001,
  kUsername = 0x0006,
  kMessageIntegrity = 0x0008,
  kErrorCode = 0x0009,
  kUnknownAttributes = 0x000A,
  kChannelNumber = 0x000C,
  kLifetime = 0x000D,
  kXorPeerAddress = 0x0012,
  kData = 0x0013,
  kRealm = 0x0014,
  kNonce = 0x0015,
  kXorRelayedAddress = 0x0016,
  kRequestedTransport = 0x0019,
  kXorMappedAddress = 0x0020,
  kPriority = 0x0024,
  kUseCandidate = 0x0025,
  kSoftware = 0x8022,
  kFingerprint = 0x8028,
  kIceControlled = 0x8029,
  kIceControlling = 0x802A,
};

struct Attr {
  uint16_t type;
  std::string value;
};

class Message {
 public:
  uint16_t type = 0;
  uint8_t tid[12] = {};
  std::vector<Attr> attrs;
  // Offsets into the parsed buffer (for integrity verification); -1 if absent.
  int integrity_off = -1;
  int fingerprint_off = -1;

  static Message make(uint16_t type);  // random transaction id
  void add(uint16_t t, std::string v) { attrs.push_back({t, std::move(v)}); }
  void add(uint16_t t, const void* p, size_t n) { attrs.push_back({t, std::string(static_cast<const char*>(p), n)}); }
  void add_u32(uint16_t t, uint32_t v);
  void add_u64(uint16_t t, uint64_t v);
  void add_xor_addr(uint16_t t, const SockAddr& a);
  void add_error(int code, const std::string& reason);

  const Attr* get(uint16_t t) const;
  bool get_u32(uint16_t t, uint32_t& v) const;
  bool get_u64(uint16_t t, uint64_t& v) const;
  bool get_xor_addr(uint16_t t, SockAddr& out) const;
  bool get_addr(uint16_t t, SockAddr& out) const;  // plain MAPPED-ADDRESS
  int error_code() const;                          // 0 if none
  std::string tid_key() const { return std::string(reinterpret_cast<const char*>(tid), 12); }

  // Serialise; if `key` is non-null appends MESSAGE-INTEGRITY (HMAC-SHA1),
  // then FINGERPRINT when requested.
  std::vector<uint8_t> serialize(const std::string* key, bool fingerprint) const;
  static bool parse(const uint8_t* p, size_t n, Message& out);

  uint16_t method() const { return type & 0x3EEF; }
  int cls() const { return ((type & 0x0100) >> 7) | ((type & 0x0010) >> 4); }  // 0 req,1 ind,2 ok,3 err
};

// First-byte demultiplexing (RFC 7983) + magic-cookie check.
bool looks_like_stun(const uint8_t* p, size_t n);
bool verify_integrity(const uint8_t* raw, size_t n, const Message& m, const std::string& key);
bool verify_fingerprint(const uint8_t* raw, size_t n, const Message& m);
// Long-term credential key: MD5(username ":" realm ":" password) (RFC 8489 §9.2.2).
std::string long_term_key(const std::string& user, const std::string& realm, const std::string& pass);

}  // namespace p2pt::stun
