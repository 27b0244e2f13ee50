#include "rtc/stun.h"

#include <arpa/inet.h>

#include <cstring>

#include "core/buf.h"
#include "core/crypto.h"

namespace p2pt::stun {

Message Message::make(uint16_t type) {
  Message m;
  m.type = type;
  random_bytes(m.tid, 12);
  return m;
}

void Message::add_u32(uint16_t t, uint32_t v) {
  uint8_t b[4];
  wr32(b, v);
  add(t, b, 4);
}

void Message::add_u64(uint16_t t, uint64_t v) {
  uint8_t b[8];
  wr32(b, uint32_t(v >> 32));
  wr32(b + 4, uint32_t(v));
  add(t, b, 8);
}

void Message::add_xor_addr(uint16_t t, const SockAddr& a) {
  std::string v;
  v.push_back(0);
  uint16_t xport = uint16_t(a.port() ^ (kMagic >> 16));
  if (a.family() == AF_INET) {
    v.push_back(1);
    v.push_back(char(xport >> 8));
    v.push_back(char(xport));
    uint32_t ip = ntohl(reinterpret_cast<const sockaddr_in*>(&a.ss)->sin_addr.s_addr) ^ kMagic;
    uint8_t b[4];
    wr32(b, ip);
    v.append(reinterpret_cast<char*>(b), 4);
  } else {
    v.push_back(2);
    v.push_back(char(xport >> 8));
    v.push_back(char(xport));
    uint8_t x[16];
    memcpy(x, &reinterpret_cast<const sockaddr_in6*>(&a.ss)->sin6_addr, 16);
    uint8_t mask[16];
    wr32(mask, kMagic);
    memcpy(mask + 4, tid, 12);
    for (int i = 0; i < 16; i++) x[i] ^= mask[i];
    v.append(reinterpret_cast<char*>(x), 16);
  }
  add(t, std::move(v));
}

void Message::add_error(int code, const std::string& reason) {
  std::string v(4, '\0');
  v[2] = char(code / 100);
  v[3] = char(code % 100);
  v += reason;
  add(kErrorCode, std::move(v));
}

const Attr* Message::get(uint16_t t) const {
  for (auto& a : attrs)
    if (a.type == t) return &a;
  return nullptr;
}

bool Message::get_u32(uint16_t t, uint32_t& v) const {
  const Attr* a = get(t);
  if (!a || a->value.size() != 4) return false;
  v = rd32(reinterpret_cast<const uint8_t*>(a->value.data()));
  return true;
}

bool Message::get_u64(uint16_t t, uint64_t& v) const {
  const Attr* a = get(t);
  if (!a || a->value.size() != 8) return false;
  v = rd64(reinterpret_cast<const uint8_t*>(a->value.data()));
  return true;
}

static bool decode_addr(const std::string& v, bool x, const uint8_t* tid, SockAddr& out) {
  if (v.size() < 8) return false;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(v.data());
  uint16_t port = rd16(p + 2);
  if (x) port ^= uint16_t(kMagic >> 16);
  out = SockAddr{};
  if (p[1] == 1) {
    auto* s = reinterpret_cast<sockaddr_in*>(&out.ss);
    s->sin_family = AF_INET;
    s->sin_port = htons(port);
    uint32_t ip = rd32(p + 4);
    if (x) ip ^= kMagic;
    s->sin_addr.s_addr = htonl(ip);
    out.len = sizeof(sockaddr_in);
    return true;
  }
  if (p[1] == 2 && v.size() >= 20) {
    auto* s = reinterpret_cast<sockaddr_in6*>(&out.ss);
    s->sin6_family = AF_INET6;
    s->sin6_port = htons(port);
    uint8_t a[16];
    memcpy(a, p + 4, 16);
    if (x) {
      uint8_t mask[16];
      wr32(mask, kMagic);
      memcpy(mask + 4, tid, 12);
      for (int i = 0; i < 16; i++) a[i] ^= mask[i];
    }
    memcpy(&s->sin6_addr, a, 16);
    out.len = sizeof(sockaddr_in6);
    return true;
  }
  return false;
}

bool Message::get_xor_addr(uint16_t t, SockAddr& out) const {
  const Attr* a = get(t);
  return a && decode_addr(a->value, true, tid, out);
}

bool Message::get_addr(uint16_t t, SockAddr& out) const {
  const Attr* a = get(t);
  return a && decode_addr(a->value, false, tid, out);
}

int Message::error_code() const {
  const Attr* a = get(kErrorCode);
  if (!a || a->value.size() < 4) return 0;
  return (a->value[2] & 7) * 100 + uint8_t(a->value[3]);
}

std::vector<uint8_t> Message::serialize(const std::string* key, bool fingerprint) const {
  std::vector<uint8_t> out;
  out.reserve(128);
  ByteWriter w(out);
  w.u16(type);
  w.u16(0);
  w.u32(kMagic);
  w.bytes(tid, 12);
  for (auto& a : attrs) {
    if (a.type == kMessageIntegrity || a.type == kFingerprint) continue;
    w.u16(a.type);
    w.u16(uint16_t(a.value.size()));
    w.bytes(a.value);
    w.zeros((4 - a.value.size() % 4) % 4);
  }
  if (key) {
    wr16(out.data() + 2, uint16_t(out.size() - 20 + 24));
    auto mac = hmac_sha1(key->data(), key->size(), out.data(), out.size());
    w.u16(kMessageIntegrity);
    w.u16(20);
    w.bytes(mac.data(), 20);
  }
  if (fingerprint) {
    wr16(out.data() + 2, uint16_t(out.size() - 20 + 8));
    uint32_t crc = crc32_ieee(out.data(), out.size()) ^ 0x5354554e;
    w.u16(kFingerprint);
    w.u16(4);
    w.u32(crc);
  }
  wr16(out.data() + 2, uint16_t(out.size() - 20));
  return out;
}

bool looks_like_stun(const uint8_t* p, size_t n) {
  return n >= 20 && p[0] < 4 && rd32(p + 4) == kMagic && (rd16(p + 2) & 3) == 0 && size_t(rd16(p + 2)) + 20 <= n;
}

bool Message::parse(const uint8_t* p, size_t n, Message& out) {
  if (!looks_like_stun(p, n)) return false;
  out = Message{};
  out.type = rd16(p);
  memcpy(out.tid, p + 8, 12);
  size_t len = rd16(p + 2);
  size_t off = 20, end = 20 + len;
  while (off + 4 <= end) {
    uint16_t t = rd16(p + off), l = rd16(p + off + 2);
    if (off + 4 + l > end) return false;
    if (t == kMessageIntegrity) out.integrity_off = int(off);
    if (t == kFingerprint) out.fingerprint_off = int(off);
    out.attrs.push_back({t, std::string(reinterpret_cast<const char*>(p + off + 4), l)});
    off += 4 + l + (4 - l % 4) % 4;
  }
  return off == end || off == end + 0;
}

bool verify_integrity(const uint8_t* raw, size_t n, const Message& m, const std::string& key) {
  if (m.integrity_off < 0 || size_t(m.integrity_off) + 24 > n) return false;
  std::vector<uint8_t> buf(raw, raw + m.integrity_off);
  wr16(buf.data() + 2, uint16_t(m.integrity_off - 20 + 24));
  auto mac = hmac_sha1(key.data(), key.size(), buf.data(), buf.size());
  return memcmp(mac.data(), raw + m.integrity_off + 4, 20) == 0;
}

bool verify_fingerprint(const uint8_t* raw, size_t n, const Message& m) {
  if (m.fingerprint_off < 0 || size_t(m.fingerprint_off) + 8 > n) return false;
  std::vector<uint8_t> buf(raw, raw + m.fingerprint_off);
  wr16(buf.data() + 2, uint16_t(m.fingerprint_off - 20 + 8));
  uint32_t crc = crc32_ieee(buf.data(), buf.size()) ^ 0x5354554e;
  return crc == rd32(raw + m.fingerprint_off + 4);
}

std::string long_term_key(const std::string& user, const std::string& realm, const std::string& pass) {
  std::string s = user + ":" + realm + ":" + pass;
  auto d = md5(s.data(), s.size());
  return std::string(reinterpret_cast<const char*>(d.data()), 16);
}

}  // namespace p2pt::stun
