// STUN codec against the RFC 5769 test vectors, ICE candidate and SDP codecs.
#include <cstring>

#include "rtc/ice.h"
#include "rtc/sdp.h"
#include "rtc/stun.h"
#include "tests/testing.h"

using namespace p2pt;
using namespace p2pt::rtc;

static std::vector<uint8_t> hex(const char* s) {
  std::vector<uint8_t> v;
  int hi = -1;
  for (; *s; s++) {
    int d;
    if (*s >= '0' && *s <= '9') d = *s - '0';
    else if (*s >= 'a' && *s <= 'f') d = *s - 'a' + 10;
    else continue;
    if (hi < 0) hi = d;
    else {
      v.push_back(uint8_t(hi << 4 | d));
      hi = -1;
    }
  }
  return v;
}

// RFC 5769 §2.1 sample request.
static const char* kReq =
    "00 01 00 58 21 12 a4 42 b7 e7 a7 01 bc 34 d6 86 fa 87 df ae"
    "80 22 00 10 53 54 55 4e 20 74 65 73 74 20 63 6c 69 65 6e 74"
    "00 24 00 04 6e 00 01 ff 80 29 00 08 93 2f f9 b1 51 26 3b 36"
    "00 06 00 09 65 76 74 6a 3a 68 36 76 59 20 20 20"
    "00 08 00 14 9a ea a7 0c bf d8 cb 56 78 1e f2 b5 b2 d3 f2 49 c1 b5 71 a2"
    "80 28 00 04 e5 7a 3b cf";
// §2.2 sample IPv4 response.
static const char* kResp4 =
    "01 01 00 3c 21 12 a4 42 b7 e7 a7 01 bc 34 d6 86 fa 87 df ae"
    "80 22 00 0b 74 65 73 74 20 76 65 63 74 6f 72 20"
    "00 20 00 08 00 01 a1 47 e1 12 a6 43"
    "00 08 00 14 2b 91 f5 99 fd 9e 90 c3 8c 74 89 f9 2a f9 ba 53 f0 6b e7 d7"
    "80 28 00 04 c0 7d 4c 96";
// §2.3 sample IPv6 response.
static const char* kResp6 =
    "01 01 00 48 21 12 a4 42 b7 e7 a7 01 bc 34 d6 86 fa 87 df ae"
    "80 22 00 0b 74 65 73 74 20 76 65 63 74 6f 72 20"
    "00 20 00 14 00 02 a1 47 01 13 a9 fa a5 d3 f1 79 bc 25 f4 b5 be d2 b9 d9"
    "00 08 00 14 a3 82 95 4e 4b e6 7b f1 17 84 c9 7c 82 92 c2 75 bf e3 ed 41"
    "80 28 00 04 c8 fb 0b 4c";
static const std::string kPwd = "VOkJxbRl1RmTxUk/WvJxBt";

TEST(stun_rfc5769_request) {
  auto b = hex(kReq);
  stun::Message m;
  CHECK(stun::Message::parse(b.data(), b.size(), m));
  CHECK_EQ(m.type, uint16_t(stun::kBindingRequest));
  CHECK_EQ(m.get(stun::kUsername)->value, std::string("evtj:h6vY"));
  uint32_t prio = 0;
  CHECK(m.get_u32(stun::kPriority, prio) && prio == 0x6e0001ffu);
  CHECK(stun::verify_fingerprint(b.data(), b.size(), m));
  CHECK(stun::verify_integrity(b.data(), b.size(), m, kPwd));
  CHECK(!stun::verify_integrity(b.data(), b.size(), m, "wrong"));
}

TEST(stun_rfc5769_responses) {
  auto b = hex(kResp4);
  stun::Message m;
  CHECK(stun::Message::parse(b.data(), b.size(), m));
  SockAddr a;
  CHECK(m.get_xor_addr(stun::kXorMappedAddress, a));
  CHECK_EQ(a.str(), std::string("192.0.2.1:32853"));
  CHECK(stun::verify_fingerprint(b.data(), b.size(), m));
  CHECK(stun::verify_integrity(b.data(), b.size(), m, kPwd));
  auto b6 = hex(kResp6);
  CHECK(stun::Message::parse(b6.data(), b6.size(), m));
  CHECK(m.get_xor_addr(stun::kXorMappedAddress, a));
  CHECK_EQ(a.str(), std::string("[2001:db8:1234:5678:11:2233:4455:6677]:32853"));
  CHECK(stun::verify_integrity(b6.data(), b6.size(), m, kPwd));
}

TEST(stun_serialize_roundtrip) {
  auto m = stun::Message::make(stun::kBindingRequest);
  m.add(stun::kUsername, "a:b");
  m.add_u64(stun::kIceControlling, 0x0102030405060708ull);
  m.add(stun::kUseCandidate, "");
  SockAddr a;
  SockAddr::parse("10.1.2.3", 4444, a);
  m.add_xor_addr(stun::kXorMappedAddress, a);
  std::string key = "secret";
  auto b = m.serialize(&key, true);
  stun::Message p;
  CHECK(stun::Message::parse(b.data(), b.size(), p));
  CHECK(stun::verify_integrity(b.data(), b.size(), p, key));
  CHECK(stun::verify_fingerprint(b.data(), b.size(), p));
  SockAddr back;
  CHECK(p.get_xor_addr(stun::kXorMappedAddress, back) && back == a);
  uint64_t tb;
  CHECK(p.get_u64(stun::kIceControlling, tb) && tb == 0x0102030405060708ull);
  CHECK(p.get(stun::kUseCandidate) != nullptr);
  CHECK(stun::looks_like_stun(b.data(), b.size()));
  b[0] = 0x16;  // DTLS handshake byte: not STUN
  CHECK(!stun::looks_like_stun(b.data(), b.size()));
}

TEST(candidate_codec) {
  Candidate c;
  CHECK(Candidate::parse("candidate:1966762133 1 udp 2130706431 192.168.1.5 50001 typ host generation 0", c));
  CHECK(c.addr.str() == "192.168.1.5:50001" && c.type == "host" && c.priority == 2130706431u);
  CHECK(Candidate::parse("a=candidate:2 1 UDP 1694498815 203.0.113.7 61000 typ srflx raddr 10.0.0.2 rport 50001", c));
  CHECK(c.type == "srflx" && c.has_related && c.related.str() == "10.0.0.2:50001");
  Candidate back;
  CHECK(Candidate::parse(c.to_sdp(), back));
  CHECK(back.addr == c.addr && back.priority == c.priority);
  CHECK(!Candidate::parse("candidate:1 1 tcp 1 1.2.3.4 9 typ host tcptype active", c));
  CHECK(!Candidate::parse("candidate:1 1 udp 1 abc.local 9 typ host", c));
  CHECK_EQ(candidate_priority("host", 65535), 2130706431u);
}

TEST(sdp_roundtrip) {
  SessionDesc d;
  d.type = "offer";
  d.ice_ufrag = "ufrag";
  d.ice_pwd = "passwordpasswordpassword";
  d.fingerprint = "sha-256 AA:BB";
  d.jumbo = 16000;
  Candidate c;
  Candidate::parse("candidate:1 1 udp 2130706431 127.0.0.1 5000 typ host", c);
  d.candidates.push_back(c);
  d.end_of_candidates = true;
  std::string s = d.to_string();
  CHECK(s.find("m=application 9 UDP/DTLS/SCTP webrtc-datachannel") != std::string::npos);
  SessionDesc p;
  std::string err;
  CHECK(SessionDesc::parse(s, p, &err));
  CHECK(p.ice_ufrag == "ufrag" && p.ice_pwd == d.ice_pwd && p.fingerprint == d.fingerprint);
  CHECK(p.setup == "actpass" && p.sctp_port == 5000 && p.jumbo == 16000);
  CHECK(p.candidates.size() == 1 && p.end_of_candidates);
  // Legacy form.
  std::string legacy =
      "v=0\r\no=- 1 1 IN IP4 0.0.0.0\r\ns=-\r\nt=0 0\r\na=ice-ufrag:u\r\na=ice-pwd:p\r\n"
      "a=fingerprint:SHA-256 01:02\r\nm=application 9 DTLS/SCTP 5001\r\na=setup:active\r\na=sctpmap:5001 webrtc-datachannel 1024\r\n";
  CHECK(SessionDesc::parse(legacy, p, &err));
  CHECK(p.sctp_port == 5001 && p.setup == "active" && p.fingerprint == "sha-256 01:02");
  CHECK(!SessionDesc::parse("v=0\r\n", p, &err));
}
