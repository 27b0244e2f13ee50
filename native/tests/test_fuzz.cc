// Mutation fuzzing of every wire parser: seeded random
// mutations (bit flips, byte sets, truncation, insertion, boundary integers,
// slice duplication) of valid inputs, fed to the tunnel-frame decoder, JSON,
// STUN, HTTP heads + body decoder, WebSocket frame parser, SDP and an
// established SCTP association. Deterministic (fixed seeds). Plain builds
// check round-trip invariants; `make sanitize` runs the same cases under
// ASan/UBSan. P2PT_FUZZ_ITERS scales the iteration count (default 3000).
#include <cstdlib>
#include <random>

#include "core/crypto.h"
#include "core/json.h"
#include "core/reactor.h"
#include "http/http.h"
#include "proto/frame.h"
#include "rtc/sctp.h"
#include "rtc/sdp.h"
#include "rtc/stun.h"
#include "tests/testing.h"
#include "ws/ws.h"

using namespace p2pt;

namespace {

size_t iters() {
  const char* e = getenv("P2PT_FUZZ_ITERS");
  return e ? size_t(strtoul(e, nullptr, 10)) : 3000;
}

using Buf = std::vector<uint8_t>;

Buf to_buf(std::string_view s) { return Buf(s.begin(), s.end()); }

struct Mutator {
  std::mt19937 g;
  explicit Mutator(uint32_t seed) : g(seed) {}
  size_t below(size_t n) { return n ? size_t(g()) % n : 0; }

  // `keep` leading bytes are never touched (e.g. an SCTP common header).
  Buf mutate(const Buf& seed, size_t keep = 0) {
    Buf v = seed;
    if (below(32) == 0) {  // occasionally: pure noise after the prefix
      v.resize(std::min(v.size(), keep));
      size_t n = below(256);
      for (size_t i = 0; i < n; i++) v.push_back(uint8_t(g()));
      return v;
    }
    int rounds = 1 + int(below(6));
    for (int r = 0; r < rounds; r++) {
      size_t span = v.size() > keep ? v.size() - keep : 0;
      switch (below(7)) {
        case 0:
          if (span) v[keep + below(span)] ^= uint8_t(1u << below(8));
          break;
        case 1:
          if (span) v[keep + below(span)] = uint8_t(g());
          break;
        case 2:
          if (span) v.resize(keep + below(span));
          break;
        case 3: {
          size_t pos = keep + below(span + 1), n = 1 + below(16);
          for (size_t i = 0; i < n; i++) v.insert(v.begin() + long(pos), uint8_t(g()));
          break;
        }
        case 4: {  // boundary integers, big-endian, 1/2/4 bytes
          static const uint32_t vals[] = {0, 1, 0x7f, 0x80, 0xff, 0x7fff, 0x8000, 0xffff, 0x7fffffff, 0xffffffff};
          uint32_t x = vals[below(10)];
          size_t w = size_t(1) << below(3);
          if (span >= w) {
            size_t pos = keep + below(span - w + 1);
            for (size_t i = 0; i < w; i++) v[pos + i] = uint8_t(x >> (8 * (w - 1 - i)));
          }
          break;
        }
        case 5:
          if (span) {  // duplicate a slice
            size_t a = keep + below(span), n = 1 + below(std::min<size_t>(64, v.size() - a));
            Buf s(v.begin() + long(a), v.begin() + long(a + n));
            v.insert(v.begin() + long(keep + below(span)), s.begin(), s.end());
          }
          break;
        case 6:
          if (span > 1) std::swap(v[keep + below(span)], v[keep + below(span)]);
          break;
      }
    }
    return v;
  }
};

}  // namespace

TEST(fuzz_frame_decode) {
  std::vector<Buf> seeds;
  proto::Hello h;
  seeds.push_back(to_buf(proto::make_hello(h).encode().str()));
  proto::RequestHeaders rq;
  rq.stream_id = 7;
  rq.method = "POST";
  rq.path = "/v1/chat/completions?x=1";
  proto::header_set(rq.headers, "content-type", "application/json");
  seeds.push_back(to_buf(proto::make_req_headers(rq).encode().str()));
  seeds.push_back(to_buf(proto::make_body(proto::MsgType::ResBody, 0xffffffffu, Bytes::copy("data: {}\n\n", 10)).encode().str()));
  seeds.push_back(to_buf(proto::make_empty(proto::MsgType::Ping, 0).encode().str()));
  seeds.push_back(to_buf(proto::make_error(3, "upstream error: boom").encode().str()));
  Mutator m(1);
  size_t ok = 0;
  for (size_t i = 0; i < iters() * 4; i++) {
    Buf in = m.mutate(seeds[i % seeds.size()]);
    proto::Frame f;
    std::string err;
    if (proto::decode(Bytes::copy(in.data(), in.size()), f, &err)) {
      ok++;
      CHECK(f.encode().str() == std::string(in.begin(), in.end()));  // lossless round trip
      // Handshake/header payloads go through the JSON parser on receipt.
      Json j;
      (void)Json::parse(f.payload.str(), j, nullptr);
    } else {
      CHECK(!err.empty());
    }
  }
  CHECK(ok > 0);
}

TEST(fuzz_json) {
  std::vector<Buf> seeds = {
      to_buf(R"({"proto":"httptunnel","min_version":1,"max_version":1,"features":["sse","cancel"]})"),
      to_buf(R"({"stream_id":4294967295,"method":"GET","path":"/a?b=c","headers":{"x":"é😀\n\"q\""}})"),
      to_buf(R"([1,-2.5e-3,true,false,null,{"a":[[[]]]},"\\\/\b\f\r\t"])"),
      to_buf(R"({"type":"candidate","candidate":"{\"candidate\":\"candidate:1 1 udp 1 1.2.3.4 5 typ host\"}"})"),
  };
  Mutator m(2);
  for (size_t i = 0; i < iters() * 4; i++) {
    Buf in = m.mutate(seeds[i % seeds.size()]);
    Json j;
    std::string err;
    if (Json::parse(std::string_view(reinterpret_cast<const char*>(in.data()), in.size()), j, &err)) {
      std::string d1 = j.dump();
      Json j2;
      CHECK(Json::parse(d1, j2, nullptr));
      CHECK(j2.dump() == d1);  // dump is a fixed point
    }
  }
}

TEST(fuzz_stun) {
  using namespace p2pt::rtc;
  std::vector<Buf> seeds;
  std::string key = "VOkJxbRl1RmTxUk/WvJxBt";
  auto req = p2pt::stun::Message::make(0x0001);
  req.add(0x0006, "evtj:h6vY");
  req.add_u32(0x0024, 0x6e0001ff);
  req.add_u64(0x802A, 0x932ff9b151263b36ull);
  req.add(0x0025, "");
  seeds.push_back(req.serialize(&key, true));
  auto resp = p2pt::stun::Message::make(0x0101);
  SockAddr a;
  SockAddr::parse("192.0.2.1", 32853, a);
  resp.add_xor_addr(0x0020, a);
  seeds.push_back(resp.serialize(&key, true));
  auto err = p2pt::stun::Message::make(0x0113);
  err.add_error(401, "Unauthorized");
  err.add(0x0014, "example.org");
  err.add(0x0015, "f//499k954d6OL34oL9FSTvy64sA");
  seeds.push_back(err.serialize(nullptr, true));
  Mutator m(3);
  size_t parsed = 0;
  for (size_t i = 0; i < iters() * 4; i++) {
    Buf in = m.mutate(seeds[i % seeds.size()]);
    p2pt::stun::Message msg;
    (void)p2pt::stun::looks_like_stun(in.data(), in.size());
    if (p2pt::stun::Message::parse(in.data(), in.size(), msg)) {
      parsed++;
      (void)p2pt::stun::verify_integrity(in.data(), in.size(), msg, key);
      (void)p2pt::stun::verify_fingerprint(in.data(), in.size(), msg);
      SockAddr out;
      (void)msg.get_xor_addr(0x0020, out);
      (void)msg.get_addr(0x0001, out);
      (void)msg.error_code();
      uint32_t u32;
      uint64_t u64;
      (void)msg.get_u32(0x0024, u32);
      (void)msg.get_u64(0x802A, u64);
    }
  }
  CHECK(parsed > 0);
}

TEST(fuzz_http) {
  using namespace p2pt::http;
  std::vector<Buf> seeds = {
      to_buf("POST /v1/chat/completions HTTP/1.1\r\nHost: a\r\nContent-Length: 5\r\n\r\nhello"),
      to_buf("GET /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n"),
      to_buf("HTTP/1.1 200 OK\r\nContent-Type: text/event-stream\r\nTransfer-Encoding: chunked\r\n\r\n"
             "1a;ext=1\r\ndata: {\"x\":1}\n\n0123456789\r\n0\r\nTrailer: v\r\n\r\n"),
      to_buf("HTTP/1.0 200 OK\r\nContent-Type: text/plain\r\n\r\nok"),
  };
  Mutator m(4);
  for (size_t i = 0; i < iters() * 4; i++) {
    Buf in = m.mutate(seeds[i % seeds.size()]);
    std::string_view sv(reinterpret_cast<const char*>(in.data()), in.size());
    Head h;
    size_t used = 0;
    std::string err;
    bool response = sv.rfind("HTTP/", 0) == 0;
    ParseResult r = response ? parse_response_head(sv, h, used, &err) : parse_request_head(sv, h, used, &err);
    if (r != ParseResult::Done) continue;
    CHECK(used <= in.size());
    uint64_t len = 0;
    BodyDecoder::Mode mode = response ? response_body_mode(h, "GET", len) : request_body_mode(h, len, &err);
    BodyDecoder bd;
    bd.reset(mode, len);
    // Feed the body in random splits; the decoder must never claim more than it got.
    size_t off = used;
    size_t delivered = 0;
    while (off < in.size() && !bd.done()) {
      size_t n = 1 + m.below(in.size() - off);
      size_t k = bd.feed(in.data() + off, n, [&](const uint8_t*, size_t c) { delivered += c; });
      if (k == SIZE_MAX) break;
      CHECK(k <= n);
      if (k == 0) break;
      off += k;
    }
    (void)bd.on_eof();
    CHECK(delivered <= in.size());
  }
}

TEST(fuzz_ws_frames) {
  std::vector<Buf> seeds;
  for (bool mask : {false, true}) {
    seeds.push_back(to_buf(ws::encode_frame(ws::Op::Text, R"({"type":"join","room":"r"})", mask)));
    seeds.push_back(to_buf(ws::encode_frame(ws::Op::Binary, std::string(300, 'x'), mask)));
    seeds.push_back(to_buf(ws::encode_frame(ws::Op::Ping, "p", mask)));
    seeds.push_back(to_buf(ws::encode_frame(ws::Op::Text, "frag", mask, false) +
                           ws::encode_frame(ws::Op::Cont, "ment", mask)));
    seeds.push_back(to_buf(ws::encode_frame(ws::Op::Close, std::string("\x03\xe8", 2), mask)));
  }
  Mutator m(5);
  for (size_t i = 0; i < iters() * 4; i++) {
    const Buf& seed = seeds[i % seeds.size()];
    Buf in = m.mutate(seed);
    ws::FrameParser p(/*expect_masked=*/(i % seeds.size()) >= seeds.size() / 2, /*max_frame=*/1 << 16);
    size_t off = 0;
    while (off < in.size()) {
      size_t n = 1 + m.below(in.size() - off);
      if (!p.feed(in.data() + off, n, [&](ws::Op, bool, std::string&& payload) { CHECK(payload.size() <= (1u << 16)); }))
        break;
      off += n;
    }
  }
}

TEST(fuzz_sdp) {
  using namespace p2pt::rtc;
  SessionDesc d;
  d.type = "offer";
  d.ice_ufrag = "ufrag";
  d.ice_pwd = "passwordpasswordpassword";
  d.fingerprint = "sha-256 AA:BB:CC";
  d.jumbo = 16000;
  Candidate c;
  Candidate::parse("candidate:1 1 udp 2130706431 127.0.0.1 5000 typ host", c);
  d.candidates.push_back(c);
  Candidate::parse("candidate:2 1 udp 1694498815 203.0.113.7 6000 typ srflx raddr 10.0.0.2 rport 6000", c);
  d.candidates.push_back(c);
  d.end_of_candidates = true;
  std::vector<Buf> seeds = {to_buf(d.to_string())};
  Mutator m(6);
  size_t ok = 0;
  for (size_t i = 0; i < iters() * 2; i++) {
    Buf in = m.mutate(seeds[0]);
    SessionDesc out;
    std::string err;
    if (SessionDesc::parse(std::string(in.begin(), in.end()), out, &err)) {
      ok++;
      SessionDesc again;
      CHECK(SessionDesc::parse(out.to_string(), again, &err));
    }
    Candidate cc;
    std::string line(in.begin(), in.begin() + long(std::min<size_t>(in.size(), 120)));
    (void)Candidate::parse(line, cc);
  }
  CHECK(ok > 0);
}

TEST(fuzz_sctp_packets) {
  using namespace p2pt::rtc;
  // A real exchange between two associations provides the seed packets
  // (INIT, INIT-ACK, COOKIE-ECHO/ACK, DATA, SACK, RE-CONFIG...).
  Reactor r;
  std::vector<Buf> captured;
  std::shared_ptr<SctpAssociation> a, b;
  SctpConfig cfg;
  cfg.sack_delay_us = 0;
  a = SctpAssociation::create(r, cfg, [&](const iovec* iov, const Bytes* const*, int cnt) {
    auto flat = SctpAssociation::flatten(iov, cnt);
    const uint8_t* p = flat.data();
    size_t n = flat.size();
    captured.emplace_back(p, p + n);
    auto pkt = std::make_shared<Buf>(p, p + n);
    r.post([&b, pkt] { if (b) b->on_packet(pkt->data(), pkt->size()); });
  });
  b = SctpAssociation::create(r, cfg, [&](const iovec* iov, const Bytes* const*, int cnt) {
    auto flat = SctpAssociation::flatten(iov, cnt);
    const uint8_t* p = flat.data();
    size_t n = flat.size();
    captured.emplace_back(p, p + n);
    auto pkt = std::make_shared<Buf>(p, p + n);
    r.post([&a, pkt] { if (a) a->on_packet(pkt->data(), pkt->size()); });
  });
  size_t got = 0;
  b->on_message = [&](uint16_t, uint32_t, Bytes) { got++; };
  r.add_flush_hook([&] {
    a->flush();
    b->flush();
  });
  a->connect();
  CHECK(r.run_until([&] { return a->established() && b->established(); }, 2000));
  for (int i = 0; i < 20; i++) a->send(uint16_t(i % 3), 53, {Bytes::copy(std::string(size_t(1 + i * 997), char('a' + i)))});
  a->request_stream_reset(2);
  CHECK(r.run_until([&] { return got >= 20 && a->bytes_in_flight() == 0; }, 5000));
  CHECK(!captured.empty());

  // Mutate chunks behind an intact common header and fix the CRC32c, so the
  // packets reach the chunk parsers of an established association.
  auto victim = b;
  victim->on_message = [](uint16_t, uint32_t, Bytes) {};
  Mutator m(7);
  for (size_t i = 0; i < iters() * 2; i++) {
    Buf in = m.mutate(captured[i % captured.size()], 12);
    if (in.size() >= 12 && m.below(8) != 0) {
      in[8] = in[9] = in[10] = in[11] = 0;
      uint32_t crc = crc32c(in.data(), in.size());
      in[8] = uint8_t(crc);
      in[9] = uint8_t(crc >> 8);
      in[10] = uint8_t(crc >> 16);
      in[11] = uint8_t(crc >> 24);
    }
    victim->on_packet(in.data(), in.size());
    if (i % 64 == 0) r.run_until([] { return false; }, 1);  // let timers / flushes run
  }
  r.run_until([] { return false; }, 5);
  a.reset();
  b.reset();
}
