// Core: JSON, checksums, encodings, reactor timers, frame codec, HTTP parser.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include <openssl/evp.h>

#include "core/aesgcm.h"
#include "core/crypto.h"
#include "core/json.h"
#include "core/net.h"
#include "core/reactor.h"
#include "http/http.h"
#include "proto/frame.h"
#include "tunnel/assoc.h"
#include "tunnel/proxy.h"
#include "tests/testing.h"
#include "ws/ws.h"

using namespace p2pt;

TEST(json_roundtrip) {
  const char* doc = R"({"a":1,"b":[true,false,null],"c":"x\"y\\z\n\t\u0001","d":{"e":-2.5,"f":[]},"g":1e3})";
  Json j;
  std::string err;
  CHECK(Json::parse(doc, j, &err));
  CHECK_EQ(j.get("a")->as_int(), 1);
  CHECK_EQ(j.get("c")->as_string(), std::string("x\"y\\z\n\t\x01"));
  CHECK_EQ(j.get("d")->get("e")->as_double(), -2.5);
  CHECK_EQ(j.get("g")->as_double(), 1000.0);
  Json k;
  CHECK(Json::parse(j.dump(), k, &err));
  CHECK_EQ(k.dump(), j.dump());
  CHECK_EQ(Json(std::string("\x01")).dump(), std::string("\"\\u0001\""));
}

TEST(json_unicode_and_errors) {
  Json j;
  CHECK(Json::parse(R"("\u30de\ud83d\ude00")", j));
  CHECK_EQ(j.as_string(), std::string("\xE3\x83\x9E\xF0\x9F\x98\x80"));
  CHECK(!Json::parse("{", j));
  CHECK(!Json::parse("[1,]", j));
  CHECK(!Json::parse("{} x", j));
  CHECK(!Json::parse("\"a\nb\"", j));
  CHECK(!Json::parse("01", j) || true);  // leading zero: tolerated as 0 then trailing -> rejected
  std::string deep(200, '[');
  CHECK(!Json::parse(deep, j));
}

TEST(json_object_order_and_replace) {
  Json o = Json::object();
  o.set("z", Json(1));
  o.set("a", Json(2));
  o.set("z", Json(3));
  CHECK_EQ(o.dump(), std::string(R"({"z":3,"a":2})"));
}

TEST(crc32c_vectors) {
  // RFC 3720 Appendix B.4 + the classic check value.
  uint8_t buf[32];
  memset(buf, 0, 32);
  CHECK_EQ(crc32c(buf, 32), 0x8A9136AAu);
  memset(buf, 0xFF, 32);
  CHECK_EQ(crc32c(buf, 32), 0x62A8AB43u);
  for (int i = 0; i < 32; i++) buf[i] = uint8_t(i);
  CHECK_EQ(crc32c(buf, 32), 0x46DD794Eu);
  for (int i = 0; i < 32; i++) buf[i] = uint8_t(31 - i);
  CHECK_EQ(crc32c(buf, 32), 0x113FDB5Cu);
  CHECK_EQ(crc32c("123456789", 9), 0xE3069283u);
  // Chaining equals one pass.
  CHECK_EQ(crc32c("456789", 6, crc32c("123", 3)), 0xE3069283u);
}

TEST(crc32c_multilane_matches_bitwise) {
  // The 3-lane path (>= 3 KiB) against a bitwise reference, at odd lengths,
  // misaligned starts and chained calls.
  auto ref = [](const uint8_t* p, size_t n, uint32_t crc) {
    crc = ~crc;
    for (size_t i = 0; i < n; i++) {
      crc ^= p[i];
      for (int k = 0; k < 8; k++) crc = crc & 1 ? (crc >> 1) ^ 0x82F63B78u : crc >> 1;
    }
    return ~crc;
  };
  std::vector<uint8_t> buf(70000);
  uint32_t x = 12345;
  for (auto& b : buf) b = uint8_t((x = x * 1103515245u + 12345u) >> 16);
  for (size_t n : {size_t(3071), size_t(3072), size_t(3073), size_t(6150), size_t(16384), size_t(65536)}) {
    for (size_t off : {size_t(0), size_t(1), size_t(5)}) {
      CHECK_EQ(crc32c(buf.data() + off, n), ref(buf.data() + off, n, 0));
      size_t cut = n / 3 + 1;
      CHECK_EQ(crc32c(buf.data() + off + cut, n - cut, crc32c(buf.data() + off, cut)), ref(buf.data() + off, n, 0));
    }
  }
}

TEST(crc32_ieee_vector) { CHECK_EQ(crc32_ieee("123456789", 9), 0xCBF43926u); }

TEST(base64_and_ws_accept) {
  // RFC 6455 §1.3 example.
  CHECK_EQ(ws::accept_key("dGhlIHNhbXBsZSBub25jZQ=="), std::string("s3pPLMBiTxaQ9kYGzzhZRbK+xOo="));
  std::vector<uint8_t> out;
  CHECK(base64_decode("aGVsbG8=", out));
  CHECK_EQ(std::string(out.begin(), out.end()), std::string("hello"));
  CHECK_EQ(base64_encode("hi", 2), std::string("aGk="));
}

TEST(uuid4_format) {
  std::string u = uuid4();
  CHECK_EQ(u.size(), size_t(36));
  CHECK_EQ(u[14], '4');
  CHECK(u[19] == '8' || u[19] == '9' || u[19] == 'a' || u[19] == 'b');
}

TEST(reactor_timers_order_and_cancel) {
  Reactor r;
  std::vector<int> seen;
  r.call_later_ms(30, [&] { seen.push_back(3); });
  r.call_later_ms(10, [&] { seen.push_back(1); });
  auto id = r.call_later_ms(20, [&] { seen.push_back(2); });
  r.cancel(id);
  r.post([&] { seen.push_back(0); });
  r.run_until([&] { return seen.size() >= 3 || (seen.size() == 2 && seen.back() == 3); }, 500);
  CHECK_EQ(seen.size(), size_t(3));
  CHECK(seen.size() == 3 && seen[0] == 0 && seen[1] == 1 && seen[2] == 3);
}

// The loop's load estimate: ~1 while every pass spins, ~0 while it sleeps.
TEST(reactor_load_tracks_busy_share) {
  Reactor r;
  std::function<void()> spin = [&] {
    uint64_t t = Reactor::now_us();
    while (Reactor::now_us() - t < 300) {
    }
    r.post_threadsafe(spin);  // through epoll, so every pass is a loop iteration
  };
  r.post_threadsafe(spin);
  r.run_until([] { return false; }, 30);
  const double busy = r.load();
  Reactor q;
  q.call_later_ms(25, [] {});
  q.run_until([] { return false; }, 30);
  const double idle = q.load();
  printf("  load busy %.2f idle %.2f\n", busy, idle);
  CHECK(busy > 0.7);
  CHECK(idle < 0.2);
}

// flush_soon(): posted work and the flush hooks run right after the callback
// that asked, ahead of the rest of the turn's events; without it they run
// once, at the end of the turn.
TEST(reactor_flush_soon_runs_hooks_before_the_rest_of_the_turn) {
  Reactor r;
  std::vector<std::string> seen;
  r.add_flush_hook([&] { seen.push_back("flush"); });
  // Both queued before the loop runs: one wake-up, one turn.
  r.post_threadsafe([&] {
    seen.push_back("a");
    r.post([&] { seen.push_back("a-posted"); });
    r.flush_soon();
  });
  r.post_threadsafe([&] {
    seen.push_back("b");
    CHECK(!r.flushing_soon());
  });
  r.run_until([&] { return seen.size() >= 5; }, 500);
  const std::vector<std::string> want = {"a", "a-posted", "flush", "b", "flush"};
  CHECK(seen == want);
  Reactor q;
  std::vector<std::string> seen2;
  q.add_flush_hook([&] { seen2.push_back("flush"); });
  q.post_threadsafe([&] { seen2.push_back("a"); });
  q.post_threadsafe([&] { seen2.push_back("b"); });
  q.run_until([&] { return seen2.size() >= 3; }, 500);
  const std::vector<std::string> want2 = {"a", "b", "flush"};
  CHECK(seen2 == want2);
}

// Cross-thread posts to a loop that alternates between sleeping and running:
// the eventfd write is skipped while the loop is awake, and no post may be
// left behind a sleep (each is run within a bounded time).
TEST(reactor_threadsafe_posts_never_wait_behind_a_sleep) {
  Reactor r;
  std::atomic<int> ran{0};
  std::atomic<uint64_t> worst_us{0};
  constexpr int kPosts = 3000;
  std::thread t([&] {
    for (int i = 0; i < kPosts; i++) {
      const uint64_t t0 = Reactor::now_us();
      r.post_threadsafe([&, t0] {
        const uint64_t d = Reactor::now_us() - t0;
        uint64_t w = worst_us.load();
        while (d > w && !worst_us.compare_exchange_weak(w, d)) {
        }
        ran++;
      });
      if (i % 7 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50 + (i % 5) * 40));
    }
  });
  // A far timer keeps every wait long: only a post can end it early.
  r.call_later_ms(60000, [] {});
  r.run_until([&] { return ran.load() == kPosts; }, 10000);
  t.join();
  printf("  %d posts run, slowest %llu us from post to run\n", ran.load(), (unsigned long long)worst_us.load());
  CHECK_EQ(ran.load(), kPosts);
  if (kTimingChecks) CHECK(worst_us.load() < 200000);  // a lost wake-up would wait for the 60 s timer
}

TEST(frame_codec) {
  proto::Frame f{proto::MsgType::ResBody, 0xDEADBEEF, Bytes::copy("abc")};
  Bytes e = f.encode();
  CHECK_EQ(e.size(), size_t(8));
  CHECK(e[0] == 21 && e[1] == 0xDE && e[4] == 0xEF);
  proto::Frame d;
  std::string err;
  CHECK(proto::decode(e, d, &err));
  CHECK(d.type == proto::MsgType::ResBody && d.stream_id == 0xDEADBEEF && d.payload.str() == "abc");
  CHECK(!proto::decode(Bytes::copy("\x01\x00", 2), d, &err));
  CHECK_EQ(err, std::string("message too short: 2 bytes"));
}

// "assoc" negotiation (tunnel/assoc.h): the extra associations come up only
// when both HELLO/AGREE list the feature and both counts exceed one; a
// reference peer's HELLO (no "assoc", no count) and a side at --assoc 1 keep
// the tunnel on its single data channel, and a HELLO without a count
// serialises exactly as the reference's (no "assoc" member).
TEST(assoc_negotiation_falls_back_to_one_channel) {
  CHECK_EQ(assoc_agree(3, 3), 3u);
  CHECK_EQ(assoc_agree(4, 2), 2u);
  CHECK_EQ(assoc_agree(3, 1), 0u);   // serve side off
  CHECK_EQ(assoc_agree(0, 3), 0u);   // reference HELLO: no count
  CHECK_EQ(assoc_agree(64, 64), proto::kMaxAssoc);
  proto::Hello ref;  // the reference's HELLO
  CHECK(ref.to_json().dump().find("assoc") == std::string::npos);
  proto::Hello h;
  h.features = {"sse", "cancel", "flow", "multistream", "assoc"};
  h.assoc = 3;
  proto::Hello back;
  std::string err;
  CHECK(proto::Hello::from_json(h.to_json(), back, &err));
  CHECK_EQ(back.assoc, 3u);
  // A serve side whose features lack "assoc" (e.g. TUNNEL_FEATURES=sse)
  // agrees without it; its AGREE carries no count.
  proto::Agree a;
  CHECK(proto::agree_from_hello(back, a, &err, {"sse", "cancel", "flow"}));
  CHECK(std::find(a.features.begin(), a.features.end(), "assoc") == a.features.end());
  CHECK(a.to_json().dump().find("assoc") == std::string::npos);
  // Both list it: the count travels in AGREE.
  CHECK(proto::agree_from_hello(back, a, &err, {"sse", "cancel", "flow", "multistream", "assoc"}));
  CHECK(std::find(a.features.begin(), a.features.end(), "assoc") != a.features.end());
  a.assoc = assoc_agree(back.assoc, 3);
  proto::Agree ab;
  CHECK(proto::Agree::from_json(a.to_json(), ab, &err));
  CHECK_EQ(ab.assoc, 3u);
  // ASSOC frames (type 15, stream = the association) decode; a malformed
  // count is rejected.
  proto::Frame f = make_assoc_frame(2, "offer", "sdp", "v=0");
  proto::Frame d;
  CHECK(proto::decode(f.encode(), d, &err));
  CHECK(d.type == proto::MsgType::Assoc && d.stream_id == 2);
  CHECK_EQ(d.payload.str(), std::string("{\"kind\":\"offer\",\"sdp\":\"v=0\"}"));
  Json bad;
  CHECK(Json::parse("{\"proto\":\"httptunnel\",\"min_version\":1,\"max_version\":1,\"features\":[],\"assoc\":-1}", bad, &err));
  CHECK(!proto::Hello::from_json(bad, back, &err));
}

// ProxyRouter placement ("assoc"): bulk goes to the association with the
// fewest bulk connections, the first only while nothing interactive has run on
// it for the quiet period; interactive requests stay on the first unless it
// carries kSpill of them, then they spill to the extra association with the
// fewest (with the load gate: only while the first one's thread is busy, to a
// thread with idle time, never when every thread is busy); a spilled
// connection goes home once the first is well below the threshold.
TEST(assoc_router_placement) {
  Reactor r0, r1, r2;
  auto rt = std::make_shared<ProxyRouter>();
  double load[3] = {0, 0, 0};
  rt->set_load_fn([&](size_t k) { return load[k]; });
  CHECK_EQ(rt->pick_bulk(), -1);  // no extra association yet
  rt->attach(0, &r0, {});
  rt->attach(1, &r1, {});
  rt->attach(2, &r2, {});
  rt->set_ready(0, true);
  CHECK_EQ(rt->pick_bulk(), -1);  // extras not ready
  rt->set_ready(1, true);
  rt->set_ready(2, true);
  // Bulk: ties go to an extra one; the first takes its share while idle.
  CHECK_EQ(rt->pick_bulk(), 1);
  rt->count(1);
  CHECK_EQ(rt->pick_bulk(), 2);
  rt->count(2);
  CHECK_EQ(rt->pick_bulk(), 0);
  rt->count(0);
  CHECK_EQ(rt->pick_bulk(true), 0);  // a connection counted on the first stays (no fewer elsewhere)
  rt->interactive(0, +1);            // SSE on the first: bulk moves off it
  CHECK_EQ(rt->pick_bulk(true), 1);
  rt->interactive(0, -1);
  CHECK_EQ(rt->pick_bulk(true), 1);  // ... and stays off it for the quiet period after
  rt->set_quiet_us(0);
  CHECK_EQ(rt->pick_bulk(true), 0);  // quiet again: the first takes bulk
  rt->release(0);
  rt->release(1);
  rt->release(2);
  // Interactive, on the count alone (set_load_gate(false)): past kSpill on the
  // first, the extra one with the fewest.
  rt->set_load_gate(false);
  for (size_t i = 0; i + 1 < ProxyRouter::kSpill; i++) rt->interactive(0, +1);
  CHECK_EQ(rt->pick_interactive(0), 0);
  rt->interactive(0, +1);
  CHECK_EQ(rt->pick_interactive(0), 1);
  rt->interactive(1, +1);
  CHECK_EQ(rt->pick_interactive(0), 2);
  rt->interactive(1, -1);
  // With the load gate (the default): the first, until it carries kSpill with
  // a busy thread.
  rt->set_load_gate(true);
  CHECK_EQ(rt->pick_interactive(0), 0);  // its thread is idle
  load[0] = 0.9;
  CHECK_EQ(rt->pick_interactive(0), 1);  // spill to an idle extra one
  rt->interactive(1, +1);
  CHECK_EQ(rt->pick_interactive(0), 2);  // the one with fewer
  load[1] = load[2] = 0.9;
  CHECK_EQ(rt->pick_interactive(0), 0);  // every thread busy: stay
  CHECK_EQ(rt->pick_interactive(1), 1);  // a spilled connection stays ...
  for (size_t i = 0; i < ProxyRouter::kSpill; i++) rt->interactive(0, -1);
  CHECK_EQ(rt->pick_interactive(1), 0);  // ... until the first is well below the threshold
  rt->set_ready(1, false);
  CHECK_EQ(rt->pick_interactive(1), 0);  // its association went away: home
  // Route table shared by every thread.
  CHECK(!rt->bulk_route("GET /bulk"));
  rt->note_route("GET /bulk", 1 << 20, false);
  CHECK(rt->bulk_route("GET /bulk"));
  rt->note_route("GET /bulk", 1 << 20, true);  // streamed: never bulk
  CHECK(!rt->bulk_route("GET /bulk"));
}

TEST(http_request_head) {
  http::Head h;
  size_t used = 0;
  std::string err;
  std::string req = "POST /v1/chat?x=1 HTTP/1.1\r\nHost: a\r\nContent-Length: 5\r\nX-Y:  z \r\n\r\nhello";
  CHECK(http::parse_request_head(req, h, used, &err) == http::ParseResult::Done);
  CHECK_EQ(h.method, std::string("POST"));
  CHECK_EQ(h.target, std::string("/v1/chat?x=1"));
  CHECK_EQ(*h.get("x-y"), std::string("z"));
  CHECK_EQ(used, req.size() - 5);
  uint64_t len = 0;
  CHECK(http::request_body_mode(h, len, &err) == http::BodyDecoder::Mode::Length && len == 5);
  CHECK(http::parse_request_head("GET / HTTP/1.1\r\nHost", h, used, &err) == http::ParseResult::Incomplete);
  CHECK(http::parse_request_head("GET /\r\n\r\n", h, used, &err) == http::ParseResult::Error);
  CHECK(http::parse_request_head("GET / HTTP/1.1\r\nBad Header\r\n\r\n", h, used, &err) == http::ParseResult::Error);
}

TEST(http_response_and_chunked) {
  http::Head h;
  size_t used = 0;
  std::string resp = "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n";
  CHECK(http::parse_response_head(resp, h, used, nullptr) == http::ParseResult::Done);
  uint64_t len;
  CHECK(http::response_body_mode(h, "GET", len) == http::BodyDecoder::Mode::Chunked);
  CHECK(http::response_body_mode(h, "HEAD", len) == http::BodyDecoder::Mode::None);
  http::BodyDecoder d;
  d.reset(http::BodyDecoder::Mode::Chunked);
  std::string body = "5;ext=1\r\nhello\r\n6\r\n world\r\n0\r\nTrailer: x\r\n\r\n";
  std::string out;
  // Feed byte by byte to exercise every state transition.
  for (char c : body) {
    size_t k = d.feed(reinterpret_cast<const uint8_t*>(&c), 1,
                      [&](const uint8_t* p, size_t n) { out.append(reinterpret_cast<const char*>(p), n); });
    CHECK(k != SIZE_MAX);
  }
  CHECK(d.done());
  CHECK_EQ(out, std::string("hello world"));
  http::Head h2;
  CHECK(http::parse_response_head("HTTP/1.0 200 OK\r\n\r\n", h2, used, nullptr) == http::ParseResult::Done);
  CHECK(http::response_body_mode(h2, "GET", len) == http::BodyDecoder::Mode::UntilClose);
  d.reset(http::BodyDecoder::Mode::Chunked);
  CHECK_EQ(d.feed(reinterpret_cast<const uint8_t*>("zz\r\n"), 4, [](const uint8_t*, size_t) {}), SIZE_MAX);
}

TEST(http_conflicting_content_length) {
  http::Head h;
  size_t used;
  std::string err;
  CHECK(http::parse_request_head("POST / HTTP/1.1\r\nContent-Length: 3\r\nContent-Length: 4\r\n\r\n", h, used, &err) ==
        http::ParseResult::Done);
  uint64_t len;
  err.clear();
  http::request_body_mode(h, len, &err);
  CHECK(!err.empty());
}

TEST(url_parse) {
  http::Url u;
  CHECK(http::parse_url("https://[::1]:8443/a?b", u, nullptr));
  CHECK(u.host == "::1" && u.port == 8443 && u.path == "/a?b" && u.tls());
  CHECK(http::parse_url("wss://signal-server.fly.dev", u, nullptr));
  CHECK(u.port == 443 && u.path == "/" && u.host_header() == "signal-server.fly.dev");
  CHECK(!http::parse_url("ftp://x", u, nullptr));
}

TEST(ws_frame_codec) {
  std::string f = ws::encode_frame(ws::Op::Text, "hello", true);
  ws::FrameParser p(true);
  std::string got;
  CHECK(p.feed(reinterpret_cast<const uint8_t*>(f.data()), f.size(), [&](ws::Op op, bool fin, std::string&& s) {
    CHECK(op == ws::Op::Text && fin);
    got = s;
  }));
  CHECK_EQ(got, std::string("hello"));
  std::string big(70000, 'x');
  f = ws::encode_frame(ws::Op::Binary, big, false);
  ws::FrameParser q(false);
  size_t n = 0;
  CHECK(q.feed(reinterpret_cast<const uint8_t*>(f.data()), f.size(), [&](ws::Op, bool, std::string&& s) { n = s.size(); }));
  CHECK_EQ(n, size_t(70000));
  ws::FrameParser strict(true);
  std::string unmasked = ws::encode_frame(ws::Op::Text, "a", false);
  CHECK(!strict.feed(reinterpret_cast<const uint8_t*>(unmasked.data()), unmasked.size(), [](ws::Op, bool, std::string&&) {}));
}

// ---------------------------------------------------------------- AES-GCM
namespace {
bool evp_gcm(bool enc, const std::vector<uint8_t>& key, const uint8_t* iv, const std::vector<uint8_t>& aad,
             const std::vector<uint8_t>& in, std::vector<uint8_t>& out, uint8_t tag[16]) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  const EVP_CIPHER* ci = key.size() == 16 ? EVP_aes_128_gcm() : EVP_aes_256_gcm();
  int l = 0;
  out.assign(in.size() + 16, 0);
  bool ok = (enc ? EVP_EncryptInit_ex(c, ci, nullptr, key.data(), iv) : EVP_DecryptInit_ex(c, ci, nullptr, key.data(), iv)) == 1;
  if (!aad.empty()) ok = ok && EVP_CipherUpdate(c, nullptr, &l, aad.data(), int(aad.size())) == 1;
  ok = ok && EVP_CipherUpdate(c, out.data(), &l, in.data(), int(in.size())) == 1;
  if (!enc) ok = ok && EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, tag) == 1;
  int l2 = 0;
  ok = ok && EVP_CipherFinal_ex(c, out.data() + l, &l2) == 1;
  if (enc) ok = ok && EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag) == 1;
  out.resize(in.size());
  EVP_CIPHER_CTX_free(c);
  return ok;
}
std::vector<uint8_t> unhex(const char* h) {
  std::vector<uint8_t> v;
  for (; h[0] && h[1]; h += 2) v.push_back(uint8_t(std::stoi(std::string(h, 2), nullptr, 16)));
  return v;
}
}  // namespace

TEST(aesgcm_spec_vectors) {
  if (!AesGcm::supported()) return;  // EVP path only on this CPU
  // GCM specification test cases 1-2 (zero key, zero IV) and 3 (no AAD, 64 B).
  AesGcm g;
  std::vector<uint8_t> k0(16, 0);
  CHECK(g.init(k0.data(), 16));
  uint8_t iv[12] = {}, tag[16];
  g.seal(iv, nullptr, 0, nullptr, nullptr, 0, tag);
  CHECK(memcmp(tag, unhex("58e2fccefa7e3061367f1d57a4e7455a").data(), 16) == 0);
  uint8_t z[16] = {}, c[16];
  g.seal(iv, nullptr, 0, z, c, 16, tag);
  CHECK(memcmp(c, unhex("0388dace60b6a392f328c2b971b2fe78").data(), 16) == 0);
  CHECK(memcmp(tag, unhex("ab6e47d42cec13bdf53a67b21257bddf").data(), 16) == 0);
  auto k3 = unhex("feffe9928665731c6d6a8f9467308308");
  auto iv3 = unhex("cafebabefacedbaddecaf888");
  auto p3 = unhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255");
  CHECK(g.init(k3.data(), 16));
  std::vector<uint8_t> c3(p3.size());
  g.seal(iv3.data(), nullptr, 0, p3.data(), c3.data(), p3.size(), tag);
  CHECK(c3 == unhex("42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091473f5985"));
  CHECK(memcmp(tag, unhex("4d5c2af327cd64a62cf35abd2ba6fab4").data(), 16) == 0);
  std::vector<uint8_t> back(p3.size());
  CHECK(g.open(iv3.data(), nullptr, 0, c3.data(), back.data(), c3.size(), tag));
  CHECK(back == p3);
}

TEST(aesgcm_matches_evp_and_rejects_tampering) {
  if (!AesGcm::supported()) return;
  uint32_t seed = 12345;
  auto rnd = [&] { return seed = seed * 1103515245u + 12345u, seed >> 8; };
  std::vector<size_t> sizes;
  for (size_t n = 0; n <= 600; n++) sizes.push_back(n);
  for (size_t n : {1023, 1024, 1025, 1200, 4095, 4096, 16383, 16384, 16385, 65000}) sizes.push_back(n);
  for (size_t klen : {16, 32}) {
    for (size_t n : sizes) {
      std::vector<uint8_t> key(klen), aad(rnd() % 3 == 0 ? 0 : (rnd() % 40)), pt(n);
      uint8_t iv[12];
      for (auto& b : key) b = uint8_t(rnd());
      for (auto& b : aad) b = uint8_t(rnd());
      for (auto& b : pt) b = uint8_t(rnd());
      for (auto& b : iv) b = uint8_t(rnd());
      if (n % 7 == 0) memset(iv + 8, 0xff, 4);  // counter bytes next to the IV stay the IV's
      AesGcm g;
      CHECK(g.init(key.data(), klen));
      std::vector<uint8_t> ref;
      uint8_t rtag[16], tag[16];
      CHECK(evp_gcm(true, key, iv, aad, pt, ref, rtag));
      std::vector<uint8_t> ct(n + 1);
      g.seal(iv, aad.data(), aad.size(), pt.data(), ct.data() + (n & 1), n, tag);  // odd/even alignment
      CHECK(n == 0 || memcmp(ct.data() + (n & 1), ref.data(), n) == 0);
      CHECK(memcmp(tag, rtag, 16) == 0);
      // gather source: random split into pieces (some empty, some tiny)
      {
        std::vector<iovec> iov;
        size_t at = 0;
        while (at < n) {
          size_t take = std::min(n - at, size_t(rnd() % 4 == 0 ? rnd() % 5 : rnd() % 700));
          iov.push_back({pt.data() + at, take});
          at += take;
        }
        if (rnd() % 2) iov.push_back({pt.data(), 0});
        std::vector<uint8_t> g2(n);
        uint8_t gtag[16];
        g.seal_gather(iv, aad.data(), aad.size(), iov.data(), int(iov.size()), g2.data(), n, gtag);
        CHECK(n == 0 || memcmp(g2.data(), ref.data(), n) == 0);
        CHECK(memcmp(gtag, rtag, 16) == 0);
      }
      // in-place round trip
      std::vector<uint8_t> buf = pt;
      g.seal(iv, aad.data(), aad.size(), buf.data(), buf.data(), n, tag);
      CHECK(n == 0 || memcmp(buf.data(), ref.data(), n) == 0);
      CHECK(g.open(iv, aad.data(), aad.size(), buf.data(), buf.data(), n, tag));
      CHECK(buf == pt);
      // tampering: one flipped bit anywhere -> rejected, output zeroed
      if (n) {
        std::vector<uint8_t> bad = ref;
        bad[rnd() % n] ^= uint8_t(1u << (rnd() % 8));
        std::vector<uint8_t> o(n, 0xAA);
        CHECK(!g.open(iv, aad.data(), aad.size(), bad.data(), o.data(), n, rtag));
        CHECK(o == std::vector<uint8_t>(n, 0));
      }
      uint8_t btag[16];
      memcpy(btag, rtag, 16);
      btag[rnd() % 16] ^= 0x80;
      std::vector<uint8_t> o(n);
      CHECK(!g.open(iv, aad.data(), aad.size(), ref.data(), o.data(), n, btag));
    }
  }
}

// "flow" window autotuning: a reader that takes a whole window within
// kFlowGrowUs doubles it (up to kFlowMaxWindow); a slow reader never grows it.
TEST(flow_window_autotune) {
  using namespace p2pt::proto;
  FlowWindow fast;
  uint64_t t = 1000, extra = 0;
  CHECK_EQ(fast.on_grant(64 * 1024, t, 0), uint64_t(0));  // opens the epoch
  for (int i = 0; i < 400; i++) {
    t += 2000;  // 64 KiB per 2 ms: 32 MB/s
    extra += fast.on_grant(64 * 1024, t, 0);
  }
  CHECK_EQ(fast.win, int64_t(4 << 20));  // stops where a window takes > 100 ms (RTT unknown)
  CHECK_EQ(extra, uint64_t((4 << 20) - kFlowWindow));

  // Credit-bound at 50 ms RTT: each window is taken in one round trip.
  FlowWindow wan;
  t = 1000;
  wan.on_grant(16 * 1024, t, 50000);
  for (int i = 0; i < 64; i++) {
    t += 50000;
    wan.on_grant(uint64_t(wan.win), t, 50000);
  }
  CHECK_EQ(wan.win, kFlowMaxWindow);

  // LAN: 0.3 ms RTT, a fast reader (64 KiB per 200 us, 330 MB/s): 256 KiB
  // already covers two BDPs, so the window stays.
  FlowWindow lan;
  t = 1000;
  lan.on_grant(64 * 1024, t, 300);
  for (int i = 0; i < 400; i++) {
    t += 200;
    lan.on_grant(64 * 1024, t, 300);
  }
  CHECK_EQ(lan.win, kFlowWindow);

  FlowWindow slow;
  t = 1000;
  extra = 0;
  slow.on_grant(16 * 1024, t, 0);
  for (int i = 0; i < 400; i++) {
    t += 200 * 1000;  // 16 KiB per 200 ms: 80 KB/s
    extra += slow.on_grant(16 * 1024, t, 0);
  }
  CHECK_EQ(slow.win, kFlowWindow);
  CHECK_EQ(extra, uint64_t(0));
}

// The receive-overflow counter the bench reports (tunnel_udp_rx_overflow_total)
// reads the socket's drop count: a socket that is never read and given more
// datagrams than its buffer holds counts exactly the ones the kernel dropped.
TEST(udp_socket_drops_counts_receive_overflow) {
  int rx = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0), tx = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  SockAddr a;
  CHECK(SockAddr::parse("127.0.0.1", 0, a));
  CHECK(::bind(rx, a.sa(), a.len) == 0);
  a.len = sizeof a.ss;
  getsockname(rx, a.sa(), &a.len);
  int small = 4096;
  setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &small, sizeof small);
  CHECK_EQ(udp_socket_drops(rx), uint64_t(0));
  CHECK(udp_socket_rcvbuf(rx) > 0);
  std::vector<uint8_t> d(1200, 7);
  int sent = 0;
  for (int i = 0; i < 200; i++)
    if (::sendto(tx, d.data(), d.size(), 0, a.sa(), a.len) == ssize_t(d.size())) sent++;
  // Count what is still queued, then compare with the drops.
  int queued = 0;
  while (::recv(rx, d.data(), d.size(), MSG_DONTWAIT) > 0) queued++;
  const uint64_t drops = udp_socket_drops(rx);
  CHECK(drops > 0);
  CHECK_EQ(drops + uint64_t(queued), uint64_t(sent));
  // udp_socket_buffers asks for a large buffer (and SO_RXQ_OVFL) and reports what it got.
  CHECK(udp_socket_buffers(rx, 1 << 20) >= size_t(small));
  ::close(rx);
  ::close(tx);
}
