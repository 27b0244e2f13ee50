// Tunnel wire protocol: frame codec, HELLO/AGREE negotiation, header schemas.
//
// Wire-compatible with the reference (tunnel/src/protocol.rs):
//   frame   = [type:u8][stream_id:u32 big-endian][payload...]  (protocol.rs:147-154)
//   decode  = >=5 bytes, known type, zero-copy payload view      (protocol.rs:157-172)
//   types   = HELLO 1, AGREE 2, PING 3, PONG 4, REQ_HEADERS 10, REQ_BODY 11,
//             REQ_END 12, RES_HEADERS 20, RES_BODY 21, RES_END 22, ERROR 99
//                                                                (protocol.rs:86-100)
//   limits  = MAX_FRAME_SIZE 65536, MAX_BODY_CHUNK 65408         (protocol.rs:9-12)
//   hello   = {"proto":"httptunnel","min_version":1,"max_version":1,"features":["sse"]}
//   agree   = highest common version, feature intersection       (protocol.rs:41-81)
//
// Encoding is split into a 5-byte header plus a payload view so transports can
// scatter/gather the two pieces instead of concatenating (the reference copies
// every body chunk three times, serve.rs:269-276).
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <string>
#include <vector>

#include "core/buf.h"
#include "core/json.h"

namespace p2pt::proto {

constexpr uint32_t kProtocolVersion = 1;
constexpr const char* kProtocolName = "httptunnel";
constexpr size_t kMaxFrameSize = 64 * 1024;
constexpr size_t kMaxBodyChunk = kMaxFrameSize - 128;
constexpr size_t kHeaderLen = 5;

enum class MsgType : uint8_t {
  Hello = 1,
  Agree = 2,
  Ping = 3,
  Pong = 4,
  ReqHeaders = 10,
  ReqBody = 11,
  ReqEnd = 12,
  // Extension (only sent when both HELLOs list "cancel"): the proxy's client
  // went away; serve aborts the upstream request. Not in the reference.
  Cancel = 13,
  // Extension "flow" (only when both HELLOs list it): per-stream credit. The
  // payload is a u32 (big-endian) number of body bytes the receiver grants the
  // sender on this stream: RES_BODY when sent by the proxy, REQ_BODY when
  // sent by serve. Each side starts with kFlowWindow bytes per stream and
  // direction. Not in the reference (which has no flow control, Q11).
  Credit = 14,
  // Extension "assoc" (only when both HELLOs list it): signalling for the
  // extra associations (parallel PeerConnections) on the first data channel.
  // stream_id = the association's index (1..N-1); the payload is JSON
  // {"kind":"offer"|"answer"|"candidate"|"bye", "sdp"|"candidate": "..."}.
  // The reference's one data channel (rtc.rs:133) is the only path either
  // side of a reference peer ever uses; see tunnel/assoc.h.
  Assoc = 15,
  ResHeaders = 20,
  ResBody = 21,
  ResEnd = 22,
  Error = 99,
};

std::optional<MsgType> msg_type_from_u8(uint8_t v);
const char* msg_type_name(MsgType t);  // "Hello", "ReqHeaders", ... (Rust Debug names)

struct Frame {
  MsgType type;
  uint32_t stream_id;
  Bytes payload;
  // A received body frame that came as several transport fragments keeps the
  // rest of its payload here (zero-copy views, in order); empty otherwise.
  // Frames built for sending never use it.
  std::vector<Bytes> more = {};

  // [type][stream_id] header.
  void header(uint8_t out[kHeaderLen]) const;
  // Header + payload in one buffer (tests / small control frames).
  Bytes encode() const;
  size_t payload_size() const {
    size_t n = payload.size();
    for (auto& b : more) n += b.size();
    return n;
  }
  size_t wire_size() const { return kHeaderLen + payload_size(); }
  // payload + more as one contiguous view (a copy only when chained).
  Bytes flat_payload() const;
};

// Decode a received message. Errors mirror the reference text:
// "message too short: N bytes", "unknown message type: T".
bool decode(const Bytes& raw, Frame& out, std::string* err);
// A message that arrived as fragments (`raw` the first, `more` the rest):
// body frames keep the fragments as their payload chain, every other type is
// made contiguous (headers are JSON, parsed in one piece).
bool decode_chain(const Bytes& raw, std::vector<Bytes>& more, Frame& out, std::string* err);

// ---- handshake
struct Hello {
  std::string proto = kProtocolName;
  uint32_t min_version = 1;
  uint32_t max_version = kProtocolVersion;
  std::vector<std::string> features{"sse"};
  // "psk" extension (only with --secret; serialised only when set, so a
  // reference peer sees the reference's HELLO): nonce and proof of the secret.
  std::string psk_nonce, psk_mac;
  // "assoc" extension: how many associations (the first data channel's plus
  // parallel ones) the proxy would use; 0 = not offered (not serialised).
  uint32_t assoc = 0;
  Json to_json() const;
  static bool from_json(const Json& j, Hello& out, std::string* err);
};

struct Agree {
  uint32_t version = 1;
  std::vector<std::string> features;
  std::string psk_mac;  // "psk" extension: the serve side's proof
  uint32_t assoc = 0;   // "assoc" extension: associations agreed (min of both sides); 0 = none
  Json to_json() const;
  static bool from_json(const Json& j, Agree& out, std::string* err);
};

// Pre-shared-secret proof (extension "psk", the reference README's planned
// `--secret`): hex HMAC-SHA256(secret, "p2pt-psk|" role "|" nonce "|" binding),
// role "hello" (proxy) or "agree" (serve). `binding` names the secured channel
// (both DTLS certificate fingerprints, sorted), so a proof observed on one
// channel is useless on another and a man in the middle — who must terminate
// DTLS with its own certificate on each leg — cannot relay it.
std::string psk_mac(const std::string& secret, const char* role, const std::string& nonce,
                    const std::string& binding);

// Features this build understands. "sse" is the reference's only feature;
// "cancel" (client-disconnect propagation), "flow" (per-stream
// credit, Q11) and "multistream" (tunnel streams spread over independently
// delivered SCTP streams, MessageChannel::set_lanes) are only *acted on* when
// both peers list them, so reference peers are unaffected.
// Lanes: 64 (the most a peer accepts, DataChannel::kMaxLanes). A tunnel stream
// rides lane sid % kLanes, so two streams share a lane (and a loss on one
// holds the other) only when their ids differ by a multiple of it; with 16,
// an SSE stream opened 16 streams after a bulk download shared its lane, and
// on the emulated 50 ms / 2 % path that put bulk loss recovery in the token
// tail.
constexpr int kLanes = 64;
// "assoc": at most this many associations per tunnel (the first included).
constexpr uint32_t kMaxAssoc = 8;
const std::vector<std::string>& our_features();
// Negotiate from a peer HELLO (reference Agree::from_hello, protocol.rs:44-80).
bool agree_from_hello(const Hello& h, Agree& out, std::string* err,
                      const std::vector<std::string>& ours = our_features());

// ---- header metadata (protocol.rs:121-136). Header maps are single-valued:
// a later header of the same (lower-cased) name replaces an earlier one,
// matching the reference's HashMap<String,String>.
using HeaderMap = std::vector<std::pair<std::string, std::string>>;
void header_set(HeaderMap& h, std::string name_lower, std::string value);
const std::string* header_get(const HeaderMap& h, std::string_view name_lower);

struct RequestHeaders {
  uint32_t stream_id = 0;
  std::string method;
  std::string path;
  HeaderMap headers;
  Json to_json() const;
  static bool from_json(const Json& j, RequestHeaders& out, std::string* err);
};

struct ResponseHeaders {
  uint32_t stream_id = 0;
  uint16_t status = 200;
  HeaderMap headers;
  Json to_json() const;
  static bool from_json(const Json& j, ResponseHeaders& out, std::string* err);
};

// Frame constructors (reference protocol.rs:176-262).
Frame make_hello(const Hello& h);
Frame make_agree(const Agree& a);
Frame make_req_headers(const RequestHeaders& h);
Frame make_res_headers(const ResponseHeaders& h);
Frame make_body(MsgType t, uint32_t stream_id, Bytes data);
Frame make_empty(MsgType t, uint32_t stream_id);
Frame make_error(uint32_t stream_id, const std::string& msg);
Frame make_credit(uint32_t stream_id, uint32_t bytes);
// Bytes granted by a Credit frame (0 if malformed).
uint32_t credit_bytes(const Frame& f);

// "flow" extension: initial per-stream, per-direction body credit, and the
// backlog below which a receiver hands consumed bytes back as credit.
constexpr int64_t kFlowWindow = 256 * 1024;
// The initial per-stream window both peers assume (a 1 MiB window lost on
// the MI355X host's 64 x 1 MB echo at jumbo MTU, profiles/r04/flow_ab).
inline int64_t flow_window() { return kFlowWindow; }
constexpr size_t kFlowGrantMin = 16 * 1024;

// "flow" receive-window autotuning, done by the receiver alone (no wire
// change: credit is additive, so granting more than was consumed grows the
// sender's window). A fixed 256 KiB window caps one stream at 256 KiB per
// round trip (5 MB/s at 50 ms RTT) however fast the path and the reader. A
// credit-bound stream's reader takes a whole window in about one round trip,
// so a window taken within 2 RTT + 20 ms whose two bandwidth-delay products
// (at the rate it was taken) exceed it doubles (within kFlowGrowUs while the
// RTT is unknown), up to kFlowMaxWindow: a path-bound stream stops near two
// BDPs, a LAN stream (a window lasts many sub-ms round trips) stays put, and
// a slow reader (a window per several round trips) never grows it, which
// keeps the per-stream memory bound that the extension exists for.
constexpr int64_t kFlowMaxWindow = 8 * 1024 * 1024;
constexpr uint64_t kFlowGrowUs = 100 * 1000;
constexpr uint64_t kFlowGrowSlackUs = 20 * 1000;

struct FlowWindow {
  int64_t win = flow_window();
  uint64_t epoch_bytes = 0;  // granted since epoch_t0
  uint64_t epoch_t0 = 0;     // 0: no grant yet
  // `n` consumed bytes are about to be granted back at `now_us` on a path of
  // base RTT `rtt_us` (0: unknown): returns the extra credit to add to
  // that grant (the window's growth, usually 0).
  uint64_t on_grant(uint64_t n, uint64_t now_us, uint64_t rtt_us);
};

// Upstream URL rewrite (reference serve.rs:167-185, incl. quirk Q1: the prefix
// is stripped without a path-segment boundary check).
std::string build_upstream_url(const std::string& upstream_base, const std::string& advertise_prefix,
                               const std::string& request_path);

bool json_parse_bytes(const Bytes& b, Json& out, std::string* err);

}  // namespace p2pt::proto
