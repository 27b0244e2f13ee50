// Session descriptions for a data-only WebRTC session (JSEP, RFC 8829;
// SDP for SCTP-over-DTLS, RFC 8841).
//
// Emits the shape webrtc-rs / browsers produce and accept for a
// datachannel-only PeerConnection: one BUNDLEd `m=application 9
// UDP/DTLS/SCTP webrtc-datachannel` section with ice-ufrag/pwd, a SHA-256
// fingerprint, a=setup (actpass in offers, active in answers), a=mid,
// a=sctp-port and a=max-message-size, plus inline candidates. The parser
// also accepts the legacy `DTLS/SCTP <port>` + a=sctpmap form.
#pragma once

#include <string>
#include <vector>

#include "rtc/ice.h"

namespace p2pt::rtc {

struct SessionDesc {
  std::string type;  // "offer" | "answer"
  std::string ice_ufrag, ice_pwd;
  std::string fingerprint;  // "sha-256 AB:CD:..."
  std::string setup = "actpass";
  std::string mid = "0";
  uint16_t sctp_port = 5000;
  size_t max_message_size = 262144;
  std::vector<Candidate> candidates;
  bool end_of_candidates = false;
  // Extension understood only by this implementation: largest SCTP packet
  // the peer accepts on same-host paths (0 = not advertised).
  size_t jumbo = 0;

  std::string to_string() const;
  static bool parse(const std::string& sdp, SessionDesc& out, std::string* err);
};

}  // namespace p2pt::rtc
