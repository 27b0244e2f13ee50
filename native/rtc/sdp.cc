#include "rtc/sdp.h"

#include <sstream>

#include "core/crypto.h"

namespace p2pt::rtc {

std::string SessionDesc::to_string() const {
  std::ostringstream o;
  uint64_t sid = random_u64() & 0x7fffffffffffffffull;
  o << "v=0\r\n"
    << "o=- " << sid << " 2 IN IP4 0.0.0.0\r\n"
    << "s=-\r\n"
    << "t=0 0\r\n"
    << "a=fingerprint:" << fingerprint << "\r\n"
    << "a=group:BUNDLE " << mid << "\r\n"
    << "m=application 9 UDP/DTLS/SCTP webrtc-datachannel\r\n"
    << "c=IN IP4 0.0.0.0\r\n"
    << "a=setup:" << setup << "\r\n"
    << "a=mid:" << mid << "\r\n"
    << "a=sendrecv\r\n"
    << "a=sctp-port:" << sctp_port << "\r\n"
    << "a=max-message-size:" << max_message_size << "\r\n"
    << "a=ice-ufrag:" << ice_ufrag << "\r\n"
    << "a=ice-pwd:" << ice_pwd << "\r\n"
    << "a=ice-options:trickle\r\n";
  if (jumbo) o << "a=x-p2pt-jumbo:" << jumbo << "\r\n";
  for (auto& c : candidates) o << "a=" << c.to_sdp() << "\r\n";
  if (end_of_candidates) o << "a=end-of-candidates\r\n";
  return o.str();
}

bool SessionDesc::parse(const std::string& sdp, SessionDesc& out, std::string* err) {
  out = SessionDesc{};
  out.setup.clear();
  std::istringstream in(sdp);
  std::string line;
  bool have_app = false;
  bool in_app = false;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.size() < 2 || line[1] != '=') continue;
    char k = line[0];
    std::string v = line.substr(2);
    if (k == 'm') {
      in_app = v.rfind("application", 0) == 0;
      if (in_app) {
        have_app = true;
        // Legacy: "application 9 DTLS/SCTP 5000"
        std::istringstream ms(v);
        std::string media, port, proto, fmt;
        ms >> media >> port >> proto >> fmt;
        if (proto == "DTLS/SCTP" && !fmt.empty()) out.sctp_port = uint16_t(atoi(fmt.c_str()));
      }
      continue;
    }
    if (k != 'a') continue;
    size_t colon = v.find(':');
    std::string name = v.substr(0, colon);
    std::string val = colon == std::string::npos ? "" : v.substr(colon + 1);
    // Session-level attributes apply unless overridden inside the m-section.
    if (name == "ice-ufrag") out.ice_ufrag = val;
    else if (name == "ice-pwd") out.ice_pwd = val;
    else if (name == "fingerprint") {
      std::string algo = val.substr(0, val.find(' '));
      for (auto& c : algo) c = char(tolower(c));
      if (algo == "sha-256") out.fingerprint = "sha-256 " + val.substr(val.find(' ') + 1);
    } else if (name == "setup") out.setup = val;
    else if (name == "mid" && in_app) out.mid = val;
    else if (name == "sctp-port") out.sctp_port = uint16_t(atoi(val.c_str()));
    else if (name == "sctpmap") out.sctp_port = uint16_t(atoi(val.c_str()));
    else if (name == "max-message-size") out.max_message_size = size_t(strtoull(val.c_str(), nullptr, 10));
    else if (name == "x-p2pt-jumbo") out.jumbo = size_t(strtoull(val.c_str(), nullptr, 10));
    else if (name == "end-of-candidates") out.end_of_candidates = true;
    else if (name == "candidate" && in_app) {
      Candidate c;
      if (Candidate::parse(v, c, nullptr)) out.candidates.push_back(c);
    }
  }
  if (!have_app) {
    if (err) *err = "SDP has no application (data channel) section";
    return false;
  }
  if (out.ice_ufrag.empty() || out.ice_pwd.empty()) {
    if (err) *err = "SDP lacks ice-ufrag/ice-pwd";
    return false;
  }
  if (out.fingerprint.empty()) {
    if (err) *err = "SDP lacks a sha-256 fingerprint";
    return false;
  }
  if (out.setup.empty()) out.setup = "actpass";
  return true;
}

}  // namespace p2pt::rtc
