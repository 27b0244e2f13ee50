// Signalling client: joins a room on the signal server and exchanges SDP and
// ICE candidates with the other peer.
//
// Mirrors reference tunnel/src/signaling.rs:
//   - connect, then immediately {"type":"join","room":R}          (:80-99)
//   - outgoing offer/answer/candidate/bye JSON                      (:9-23)
//   - incoming kebab-case tags with "peerId"; unparseable messages
//     are logged and skipped                                        (:27-65, :120-148)
//   - {"type":"bye"} on drop                                        (:72-77)
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/json.h"
#include "ws/ws.h"

namespace p2pt {

struct IncomingSignal {
  enum class Kind { Joined, PeerJoined, Offer, Answer, Candidate, PeerLeft, Error } kind;
  std::string peer_id;
  std::vector<std::string> peers;
  std::string sdp;
  std::string candidate;
  std::string message;
};

// Returns false when the JSON is not a valid incoming signal.
bool parse_incoming_signal(const std::string& text, IncomingSignal& out, std::string* err);
const char* signal_kind_name(IncomingSignal::Kind k);

class SignalingClient : public std::enable_shared_from_this<SignalingClient> {
 public:
  using ConnectCb = std::function<void(std::shared_ptr<SignalingClient>, std::string err)>;
  static void connect(Reactor& r, const std::string& url, const std::string& room, ConnectCb cb);
  ~SignalingClient();

  void send_offer(const std::string& sdp);
  void send_answer(const std::string& sdp);
  void send_candidate(const std::string& candidate_json);
  void send_bye();

  // Messages in arrival order. The consumer swaps these as its FSM advances.
  std::function<void(const IncomingSignal&)> on_signal;
  // Connection lost (EOF or error); fired once.
  std::function<void(const std::string&)> on_closed;

 private:
  void send_json(const Json& j);
  std::shared_ptr<ws::WsConn> ws_;
  bool bye_sent_ = false;
};

}  // namespace p2pt
