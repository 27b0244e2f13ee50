// Rendezvous (signal) server: rooms of at most two peers, relaying SDP
// offers/answers and ICE candidates as JSON over WebSocket.
//
// Protocol-identical to reference signal-server/src/index.ts:
//   join      -> joined{peerId, peers:[existing]} + peer-joined to existing  (:112-154)
//   offer/answer/candidate -> relayed verbatim to the other peer + peerId    (:156-193)
//   bye/close/error -> peer-left to the remaining peer; empty rooms deleted  (:56-78, :195-220)
//   errors: "invalid JSON", "already joined a room", "room name required",
//           "room '<r>' is full (max 2)", "must join a room first",
//           "unknown message type"
// Same console lines, prefixed "[signal]". Runs on the tunnel's reactor
// (C++; the reference's Node 20 build cannot run on this image's Node 12).
#pragma once

#include <map>
#include <memory>
#include <set>
#include <string>

#include "core/json.h"
#include "core/net.h"
#include "ws/ws.h"

namespace p2pt {

class SignalServer {
 public:
  explicit SignalServer(Reactor& r, size_t max_room_size = 2) : r_(r), max_room_(max_room_size) {}
  ~SignalServer();
  // host:port (port 0 = ephemeral). Returns false with *err on failure.
  bool listen(const std::string& hostport, std::string* err);
  uint16_t port() const;
  std::string local_addr() const;
  size_t room_count() const { return rooms_.size(); }
  size_t peer_count() const { return peers_.size(); }

 private:
  struct Client;
  struct Peer {
    std::string id;
    std::string room;
    std::weak_ptr<Client> client;
  };
  void on_accept(int fd);
  void on_message(const std::shared_ptr<Client>& c, const std::string& text);
  void remove_peer(const std::string& peer_id);
  void send(const std::shared_ptr<Client>& c, const Json& msg);
  Peer* other_peer(const std::string& peer_id, const std::string& room);

  Reactor& r_;
  size_t max_room_;
  std::unique_ptr<TcpListener> listener_;
  std::map<Client*, std::shared_ptr<Client>> clients_;
  std::map<std::string, std::vector<std::string>> rooms_;  // insertion-ordered peer ids
  std::map<std::string, Peer> peers_;
};

}  // namespace p2pt
