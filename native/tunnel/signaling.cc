#include "tunnel/signaling.h"

#include "core/log.h"

namespace p2pt {

static const char* kT = "tunnel::signaling";

const char* signal_kind_name(IncomingSignal::Kind k) {
  switch (k) {
    case IncomingSignal::Kind::Joined: return "Joined";
    case IncomingSignal::Kind::PeerJoined: return "PeerJoined";
    case IncomingSignal::Kind::Offer: return "Offer";
    case IncomingSignal::Kind::Answer: return "Answer";
    case IncomingSignal::Kind::Candidate: return "Candidate";
    case IncomingSignal::Kind::PeerLeft: return "PeerLeft";
    case IncomingSignal::Kind::Error: return "Error";
  }
  return "?";
}

bool parse_incoming_signal(const std::string& text, IncomingSignal& out, std::string* err) {
  Json j;
  if (!Json::parse(text, j, err)) return false;
  const Json* t = j.get("type");
  if (!t || !t->is_string()) {
    if (err) *err = "missing field `type`";
    return false;
  }
  auto str = [&](const char* k, std::string& dst) -> bool {
    const Json* v = j.get(k);
    if (!v || !v->is_string()) {
      if (err) *err = std::string("missing field `") + k + "`";
      return false;
    }
    dst = v->as_string();
    return true;
  };
  const std::string& type = t->as_string();
  out = IncomingSignal{};
  if (type == "joined") {
    out.kind = IncomingSignal::Kind::Joined;
    if (!str("peerId", out.peer_id)) return false;
    const Json* p = j.get("peers");
    if (!p || !p->is_array()) {
      if (err) *err = "missing field `peers`";
      return false;
    }
    for (auto& e : p->as_array()) {
      if (!e.is_string()) {
        if (err) *err = "invalid peers entry";
        return false;
      }
      out.peers.push_back(e.as_string());
    }
    return true;
  }
  if (type == "peer-joined") {
    out.kind = IncomingSignal::Kind::PeerJoined;
    return str("peerId", out.peer_id);
  }
  if (type == "offer" || type == "answer") {
    out.kind = type == "offer" ? IncomingSignal::Kind::Offer : IncomingSignal::Kind::Answer;
    return str("peerId", out.peer_id) && str("sdp", out.sdp);
  }
  if (type == "candidate") {
    out.kind = IncomingSignal::Kind::Candidate;
    return str("peerId", out.peer_id) && str("candidate", out.candidate);
  }
  if (type == "peer-left") {
    out.kind = IncomingSignal::Kind::PeerLeft;
    return str("peerId", out.peer_id);
  }
  if (type == "error") {
    out.kind = IncomingSignal::Kind::Error;
    return str("message", out.message);
  }
  if (err) *err = "unknown variant `" + type + "`";
  return false;
}

void SignalingClient::connect(Reactor& r, const std::string& url, const std::string& room, ConnectCb cb) {
  LOG_INFO(kT, "connecting to signaling server: %s", url.c_str());
  ws::WsConn::connect(r, url, [cb, room](std::shared_ptr<ws::WsConn> ws, std::string err) {
    if (!ws) {
      cb(nullptr, "failed to connect to signaling server: " + err);
      return;
    }
    auto sc = std::shared_ptr<SignalingClient>(new SignalingClient());
    sc->ws_ = ws;
    std::weak_ptr<SignalingClient> w = sc;
    ws->on_text = [w](std::string&& text) {
      auto s = w.lock();
      if (!s) return;
      IncomingSignal sig;
      std::string perr;
      if (!parse_incoming_signal(text, sig, &perr)) {
        LOG_WARN(kT, "failed to parse signal message: %s - %s", perr.c_str(), text.c_str());
        return;
      }
      LOG_DEBUG(kT, "received signal: %s", signal_kind_name(sig.kind));
      if (s->on_signal) s->on_signal(sig);
    };
    ws->on_closed = [w](const std::string& e) {
      auto s = w.lock();
      if (!s) return;
      if (e.empty()) LOG_INFO(kT, "signaling connection closed");
      else LOG_ERROR(kT, "signaling ws error: %s", e.c_str());
      auto cbc = std::move(s->on_closed);
      s->on_closed = nullptr;
      if (cbc) cbc(e);
    };
    Json join = Json::object();
    join.set("type", Json("join"));
    join.set("room", Json(room));
    sc->send_json(join);
    LOG_INFO(kT, "sent join for room: %s", room.c_str());
    cb(sc, "");
  });
}

SignalingClient::~SignalingClient() {
  if (ws_) {
    send_bye();
    ws_->on_closed = nullptr;
    ws_->on_text = nullptr;
    ws_->close(1000, "");
  }
}

void SignalingClient::send_json(const Json& j) {
  if (ws_ && ws_->is_open()) ws_->send_text(j.dump());
}

void SignalingClient::send_offer(const std::string& sdp) {
  Json j = Json::object();
  j.set("type", Json("offer"));
  j.set("sdp", Json(sdp));
  send_json(j);
}

void SignalingClient::send_answer(const std::string& sdp) {
  Json j = Json::object();
  j.set("type", Json("answer"));
  j.set("sdp", Json(sdp));
  send_json(j);
}

void SignalingClient::send_candidate(const std::string& c) {
  Json j = Json::object();
  j.set("type", Json("candidate"));
  j.set("candidate", Json(c));
  send_json(j);
}

void SignalingClient::send_bye() {
  if (bye_sent_) return;
  bye_sent_ = true;
  Json j = Json::object();
  j.set("type", Json("bye"));
  send_json(j);
}

}  // namespace p2pt
