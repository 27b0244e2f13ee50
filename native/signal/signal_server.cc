#include "signal/signal_server.h"

#include <cstdio>

#include "core/crypto.h"

namespace p2pt {

struct SignalServer::Client {
  std::shared_ptr<TcpConn> tcp;  // before upgrade
  std::string buf;
  std::shared_ptr<ws::WsConn> ws;
  std::string peer_id;  // empty = not joined
};

static void slog(const std::string& s) {
  printf("[signal] %s\n", s.c_str());
  fflush(stdout);
}

SignalServer::~SignalServer() {
  auto cs = std::move(clients_);
  for (auto& kv : cs) {
    if (kv.second->ws) kv.second->ws->on_closed = nullptr;
    if (kv.second->tcp) {
      kv.second->tcp->on_close(nullptr);
      kv.second->tcp->close();
    }
  }
}

bool SignalServer::listen(const std::string& hostport, std::string* err) {
  slog("starting signal server...");
  listener_ = TcpListener::bind(r_, hostport, [this](int fd, SockAddr) { on_accept(fd); }, err);
  if (!listener_) return false;
  SockAddr a = listener_->local_addr();
  slog("listening on ws://" + a.str());
  return true;
}

uint16_t SignalServer::port() const { return listener_ ? listener_->local_addr().port() : 0; }
std::string SignalServer::local_addr() const { return listener_ ? listener_->local_addr().str() : ""; }

void SignalServer::on_accept(int fd) {
  auto c = std::make_shared<Client>();
  c->tcp = TcpConn::adopt(r_, fd);
  clients_[c.get()] = c;
  std::weak_ptr<Client> w = c;
  c->tcp->on_data([this, w](const uint8_t* p, size_t n) {
    auto cl = w.lock();
    if (!cl || cl->ws) return;
    cl->buf.append(reinterpret_cast<const char*>(p), n);
    http::Head h;
    size_t used = 0;
    auto res = http::parse_request_head(cl->buf, h, used, nullptr);
    if (res == http::ParseResult::Incomplete) return;
    if (res == http::ParseResult::Error || !h.has_token("upgrade", "websocket")) {
      std::string body = "Upgrade Required";
      cl->tcp->write("HTTP/1.1 426 Upgrade Required\r\nContent-Type: text/plain\r\nContent-Length: " +
                     std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body);
      cl->tcp->close_after_flush();
      return;
    }
    std::string rest = cl->buf.substr(used);
    cl->buf.clear();
    auto tcp = cl->tcp;
    cl->ws = ws::WsConn::accept(r_, tcp, h, std::move(rest));
    cl->tcp.reset();
    if (!cl->ws) {
      clients_.erase(cl.get());
      return;
    }
    cl->ws->on_text = [this, w](std::string&& t) {
      if (auto c2 = w.lock()) on_message(c2, t);
    };
    cl->ws->on_binary = [this, w](std::string&& t) {
      if (auto c2 = w.lock()) on_message(c2, t);
    };
    cl->ws->on_closed = [this, w](const std::string& err) {
      auto c2 = w.lock();
      if (!c2) return;
      if (!err.empty()) fprintf(stderr, "[signal] ws error: %s\n", err.c_str());
      slog("ws closed for peer " + (c2->peer_id.empty() ? std::string("null") : c2->peer_id));
      if (!c2->peer_id.empty()) remove_peer(c2->peer_id);
      c2->peer_id.clear();
      r_.post([this, c2] { clients_.erase(c2.get()); });
    };
  });
  c->tcp->on_close([this, w](const std::string&) {
    auto cl = w.lock();
    if (cl && !cl->ws) clients_.erase(cl.get());
  });
}

void SignalServer::send(const std::shared_ptr<Client>& c, const Json& msg) {
  if (c && c->ws && c->ws->is_open()) c->ws->send_text(msg.dump());
}

static Json err_msg(const std::string& m) {
  Json j = Json::object();
  j.set("type", Json("error"));
  j.set("message", Json(m));
  return j;
}

SignalServer::Peer* SignalServer::other_peer(const std::string& peer_id, const std::string& room) {
  auto it = rooms_.find(room);
  if (it == rooms_.end()) return nullptr;
  for (auto& id : it->second)
    if (id != peer_id) {
      auto p = peers_.find(id);
      return p == peers_.end() ? nullptr : &p->second;
    }
  return nullptr;
}

void SignalServer::remove_peer(const std::string& peer_id) {
  auto pit = peers_.find(peer_id);
  if (pit == peers_.end()) return;
  std::string room = pit->second.room;
  auto rit = rooms_.find(room);
  if (rit != rooms_.end()) {
    auto& v = rit->second;
    for (size_t i = 0; i < v.size(); i++)
      if (v[i] == peer_id) {
        v.erase(v.begin() + long(i));
        break;
      }
    if (v.empty()) {
      rooms_.erase(rit);
    } else {
      Json m = Json::object();
      m.set("type", Json("peer-left"));
      m.set("peerId", Json(peer_id));
      for (auto& id : v) {
        auto o = peers_.find(id);
        if (o != peers_.end()) send(o->second.client.lock(), m);
      }
    }
  }
  peers_.erase(peer_id);
  slog("peer " + peer_id + " left room " + room);
}

void SignalServer::on_message(const std::shared_ptr<Client>& c, const std::string& text) {
  Json msg;
  if (!Json::parse(text, msg)) {
    send(c, err_msg("invalid JSON"));
    return;
  }
  const Json* tj = msg.get("type");
  std::string type = tj && tj->is_string() ? tj->as_string() : "";
  if (type == "join") {
    if (!c->peer_id.empty()) {
      send(c, err_msg("already joined a room"));
      return;
    }
    const Json* rj = msg.get("room");
    if (!rj || !rj->is_string() || rj->as_string().empty()) {
      send(c, err_msg("room name required"));
      return;
    }
    std::string room = rj->as_string();
    auto rit = rooms_.find(room);
    if (rit != rooms_.end() && rit->second.size() >= max_room_) {
      send(c, err_msg("room '" + room + "' is full (max " + std::to_string(max_room_) + ")"));
      return;
    }
    std::string id = uuid4();
    c->peer_id = id;
    peers_[id] = Peer{id, room, c};
    auto& members = rooms_[room];
    std::vector<std::string> existing = members;
    members.push_back(id);
    slog("peer " + id + " joined room '" + room + "' (" + std::to_string(members.size()) + "/" +
         std::to_string(max_room_) + ")");
    Json joined = Json::object();
    joined.set("type", Json("joined"));
    joined.set("peerId", Json(id));
    Json arr = Json::array();
    for (auto& e : existing) arr.push(Json(e));
    joined.set("peers", arr);
    send(c, joined);
    Json pj = Json::object();
    pj.set("type", Json("peer-joined"));
    pj.set("peerId", Json(id));
    for (auto& e : existing) {
      auto o = peers_.find(e);
      if (o != peers_.end()) send(o->second.client.lock(), pj);
    }
    return;
  }
  if (type == "offer" || type == "answer" || type == "candidate") {
    if (c->peer_id.empty()) {
      send(c, err_msg("must join a room first"));
      return;
    }
    auto me = peers_.find(c->peer_id);
    if (me == peers_.end()) return;
    Peer* other = other_peer(c->peer_id, me->second.room);
    if (!other) return;
    Json out = Json::object();
    out.set("type", Json(type));
    out.set("peerId", Json(c->peer_id));
    const char* field = type == "candidate" ? "candidate" : "sdp";
    if (const Json* v = msg.get(field)) out.set(field, *v);  // JSON.stringify drops undefined
    send(other->client.lock(), out);
    return;
  }
  if (type == "bye") {
    if (!c->peer_id.empty()) {
      remove_peer(c->peer_id);
      c->peer_id.clear();
    }
    return;
  }
  send(c, err_msg("unknown message type"));
}

}  // namespace p2pt
