#include "tunnel/assoc.h"

#include <algorithm>

#include "core/json.h"
#include "core/log.h"
#include "rtc/peer.h"
#include "tunnel/metrics.h"

namespace p2pt {

static const char* kT = "tunnel::assoc";

uint32_t assoc_agree(uint32_t proxy_count, uint32_t serve_count) {
  const uint32_t n = std::min({proxy_count, serve_count, proto::kMaxAssoc});
  return n > 1 ? n : 0;
}

proto::Frame make_assoc_frame(uint32_t index, const std::string& kind, const std::string& key,
                              const std::string& value) {
  Json j = Json::object();
  j.set("kind", Json(kind));
  if (!key.empty()) j.set(key, Json(value));
  std::string s = j.dump();
  return proto::Frame{proto::MsgType::Assoc, index, Bytes::copy(s)};
}

// One extra association: its PeerConnection, data channel and session, all on
// the link's own reactor thread. The offer / answer / candidates go through
// the group (primary thread) onto the first data channel, the way the
// rendezvous's go through the signal server (tunnel/session.cc).
class AssocLink : public std::enable_shared_from_this<AssocLink> {
 public:
  AssocLink(Reactor& r, Reactor& primary, std::weak_ptr<AssocGroup> g, size_t index, bool offerer,
            const rtc::PcConfig& pc, AssocGroup::SessionFactory f)
      : r_(r), primary_(primary), group_(std::move(g)), k_(index), offerer_(offerer), pcfg_(pc),
        factory_(std::move(f)) {}

  // The offering side creates its connection at once; the answering side only
  // when an offer arrives (a proxy that decides against the extra
  // associations — a long path — then costs no sockets or TURN allocations).
  void start() {
    if (offerer_) create_pc();
  }

  void create_pc() {
    pc_ = rtc::PeerConnection::create(r_, pcfg_, offerer_);
    std::weak_ptr<AssocLink> w = shared_from_this();
    pc_->on_ice_candidate = [w](const std::string& cand) {
      if (auto s = w.lock()) s->to_group("candidate", "candidate", cand);
    };
    pc_->on_state = [w](rtc::PcState st) {
      auto s = w.lock();
      if (s && st == rtc::PcState::Failed) s->down("ICE connection failed");
    };
    if (offerer_) {
      dc_ = pc_->create_data_channel("tunnel");
      watch_channel();
      pc_->on_gathering_complete = [w] {
        if (auto s = w.lock()) s->send_sdp();
      };
      pc_->start_gathering();
      arm_gather_timeout();
    } else {
      pc_->on_data_channel = [w](std::shared_ptr<rtc::DataChannel> dc) {
        auto s = w.lock();
        if (!s || s->dc_) return;
        s->dc_ = dc;
        s->watch_channel();
      };
      pc_->start_gathering();
    }
  }

  void on_signal(const std::string& kind, const std::string& value) {
    if (closed_) return;
    if (kind == "offer" && !offerer_ && !remote_set_) {
      if (!pc_) create_pc();
      apply_remote(value);
      if (closed_) return;
      if (pc_->gathering_complete()) {
        send_sdp();
      } else {
        std::weak_ptr<AssocLink> w = shared_from_this();
        pc_->on_gathering_complete = [w] {
          if (auto s = w.lock()) s->send_sdp();
        };
        arm_gather_timeout();
      }
    } else if (kind == "answer" && offerer_ && !remote_set_) {
      apply_remote(value);
    } else if (kind == "candidate") {
      if (remote_set_) add_candidate(value);
      else buffered_.push_back(value);
    } else if (kind == "bye") {
      down("peer closed the association");
    }
  }

  // Drops the session, then the connection (link thread; the group is going).
  void shutdown() {
    closed_ = true;
    if (gather_timer_) r_.cancel(gather_timer_);
    gather_timer_ = 0;
    session_.reset();
    if (dc_) {
      dc_->on_open = nullptr;
      dc_->on_closed = nullptr;
    }
    if (pc_) {
      pc_->on_state = nullptr;
      pc_->on_ice_candidate = nullptr;
      pc_->on_gathering_complete = nullptr;
      pc_->on_data_channel = nullptr;
      pc_->close();
    }
    dc_.reset();
    pc_.reset();
  }

 private:
  void to_group(const char* kind, const char* key, const std::string& value) {
    std::weak_ptr<AssocGroup> g = group_;
    const size_t k = k_;
    primary_.post_threadsafe([g, k, kind = std::string(kind), key = std::string(key), value] {
      if (auto gg = g.lock()) gg->send_signal(k, kind, key, value);
    });
  }
  void state(bool up, const std::string& why) {
    std::weak_ptr<AssocGroup> g = group_;
    const size_t k = k_;
    primary_.post_threadsafe([g, k, up, why] {
      if (auto gg = g.lock()) gg->link_state(k, up, why);
    });
  }
  // The link is gone (its connection failed, its session ended, the peer
  // said bye): reported once; the teardown runs after the current callback,
  // which may be the connection's own.
  void down(const std::string& why) {
    if (closed_ || down_) return;
    down_ = true;
    LOG_WARN(kT, "association %zu down: %s", k_, why.c_str());
    state(false, why);
    std::weak_ptr<AssocLink> w = shared_from_this();
    r_.post([w] {
      if (auto s = w.lock()) s->shutdown();
    });
  }

  void arm_gather_timeout() {
    std::weak_ptr<AssocLink> w = shared_from_this();
    gather_timer_ = r_.call_later_ms(gather_timeout_ms(), [w] {
      if (auto s = w.lock()) {
        s->gather_timer_ = 0;
        s->send_sdp();
      }
    });
  }
  uint64_t gather_timeout_ms() const { return 5000; }  // as the rendezvous (rtc.rs:181-182)

  void send_sdp() {
    if (sdp_sent_ || closed_ || !pc_) return;
    if (!offerer_ && !remote_set_) return;
    sdp_sent_ = true;
    if (gather_timer_) r_.cancel(gather_timer_);
    gather_timer_ = 0;
    to_group(offerer_ ? "offer" : "answer", "sdp", pc_->local_description());
  }

  void apply_remote(const std::string& sdp) {
    std::string err;
    if (!pc_->set_remote_description(sdp, &err)) {
      down("invalid remote description: " + err);
      return;
    }
    remote_set_ = true;
    for (auto& c : buffered_) add_candidate(c);
    buffered_.clear();
  }

  void add_candidate(const std::string& c) {
    std::string err;
    if (!pc_->add_ice_candidate(c, &err)) LOG_WARN(kT, "association %zu: skipping bad ICE candidate: %s", k_, err.c_str());
  }

  void watch_channel() {
    std::weak_ptr<AssocLink> w = shared_from_this();
    auto opened = [w] {
      auto s = w.lock();
      if (!s || s->closed_ || s->session_) return;
      LOG_INFO(kT, "association %zu established via %s", s->k_, s->pc_->describe_path().c_str());
      auto done = [w](const std::string& why) {
        auto s2 = w.lock();
        if (!s2) return;
        s2->down(why);
      };
      s->session_ = s->factory_(s->r_, s->dc_, s->k_, done);
      s->state(true, "");
      if (const uint64_t ms = rtc::fault_assoc_down_ms()) {  // TUNNEL_FAULT fail-over tests
        s->r_.call_later_ms(ms, [w] {
          if (auto s2 = w.lock()) s2->down("fault injection (TUNNEL_FAULT assoc_down_ms)");
        });
      }
    };
    if (dc_->is_open()) opened();
    else dc_->on_open = opened;
  }

  Reactor& r_;
  Reactor& primary_;
  std::weak_ptr<AssocGroup> group_;
  size_t k_;
  bool offerer_;
  rtc::PcConfig pcfg_;
  AssocGroup::SessionFactory factory_;
  std::shared_ptr<rtc::PeerConnection> pc_;
  std::shared_ptr<rtc::DataChannel> dc_;
  std::shared_ptr<void> session_;
  std::vector<std::string> buffered_;
  bool remote_set_ = false;
  bool sdp_sent_ = false;
  bool closed_ = false;
  bool down_ = false;
  uint64_t gather_timer_ = 0;
};

std::shared_ptr<AssocGroup> AssocGroup::create(Reactor& primary, bool offerer, uint32_t count, const rtc::PcConfig& pc,
                                               uint64_t busy_poll_us, SessionFactory factory, SendFn send,
                                               StateFn state) {
  auto g = std::shared_ptr<AssocGroup>(
      new AssocGroup(primary, offerer, count, pc, busy_poll_us, std::move(factory), std::move(send), std::move(state)));
  g->start();
  return g;
}

AssocGroup::AssocGroup(Reactor& primary, bool offerer, uint32_t count, const rtc::PcConfig& pc, uint64_t busy_poll_us,
                       SessionFactory factory, SendFn send, StateFn state)
    : primary_(primary), offerer_(offerer), pc_(std::make_unique<rtc::PcConfig>(pc)), factory_(std::move(factory)),
      send_(std::move(send)), state_(std::move(state)) {
  pc_->gauges = false;  // the metrics endpoint's transport gauges stay the first association's
  const uint32_t n = std::min(count, proto::kMaxAssoc);
  for (uint32_t k = 1; k < n; k++)
    threads_.push_back(std::make_unique<WorkerThread>(int(k), busy_poll_us, "p2pt-assoc", 80 + int(k)));
}

void AssocGroup::start() {
  std::weak_ptr<AssocGroup> self = shared_from_this();
  for (size_t k = 1; k <= threads_.size(); k++) {
    Reactor& r = threads_[k - 1]->reactor();
    auto link = std::make_shared<AssocLink>(r, primary_, self, k, offerer_, *pc_, factory_);
    links_.push_back(link);
    r.post_threadsafe([link] { link->start(); });
  }
  LOG_INFO(kT, "%zu extra association(s) %s", threads_.size(), offerer_ ? "offered" : "awaited");
}

AssocGroup::~AssocGroup() {
  // Each link is shut down and released on its own thread, then the threads
  // are joined (each drains what was posted to it).
  for (size_t k = 0; k < links_.size(); k++)
    threads_[k]->reactor().post_threadsafe([l = std::move(links_[k])]() mutable {
      l->shutdown();
      l.reset();
    });
  links_.clear();
  threads_.clear();
}

void AssocGroup::on_frame(const proto::Frame& f) {
  const size_t k = f.stream_id;
  if (k < 1 || k > links_.size()) {
    LOG_WARN(kT, "ASSOC frame for unknown association %zu", k);
    return;
  }
  Json j;
  std::string err;
  if (!proto::json_parse_bytes(f.payload, j, &err) || !j.is_object() || !j.get("kind") ||
      !j.get("kind")->is_string()) {
    LOG_WARN(kT, "malformed ASSOC frame for association %zu: %s", k, err.c_str());
    return;
  }
  const std::string kind = j.get("kind")->as_string();
  std::string value;
  for (const char* key : {"sdp", "candidate"})
    if (const Json* v = j.get(key); v && v->is_string()) value = v->as_string();
  std::weak_ptr<AssocLink> w = links_[k - 1];
  threads_[k - 1]->reactor().post_threadsafe([w, kind, value] {
    if (auto l = w.lock()) l->on_signal(kind, value);
  });
}

void AssocGroup::send_signal(size_t index, const std::string& kind, const std::string& key, const std::string& value) {
  if (send_) send_(make_assoc_frame(uint32_t(index), kind, key, value));
}

void AssocGroup::link_state(size_t index, bool up, const std::string& why) {
  metrics::counter_add(up ? "tunnel_assoc_up_total" : "tunnel_assoc_down_total");
  if (!up && send_) send_(make_assoc_frame(uint32_t(index), "bye", "", ""));
  if (state_) state_(index, up, why);
}

}  // namespace p2pt
