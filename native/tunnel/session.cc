#include "tunnel/session.h"

#include "core/log.h"
#include "rtc/peer.h"
#include "tunnel/signaling.h"

namespace p2pt {

static const char* kT = "tunnel::rtc";

namespace {

class WebrtcSession : public std::enable_shared_from_this<WebrtcSession> {
 public:
  WebrtcSession(Reactor& r, const AppConfig& cfg, ConnectCb cb) : r_(r), cfg_(cfg), cb_(std::move(cb)) {}
  ~WebrtcSession() {
    if (gather_timer_) r_.cancel(gather_timer_);
    if (pc_) {
      pc_->on_state = nullptr;
      pc_->on_ice_candidate = nullptr;
      pc_->on_gathering_complete = nullptr;
      pc_->on_data_channel = nullptr;
      pc_->close();
    }
    // sig_ destructor sends {"type":"bye"} (reference signaling.rs:72-77).
  }

  void start() {
    std::weak_ptr<WebrtcSession> w = shared_from_this();
    SignalingClient::connect(r_, cfg_.signal, cfg_.room, [w](std::shared_ptr<SignalingClient> sig, std::string err) {
      auto s = w.lock();
      if (!s) return;
      if (!sig) {
        s->finish(nullptr, err);
        return;
      }
      s->sig_ = sig;
      sig->on_signal = [w](const IncomingSignal& m) {
        if (auto s2 = w.lock()) s2->on_signal(m);
      };
      sig->on_closed = [w](const std::string&) {
        auto s2 = w.lock();
        if (s2 && !s2->done_) s2->finish(nullptr, "signaling connection lost");
      };
    });
  }

 private:
  enum class Phase { Joining, WaitPeer, Negotiating };

  void finish(std::shared_ptr<MessageChannel> ch, const std::string& err) {
    if (done_) return;
    done_ = true;
    if (gather_timer_) r_.cancel(gather_timer_);
    gather_timer_ = 0;
    auto cb = std::move(cb_);
    cb_ = nullptr;
    if (cb) cb(std::move(ch), err);
  }

  rtc::PcConfig pc_config() const { return make_pc_config(cfg_); }

  void on_signal(const IncomingSignal& m) {
    if (done_) return;  // like the reference, signalling is not consulted once connected
    using K = IncomingSignal::Kind;
    if (m.kind == K::Error) {
      finish(nullptr, "signaling error: " + m.message);
      return;
    }
    switch (phase_) {
      case Phase::Joining:
        if (m.kind != K::Joined) {
          LOG_DEBUG(kT, "ignoring signal while joining: %s", signal_kind_name(m.kind));
          return;
        }
        {
          std::string peers;
          for (auto& p : m.peers) peers += (peers.empty() ? "\"" : ", \"") + p + "\"";
          LOG_INFO(kT, "joined as peer %s - existing peers: [%s]", m.peer_id.c_str(), peers.c_str());
        }
        if (m.peers.empty()) {
          LOG_INFO(kT, "waiting for peer to join room...");
          phase_ = Phase::WaitPeer;
        } else {
          LOG_INFO(kT, "peer already in room, we are answerer");
          become(false);
        }
        return;
      case Phase::WaitPeer:
        if (m.kind == K::PeerJoined) {
          LOG_INFO(kT, "peer joined, we are offerer");
          become(true);
        } else {
          // Q7 fix: stay here instead of falling back to waiting for `joined`.
          LOG_DEBUG(kT, "ignoring signal while waiting for peer: %s", signal_kind_name(m.kind));
        }
        return;
      case Phase::Negotiating:
        negotiate(m);
        return;
    }
  }

  void become(bool offerer) {
    phase_ = Phase::Negotiating;
    offerer_ = offerer;
    pc_ = rtc::PeerConnection::create(r_, pc_config(), offerer);
    std::weak_ptr<WebrtcSession> w = shared_from_this();
    pc_->on_ice_candidate = [w](const std::string& cand) {
      auto s = w.lock();
      if (!s || !s->sig_) return;
      LOG_DEBUG(kT, "sending ICE candidate");
      s->sig_->send_candidate(cand);
    };
    pc_->on_state = [w](rtc::PcState st) {
      auto s = w.lock();
      if (!s) return;
      if (st == rtc::PcState::Failed && !s->done_) s->finish(nullptr, "ICE connection failed");
    };
    if (offerer) {
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
      pc_->start_gathering();  // candidates trickle as soon as the offer is applied
    }
  }

  void arm_gather_timeout() {
    std::weak_ptr<WebrtcSession> w = shared_from_this();
    // Reference waits <= 5 s for gathering before sending the SDP (rtc.rs:181-182).
    gather_timer_ = r_.call_later_ms(cfg_.rtc.gather_timeout_ms, [w] {
      if (auto s = w.lock()) {
        s->gather_timer_ = 0;
        s->send_sdp();
      }
    });
  }

  void send_sdp() {
    if (sdp_sent_ || !pc_ || !sig_) return;
    if (!offerer_ && !remote_set_) return;
    sdp_sent_ = true;
    if (gather_timer_) r_.cancel(gather_timer_);
    gather_timer_ = 0;
    std::string sdp = pc_->local_description();
    if (offerer_) {
      LOG_INFO(kT, "sending offer");
      sig_->send_offer(sdp);
    } else {
      LOG_INFO(kT, "sending answer");
      sig_->send_answer(sdp);
    }
  }

  void apply_remote(const std::string& sdp) {
    std::string err;
    if (!pc_->set_remote_description(sdp, &err)) {
      finish(nullptr, "invalid remote description: " + err);
      return;
    }
    remote_set_ = true;
    if (!buffered_.empty()) LOG_INFO(kT, "applying %zu buffered ICE candidate(s)", buffered_.size());
    for (auto& c : buffered_) add_candidate(c);
    buffered_.clear();
  }

  void add_candidate(const std::string& c) {
    std::string err;
    if (!pc_->add_ice_candidate(c, &err)) LOG_WARN(kT, "skipping bad ICE candidate: %s", err.c_str());
  }

  void negotiate(const IncomingSignal& m) {
    using K = IncomingSignal::Kind;
    switch (m.kind) {
      case K::Offer:
        if (offerer_) break;
        LOG_INFO(kT, "received offer");
        apply_remote(m.sdp);
        if (done_) return;
        if (pc_->gathering_complete()) {
          send_sdp();
        } else {
          std::weak_ptr<WebrtcSession> w = shared_from_this();
          pc_->on_gathering_complete = [w] {
            if (auto s = w.lock()) s->send_sdp();
          };
          arm_gather_timeout();
        }
        return;
      case K::Answer:
        if (!offerer_ || remote_set_) break;
        LOG_INFO(kT, "received answer");
        apply_remote(m.sdp);
        return;
      case K::Candidate:
        if (remote_set_) {
          LOG_DEBUG(kT, "applying ICE candidate immediately");
          add_candidate(m.candidate);
        } else {
          LOG_DEBUG(kT, "buffering ICE candidate (remote description not yet set)");
          buffered_.push_back(m.candidate);
        }
        return;
      case K::PeerLeft:
        finish(nullptr, "peer left before connection established");
        return;
      default:
        break;
    }
    LOG_DEBUG(kT, "ignoring signal during %s: %s", offerer_ ? "offer" : "answer", signal_kind_name(m.kind));
  }

  void watch_channel() {
    std::weak_ptr<WebrtcSession> w = shared_from_this();
    auto opened = [w] {
      auto s = w.lock();
      if (!s || s->done_) return;
      LOG_INFO(kT, "WebRTC connection established (%s) via %s", s->offerer_ ? "offerer" : "answerer",
               s->pc_->describe_path().c_str());
      s->finish(s->dc_, "");
    };
    if (dc_->is_open()) opened();
    else dc_->on_open = opened;
  }

  Reactor& r_;
  AppConfig cfg_;
  ConnectCb cb_;
  std::shared_ptr<SignalingClient> sig_;
  std::shared_ptr<rtc::PeerConnection> pc_;
  std::shared_ptr<rtc::DataChannel> dc_;
  Phase phase_ = Phase::Joining;
  bool offerer_ = false;
  bool remote_set_ = false;
  bool sdp_sent_ = false;
  bool done_ = false;
  uint64_t gather_timer_ = 0;
  std::vector<std::string> buffered_;
};

}  // namespace

rtc::PcConfig make_pc_config(const AppConfig& cfg) {
  rtc::PcConfig pc;
  pc.ice.stun_urls = cfg.rtc.stun_servers;
  pc.ice.turn_url = cfg.rtc.turn.url;
  pc.ice.turn_user = cfg.rtc.turn.username;
  pc.ice.turn_pass = cfg.rtc.turn.password;
  pc.ice.include_loopback = cfg.rtc.include_loopback;
  pc.ice.include_ipv6 = cfg.rtc.include_ipv6;
  pc.ice.ipv6_only = cfg.rtc.ipv6_only;
  pc.ice.relay_only = cfg.rtc.relay_only;
  pc.ice.failed_ms = cfg.rtc.ice_failed_timeout_ms;
  pc.sctp_mtu = cfg.rtc.sctp_mtu;
  pc.allow_jumbo = cfg.rtc.allow_jumbo_loopback;
  pc.sack_delay_us = cfg.mode == "serve" ? 5000 : 0;
  return pc;
}

std::shared_ptr<void> connect_webrtc(Reactor& r, const AppConfig& cfg, ConnectCb cb) {
  auto s = std::make_shared<WebrtcSession>(r, cfg, std::move(cb));
  s->start();
  return s;
}

}  // namespace p2pt
