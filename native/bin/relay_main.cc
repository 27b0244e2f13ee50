// tunnel-relay: a TURN server (RFC 8656: UDP clients, UDP relays, long-term
// credentials) whose relayed traffic crosses ONE emulated bottleneck link.
//
// Every tunnel relayed through one server competes for the same queue, which
// the per-agent WAN emulator of the ICE agent (native/rtc/ice.cc, one link per
// association) cannot model: this is what the congestion response's
// shared-bottleneck fairness is measured on (bench/bench_fairness.py). The
// Python relay the round-4 rows used (utils/turn_server.py, kept as the
// independent TURN implementation the native client is tested against) tops
// out near 17 MB/s, so its 200 Mbit/s rows were relay-bound; this one keeps
// a 1 Gbit/s link's schedule to the microsecond (Reactor timers on
// epoll_pwait2).
//
//   tunnel-relay [--port 0] [--user u --pass p --realm r]
//                [--rate-mbps R] [--delay-ms D] [--queue-kb Q] [--loss L]
//                [--back-rate-mbps R] [--seed N]
//
// Towards peers (the forward link): serialisation at R Mbit/s (0 = unlimited)
// into a drop-tail queue of Q KiB (default one BDP at D, at least 32 KiB),
// then D ms of one-way delay, Bernoulli loss L. Back towards clients: D ms of
// delay (and its own rate when --back-rate-mbps is given). Prints
// "relay listening on turn:127.0.0.1:PORT"; on SIGTERM/SIGINT prints one JSON
// line of counters and exits.
#include <netinet/in.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "core/crypto.h"
#include "core/net.h"
#include "core/reactor.h"
#include "rtc/stun.h"

using namespace p2pt;

namespace {

// One direction of the bottleneck. Delivery times are non-decreasing (FIFO
// serialisation plus a fixed delay), so a deque is the schedule.
struct Link {
  double rate = 0;  // bytes per microsecond (0 = unlimited)
  uint64_t delay_us = 0;
  size_t queue = 0;
  double loss = 0;
  uint64_t free_us = 0;  // when the link finishes serialising what it holds
  struct Pkt {
    uint64_t at;
    int fd;
    SockAddr to;
    std::vector<uint8_t> data;
  };
  std::deque<Pkt> q;
  uint64_t packets = 0, bytes = 0, queue_drops = 0, loss_drops = 0, max_queue = 0;
  Reactor::TimerId timer = 0;
};

struct Alloc {
  int relay = -1;
  SockAddr relay_addr;
  std::set<std::string> perms;               // peer IPs
  std::map<uint16_t, SockAddr> chans;        // channel -> peer
  std::map<std::string, uint16_t> peer_ch;   // peer str -> channel
};

class Relay {
 public:
  Relay(Reactor& r, std::string user, std::string pass, std::string realm, uint64_t seed)
      : r_(r), user_(std::move(user)), realm_(std::move(realm)), key_(stun::long_term_key(user_, realm_, pass)),
        rng_(seed) {
    nonce_ = "p2pt" + std::to_string(seed * 7919 + 17);
  }
  Link fwd, back;

  bool listen(uint16_t port) {
    fd_ = ::socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    SockAddr a;
    SockAddr::parse("127.0.0.1", port, a);
    if (::bind(fd_, a.sa(), a.len) != 0) return false;
    udp_socket_buffers(fd_, 8 << 20);
    socklen_t l = sizeof a.ss;
    getsockname(fd_, a.sa(), &l);
    a.len = l;
    port_ = a.port();
    r_.add(fd_, EPOLLIN, [this](uint32_t) { drain(fd_, true); });
    return true;
  }
  uint16_t port() const { return port_; }

  std::string stats() const {
    char b[768];
    snprintf(b, sizeof b,
             "{\"allocations\": %llu, \"relayed_to_peer\": %llu, \"relayed_to_client\": %llu, \"link\": {\"packets\": %llu, "
             "\"bytes\": %llu, \"queue_drops\": %llu, \"loss_drops\": %llu, \"max_queue_bytes\": %llu, \"queue_bytes\": %zu}, "
             "\"back\": {\"packets\": %llu, \"bytes\": %llu, \"queue_drops\": %llu}}",
             (unsigned long long)allocations_, (unsigned long long)to_peer_, (unsigned long long)to_client_,
             (unsigned long long)fwd.packets, (unsigned long long)fwd.bytes, (unsigned long long)fwd.queue_drops,
             (unsigned long long)fwd.loss_drops, (unsigned long long)fwd.max_queue, fwd.queue,
             (unsigned long long)back.packets, (unsigned long long)back.bytes, (unsigned long long)back.queue_drops);
    return b;
  }

 private:
  // Reads every queued datagram of one socket: the client socket (TURN
  // messages, ChannelData) or a relay socket (traffic from peers).
  void drain(int fd, bool client) {
    uint8_t buf[65536];
    for (int i = 0; i < 256; i++) {
      SockAddr from;
      from.len = sizeof from.ss;
      ssize_t n = ::recvfrom(fd, buf, sizeof buf, MSG_DONTWAIT, from.sa(), &from.len);
      if (n <= 0) return;
      if (client) on_client(buf, size_t(n), from);
      else on_peer(fd, buf, size_t(n), from);
    }
  }

  void send_to_client(const SockAddr& to, std::vector<uint8_t> data) {
    submit(back, fd_, to, std::move(data));
  }

  void reply(const SockAddr& to, const stun::Message& m, bool auth) {
    auto out = m.serialize(auth ? &key_ : nullptr, true);
    ::sendto(fd_, out.data(), out.size(), 0, to.sa(), to.len);  // control replies skip the link
  }

  void error(const SockAddr& to, const stun::Message& req, int code, const char* why) {
    stun::Message e;
    e.type = uint16_t(req.method() | 0x0110);
    memcpy(e.tid, req.tid, 12);
    e.add_error(code, why);
    e.add(stun::kRealm, realm_);
    e.add(stun::kNonce, nonce_);
    reply(to, e, false);
  }

  void on_client(const uint8_t* p, size_t n, const SockAddr& from) {
    const std::string key = from.str();
    if (n >= 4 && p[0] >= 0x40 && p[0] <= 0x7F) {  // ChannelData
      const uint16_t ch = uint16_t(p[0] << 8 | p[1]), len = uint16_t(p[2] << 8 | p[3]);
      auto it = allocs_.find(key);
      if (it == allocs_.end() || size_t(4) + len > n) return;
      auto c = it->second->chans.find(ch);
      if (c == it->second->chans.end()) return;
      to_peer_++;
      submit(fwd, it->second->relay, c->second, std::vector<uint8_t>(p + 4, p + 4 + len));
      return;
    }
    stun::Message m;
    if (!stun::Message::parse(p, n, m)) return;
    if (m.type == stun::kSendIndication) {
      auto it = allocs_.find(key);
      SockAddr peer;
      const stun::Attr* d = m.get(stun::kData);
      if (it == allocs_.end() || !d || !m.get_xor_addr(stun::kXorPeerAddress, peer)) return;
      if (!it->second->perms.count(peer.ip())) return;
      to_peer_++;
      submit(fwd, it->second->relay, peer, std::vector<uint8_t>(d->value.begin(), d->value.end()));
      return;
    }
    if (m.cls() != 0) return;  // requests only
    stun::Message ok;
    ok.type = uint16_t(m.method() | 0x0100);
    memcpy(ok.tid, m.tid, 12);
    if (m.method() == 0x0001) {  // Binding
      ok.add_xor_addr(stun::kXorMappedAddress, from);
      reply(from, ok, false);
      return;
    }
    const stun::Attr* u = m.get(stun::kUsername);
    const stun::Attr* rl = m.get(stun::kRealm);
    if (!u || u->value != user_ || !rl || rl->value != realm_ || !stun::verify_integrity(p, n, m, key_)) {
      error(from, m, 401, "Unauthorized");
      return;
    }
    auto it = allocs_.find(key);
    switch (m.method()) {
      case 0x0003: {  // Allocate
        if (it != allocs_.end()) {
          error(from, m, 437, "Allocation Mismatch");
          return;
        }
        auto a = std::make_unique<Alloc>();
        a->relay = ::socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        SockAddr ra;
        SockAddr::parse("127.0.0.1", 0, ra);
        ::bind(a->relay, ra.sa(), ra.len);
        udp_socket_buffers(a->relay, 8 << 20);
        socklen_t l = sizeof ra.ss;
        getsockname(a->relay, ra.sa(), &l);
        ra.len = l;
        a->relay_addr = ra;
        const int rfd = a->relay;
        r_.add(rfd, EPOLLIN, [this, rfd](uint32_t) { drain(rfd, false); });
        by_relay_[rfd] = from;
        allocs_[key] = std::move(a);
        allocations_++;
        ok.add_xor_addr(stun::kXorRelayedAddress, ra);
        ok.add_xor_addr(stun::kXorMappedAddress, from);
        ok.add_u32(stun::kLifetime, 600);
        reply(from, ok, true);
        return;
      }
      case 0x0004: {  // Refresh
        uint32_t lt = 600;
        m.get_u32(stun::kLifetime, lt);
        if (lt == 0 && it != allocs_.end()) {
          r_.remove(it->second->relay);
          by_relay_.erase(it->second->relay);
          ::close(it->second->relay);
          allocs_.erase(it);
        }
        ok.add_u32(stun::kLifetime, lt);
        reply(from, ok, true);
        return;
      }
      case 0x0008: {  // CreatePermission
        SockAddr peer;
        if (it != allocs_.end() && m.get_xor_addr(stun::kXorPeerAddress, peer)) it->second->perms.insert(peer.ip());
        reply(from, ok, true);
        return;
      }
      case 0x0009: {  // ChannelBind
        SockAddr peer;
        uint32_t chv = 0;
        if (it == allocs_.end() || !m.get_u32(stun::kChannelNumber, chv) || !m.get_xor_addr(stun::kXorPeerAddress, peer)) {
          error(from, m, 400, "Bad Request");
          return;
        }
        const uint16_t ch = uint16_t(chv >> 16);
        it->second->chans[ch] = peer;
        it->second->peer_ch[peer.str()] = ch;
        it->second->perms.insert(peer.ip());
        reply(from, ok, true);
        return;
      }
      default:
        error(from, m, 400, "Bad Request");
    }
  }

  // From a peer to the relay: back to the client as ChannelData (bound
  // channel) or a Data indication.
  void on_peer(int rfd, const uint8_t* p, size_t n, const SockAddr& peer) {
    auto c = by_relay_.find(rfd);
    if (c == by_relay_.end()) return;
    auto it = allocs_.find(c->second.str());
    if (it == allocs_.end() || !it->second->perms.count(peer.ip())) return;
    std::vector<uint8_t> out;
    auto ch = it->second->peer_ch.find(peer.str());
    if (ch != it->second->peer_ch.end()) {
      out.resize(4 + ((n + 3) & ~size_t(3)), 0);
      out[0] = uint8_t(ch->second >> 8);
      out[1] = uint8_t(ch->second);
      out[2] = uint8_t(n >> 8);
      out[3] = uint8_t(n);
      memcpy(out.data() + 4, p, n);
    } else {
      stun::Message d = stun::Message::make(stun::kDataIndication);
      d.add_xor_addr(stun::kXorPeerAddress, peer);
      d.add(stun::kData, p, n);
      out = d.serialize(nullptr, false);
    }
    to_client_++;
    send_to_client(c->second, std::move(out));
  }

  // Into a link: lost (Bernoulli), dropped at the tail of a full queue, or
  // scheduled for its delivery time.
  void submit(Link& l, int fd, const SockAddr& to, std::vector<uint8_t> data) {
    const uint64_t now = Reactor::now_us();
    const size_t n = data.size();
    if (l.loss > 0 && std::uniform_real_distribution<double>(0, 1)(rng_) < l.loss) {
      l.loss_drops++;
      return;
    }
    uint64_t at = now + l.delay_us;
    if (l.rate > 0) {
      const double backlog = l.free_us > now ? double(l.free_us - now) * l.rate : 0.0;
      if (backlog + double(n) > double(l.queue)) {
        l.queue_drops++;
        return;
      }
      l.max_queue = std::max<uint64_t>(l.max_queue, uint64_t(backlog) + n);
      l.free_us = std::max(now, l.free_us) + uint64_t(std::ceil(double(n) / l.rate));
      at = l.free_us + l.delay_us;
    }
    l.packets++;
    l.bytes += n;
    if (at <= now) {
      ::sendto(fd, data.data(), n, 0, to.sa(), to.len);
      return;
    }
    l.q.push_back(Link::Pkt{at, fd, to, std::move(data)});
    if (!l.timer) arm(l);
  }

  void arm(Link& l) {
    l.timer = r_.call_at(l.q.front().at, [this, &l] {
      l.timer = 0;
      const uint64_t now = Reactor::now_us();
      while (!l.q.empty() && l.q.front().at <= now) {
        auto& pk = l.q.front();
        ::sendto(pk.fd, pk.data.data(), pk.data.size(), 0, pk.to.sa(), pk.to.len);
        l.q.pop_front();
      }
      if (!l.q.empty()) arm(l);
    });
  }

  Reactor& r_;
  std::string user_, realm_, key_, nonce_;
  std::mt19937_64 rng_;
  int fd_ = -1;
  uint16_t port_ = 0;
  std::unordered_map<std::string, std::unique_ptr<Alloc>> allocs_;
  std::unordered_map<int, SockAddr> by_relay_;
  uint64_t allocations_ = 0, to_peer_ = 0, to_client_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  std::map<std::string, std::string> o = {{"port", "0"},      {"user", "u"},       {"pass", "p"},
                                          {"realm", "p2pt.test"}, {"rate-mbps", "0"}, {"delay-ms", "0"},
                                          {"queue-kb", "0"},   {"loss", "0"},       {"back-rate-mbps", "0"},
                                          {"seed", "1"}};
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i];
    if (k.rfind("--", 0) != 0 || !o.count(k.substr(2))) {
      fprintf(stderr, "usage: %s [--port N] [--user U --pass P --realm R] [--rate-mbps R] [--delay-ms D] "
                      "[--queue-kb Q] [--loss L] [--back-rate-mbps R] [--seed N]\n", argv[0]);
      return 2;
    }
    o[k.substr(2)] = argv[i + 1];
  }
  Reactor r;
  Relay relay(r, o["user"], o["pass"], o["realm"], strtoull(o["seed"].c_str(), nullptr, 10));
  const double rate = atof(o["rate-mbps"].c_str()), delay_ms = atof(o["delay-ms"].c_str());
  relay.fwd.rate = rate / 8.0;  // Mbit/s -> bytes/us
  relay.fwd.delay_us = uint64_t(delay_ms * 1000);
  relay.fwd.loss = atof(o["loss"].c_str());
  const double qkb = atof(o["queue-kb"].c_str());
  // Default queue: one BDP of the forward link at the one-way delay x 2, at least 32 KiB.
  relay.fwd.queue = qkb > 0 ? size_t(qkb * 1024) : std::max<size_t>(32 * 1024, size_t(rate / 8.0 * delay_ms * 2000));
  relay.back.rate = atof(o["back-rate-mbps"].c_str()) / 8.0;
  relay.back.delay_us = relay.fwd.delay_us;
  relay.back.queue = relay.back.rate > 0 ? std::max<size_t>(32 * 1024, size_t(relay.back.rate * delay_ms * 2000)) : 0;
  if (!relay.listen(uint16_t(atoi(o["port"].c_str())))) {
    fprintf(stderr, "cannot bind the relay port\n");
    return 1;
  }
  signal(SIGPIPE, SIG_IGN);
  r.on_signal(SIGTERM, [&r] { r.stop(); });
  r.on_signal(SIGINT, [&r] { r.stop(); });
  printf("relay listening on turn:127.0.0.1:%u (forward link %.1f Mbit/s, %.1f ms, queue %zu KiB, loss %.4f)\n",
         relay.port(), rate, delay_ms, relay.fwd.queue / 1024, relay.fwd.loss);
  fflush(stdout);
  r.run();
  printf("%s\n", relay.stats().c_str());
  fflush(stdout);
  return 0;
}
