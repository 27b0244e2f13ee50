// Thread wake-up cost on this host: how long a hop between two threads takes
// when the receiving thread sleeps in epoll_wait (and its CPU idles) against
// when it polls. Every hop of the tunnel's token path is such a hand-off
// (client -> proxy -> UDP -> serve -> upstream and back), so this is the
// floor under the added TTFT that no amount of per-packet work removes.
//
//   tunnel-wakebench [--iters N] [--gaps us,us,...] [--pin a,b]
//
// Thread A sends a ping and polls for the reply (it never sleeps, so its own
// wake-up is not measured); thread B waits for the ping (sleeping in
// epoll_wait, or polling epoll with a zero timeout), answers it at once.
// Before each ping A waits `gap` us (polling the clock), so B has been idle
// that long: a CPU idle for 100 ms sits in its deepest C-state, one idle for
// 20 us does not. One JSON line per (channel, B mode, gap): round trip
// p50/p90/p99 in us.
#include <netinet/in.h>
#include <pthread.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

void pin(int cpu) {
  if (cpu < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(cpu, &s);
  pthread_setaffinity_np(pthread_self(), sizeof s, &s);
}

// A channel carries one byte-sized message each way: two eventfds, or two
// connected loopback UDP sockets.
struct Channel {
  int a_rx = -1, a_tx = -1, b_rx = -1, b_tx = -1;
  bool udp = false;
  explicit Channel(bool u) : udp(u) {
    if (!udp) {
      a_rx = b_tx = eventfd(0, EFD_NONBLOCK);
      b_rx = a_tx = eventfd(0, EFD_NONBLOCK);
      return;
    }
    int s1 = socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK, 0), s2 = socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK, 0);
    sockaddr_in x{};
    x.sin_family = AF_INET;
    x.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t l = sizeof x;
    sockaddr_in p1 = x, p2 = x;
    bind(s1, reinterpret_cast<sockaddr*>(&p1), sizeof p1);
    bind(s2, reinterpret_cast<sockaddr*>(&p2), sizeof p2);
    getsockname(s1, reinterpret_cast<sockaddr*>(&p1), &l);
    getsockname(s2, reinterpret_cast<sockaddr*>(&p2), &l);
    connect(s1, reinterpret_cast<sockaddr*>(&p2), sizeof p2);
    connect(s2, reinterpret_cast<sockaddr*>(&p1), sizeof p1);
    a_rx = a_tx = s1;
    b_rx = b_tx = s2;
  }
  ~Channel() {
    if (udp) {
      close(a_rx);
      close(b_rx);
    } else {
      close(a_rx);
      close(b_rx);
    }
  }
  void send(int fd) const {
    if (udp) {
      char c = 1;
      (void)!::send(fd, &c, 1, 0);
    } else {
      uint64_t one = 1;
      (void)!::write(fd, &one, sizeof one);
    }
  }
  bool recv(int fd) const {
    if (udp) {
      char buf[64];
      return ::recv(fd, buf, sizeof buf, MSG_DONTWAIT) > 0;
    }
    uint64_t v;
    return ::read(fd, &v, sizeof v) == sizeof v;
  }
};

struct Result {
  double p50, p90, p99;
};

Result run(bool udp, bool spin, uint64_t gap_us, int iters, int cpu_a, int cpu_b) {
  Channel ch(udp);
  std::atomic<bool> stop{false};
  std::thread b([&] {
    pin(cpu_b);
    int ep = epoll_create1(0);
    epoll_event ev{};
    ev.events = EPOLLIN;
    epoll_ctl(ep, EPOLL_CTL_ADD, ch.b_rx, &ev);
    epoll_event out[4];
    while (!stop.load(std::memory_order_relaxed)) {
      int n = epoll_wait(ep, out, 4, spin ? 0 : 50);
      if (n <= 0) continue;
      while (ch.recv(ch.b_rx)) ch.send(ch.b_tx);
    }
    close(ep);
  });
  pin(cpu_a);
  std::vector<double> rtt;
  rtt.reserve(size_t(iters));
  for (int i = 0; i < iters + 3; i++) {
    const uint64_t until = now_ns() + gap_us * 1000;
    while (now_ns() < until) {
    }
    const uint64_t t0 = now_ns();
    ch.send(ch.a_tx);
    while (!ch.recv(ch.a_rx)) {
    }
    if (i >= 3) rtt.push_back(double(now_ns() - t0) / 1000.0);
  }
  stop = true;
  b.join();
  std::sort(rtt.begin(), rtt.end());
  auto q = [&](double p) { return rtt[std::min(rtt.size() - 1, size_t(p * double(rtt.size() - 1) + 0.5))]; };
  return {q(0.5), q(0.9), q(0.99)};
}

}  // namespace

int main(int argc, char** argv) {
  int iters = 400;
  std::vector<uint64_t> gaps = {0, 20, 100, 500, 2000, 20000, 100000};
  int cpu_a = -1, cpu_b = -1;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--iters") iters = std::max(10, atoi(v.c_str()));
    else if (k == "--gaps") {
      gaps.clear();
      size_t p = 0;
      while (p <= v.size()) {
        size_t q = v.find(',', p);
        if (q == std::string::npos) q = v.size();
        if (q > p) gaps.push_back(strtoull(v.substr(p, q - p).c_str(), nullptr, 10));
        p = q + 1;
      }
    } else if (k == "--pin") {
      sscanf(v.c_str(), "%d,%d", &cpu_a, &cpu_b);
    } else {
      fprintf(stderr, "usage: %s [--iters N] [--gaps us,...] [--pin a,b]\n", argv[0]);
      return 2;
    }
  }
  for (bool udp : {false, true})
    for (bool spin : {false, true})
      for (uint64_t g : gaps) {
        // Keep each point near a second: long gaps get fewer pings.
        const int n = g ? std::max(20, std::min(iters, int(1500000 / g))) : iters;
        Result r = run(udp, spin, g, n, cpu_a, cpu_b);
        printf("{\"channel\": \"%s\", \"b\": \"%s\", \"gap_us\": %llu, \"n\": %d, \"rtt_p50_us\": %.1f, "
               "\"rtt_p90_us\": %.1f, \"rtt_p99_us\": %.1f}\n",
               udp ? "udp" : "eventfd", spin ? "spin" : "sleep", static_cast<unsigned long long>(g), n, r.p50, r.p90,
               r.p99);
        fflush(stdout);
      }
  return 0;
}
