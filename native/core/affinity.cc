#include "core/affinity.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace p2pt::affinity {

namespace {
std::atomic<bool> g_default{false};
}  // namespace

void set_default(bool on) { g_default.store(on, std::memory_order_relaxed); }

bool enabled() {
  const char* e = getenv("TUNNEL_PIN_THREADS");
  if (e && *e) return *e == '1';
  return g_default.load(std::memory_order_relaxed);
}

namespace {
std::once_flag g_once;
std::vector<int> g_cpus;  // the process's CPU set, captured once
std::atomic<unsigned> g_next{0};
}  // namespace

static void capture() {
  std::call_once(g_once, [] {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) != 0) return;
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &set)) g_cpus.push_back(c);
  });
}

long process_cpu_count() {
  capture();
  return long(g_cpus.size());
}

void pin_this_thread(int tag) {
  if (!enabled()) return;
  capture();
  const size_t n = g_cpus.size();
  if (n < 2) return;
  size_t slot;
  if (tag == 0) {
    slot = 0;
  } else if (n >= 5) {
    // [assoc][workers ...][seal][send][reader][RX lane][open 0][open 1]: the
    // workers (which talk to the upstreams / clients over TCP) next to the
    // association thread, the receive stages last (on a set that spans two L3
    // domains, nearest the peer's side). (Seal and send sharing one CPU, the
    // workers getting the other, lost on the 64 x 1 MB echo: 1576 vs 1940
    // req/s, profiles/r04/txs30.) Below 8 CPUs the open lanes have no CPUs of
    // their own: one runs, on the RX lane's; on 5 that is the reader's own.
    const bool own_open = n >= 8;
    const size_t nw = own_open ? n - 7 : n >= 6 ? n - 5 : 1;
    const size_t seal = 1 + nw, send = seal + 1, reader = send + 1, rx = std::min(reader + 1, n - 1);
    if (tag >= 1 && tag < 90) slot = 1 + size_t(tag - 1) % nw;
    else if (tag == 90) slot = seal;
    else if (tag == 93) slot = send;
    else if (tag == 92) slot = reader;
    else if (tag == 95 && own_open) slot = rx + 1;
    else if (tag == 96 && own_open) slot = rx + 2;
    else slot = rx;  // RX lane, second sealer (and the one open lane below 8 CPUs)
  } else {
    slot = 1 + g_next.fetch_add(1, std::memory_order_relaxed) % (n - 1);
  }
  const int cpu = g_cpus[slot];
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpu, &one);
  sched_setaffinity(0, sizeof one, &one);
}

int open_lane_count(int want) {
  if (!enabled()) return want;
  capture();
  return g_cpus.size() >= 8 ? want : 1;
}

}  // namespace p2pt::affinity
