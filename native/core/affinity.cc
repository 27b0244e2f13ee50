#include "core/affinity.h"

#include <sched.h>

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
  } else if (n >= 6 && (tag == 92 || tag == 90 || tag == 93)) {
    slot = tag == 92 ? 1 : tag == 90 ? 2 : 3;  // reader, seal, send: a CPU each
  } else if (n >= 6) {
    slot = 4 + g_next.fetch_add(1, std::memory_order_relaxed) % (n - 4);  // workers, RX lane, second sealer
  } else {
    slot = 1 + g_next.fetch_add(1, std::memory_order_relaxed) % (n - 1);
  }
  const int cpu = g_cpus[slot];
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpu, &one);
  sched_setaffinity(0, sizeof one, &one);
}

}  // namespace p2pt::affinity
