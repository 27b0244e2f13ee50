#include "core/profiler.h"

#include "core/affinity.h"

#include <dlfcn.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace p2pt::profiler {
namespace {

constexpr int kDepth = 10;          // frames per sample: pc, [rsp], fp chain
constexpr size_t kSlots = 1 << 15;  // distinct stacks kept

struct Slot {
  std::atomic<uint64_t> hash{0};
  uint64_t tag;
  uint64_t pcs[kDepth];
  std::atomic<uint64_t> count{0};
};

Slot* g_slots = nullptr;
std::atomic<uint64_t> g_samples{0}, g_dropped{0};
std::string g_path;
// Stack bounds of the interrupted thread (the process timer samples whichever
// thread is running: the main reactor or a worker, see register_thread()).
thread_local uintptr_t t_stack_lo = 0, t_stack_hi = 0;
thread_local uint64_t t_tag = 0;  // 0 = main reactor thread, k = worker k
std::atomic<bool> g_dumped{false};
int g_hz = 0;  // sampling rate once started

// One CPU-time timer per registered thread (CLOCK_THREAD_CPUTIME_ID, signal
// aimed at that thread): a process-wide ITIMER_PROF is capped by the kernel
// tick and lands on whichever thread happens to run, which left a busy
// association thread with a few hundred samples for a multi-second run.
struct ThreadTimer {
  timer_t id{};
  bool armed = false;
  void arm() {
    if (armed || !g_hz) return;
    sigevent ev = {};
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGPROF;
    ev._sigev_un._tid = pid_t(syscall(SYS_gettid));
    if (timer_create(CLOCK_THREAD_CPUTIME_ID, &ev, &id) != 0) return;
    itimerspec it = {};
    it.it_interval.tv_nsec = 1000000000L / g_hz;
    it.it_value = it.it_interval;
    timer_settime(id, 0, &it, nullptr);
    armed = true;
  }
  ~ThreadTimer() {
    if (armed) timer_delete(id);
  }
};
thread_local ThreadTimer t_timer;

inline bool on_stack(uintptr_t p) { return p >= t_stack_lo && p + 16 <= t_stack_hi && (p & 7) == 0; }

void on_sigprof(int, siginfo_t*, void* uc_) {
  auto* uc = static_cast<ucontext_t*>(uc_);
  uint64_t pcs[kDepth] = {};
  int n = 0;
#if defined(__x86_64__)
  uintptr_t pc = uc->uc_mcontext.gregs[REG_RIP];
  uintptr_t sp = uc->uc_mcontext.gregs[REG_RSP];
  uintptr_t fp = uc->uc_mcontext.gregs[REG_RBP];
  pcs[n++] = pc;
  // Heuristic caller of a frameless leaf: the word at the stack pointer.
  pcs[n++] = on_stack(sp) ? *reinterpret_cast<uint64_t*>(sp) : 0;
  while (n < kDepth && on_stack(fp)) {
    uintptr_t ret = reinterpret_cast<uint64_t*>(fp)[1];
    uintptr_t next = reinterpret_cast<uint64_t*>(fp)[0];
    if (!ret) break;
    pcs[n++] = ret;
    if (next <= fp) break;
    fp = next;
  }
#else
  (void)uc;
#endif
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < kDepth; i++) h = (h ^ pcs[i]) * 1099511628211ull;
  h = (h ^ t_tag) * 1099511628211ull;
  if (h == 0) h = 1;
  g_samples.fetch_add(1, std::memory_order_relaxed);
  for (size_t probe = 0; probe < 64; probe++) {
    Slot& s = g_slots[(h + probe) & (kSlots - 1)];
    uint64_t cur = s.hash.load(std::memory_order_acquire);
    if (cur == h) {
      s.count.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    if (cur == 0) {
      // Claim the slot (several threads may be sampled at once); a loser
      // re-reads it and either matches or probes on.
      if (!s.hash.compare_exchange_strong(cur, h, std::memory_order_acq_rel)) {
        if (cur == h) s.count.fetch_add(1, std::memory_order_relaxed);
        else continue;
        return;
      }
      memcpy(s.pcs, pcs, sizeof pcs);
      s.tag = t_tag;
      s.count.fetch_add(1, std::memory_order_relaxed);
      return;
    }
  }
  g_dropped.fetch_add(1, std::memory_order_relaxed);
}

void resolve(FILE* f, uint64_t a) {
  Dl_info di;
  // Raw addresses; scripts/profile_report.py backs return addresses up by one
  // byte so the symboliser attributes the call site.
  if (a && dladdr(reinterpret_cast<void*>(a), &di) && di.dli_fname) {
    fprintf(f, " %s+0x%lx", di.dli_fname, static_cast<unsigned long>(a - reinterpret_cast<uintptr_t>(di.dli_fbase)));
  } else {
    fprintf(f, " ?+0x%lx", static_cast<unsigned long>(a));
  }
}

}  // namespace

namespace timeline {
constexpr int kBuckets = 6;  // < 10 %, < 25 %, < 50 %, < 75 %, < 90 %, >= 90 % of an interval
struct Th {
  int tag;
  clockid_t cid;
  uint64_t last_ns = 0;
  uint64_t busy_ns = 0;
  uint32_t hist[kBuckets] = {};
  bool dead = false;
};
std::mutex mu;
std::vector<Th> threads;
std::atomic<bool> on{false};
std::string path;
uint64_t intervals = 0;

uint64_t cpu_ns(clockid_t c, bool* ok) {
  timespec ts;
  *ok = clock_gettime(c, &ts) == 0;
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

void add_self(int tag) {
  clockid_t c;
  if (pthread_getcpuclockid(pthread_self(), &c) != 0) return;
  bool ok;
  Th t{tag, c};
  t.last_ns = cpu_ns(c, &ok);
  std::lock_guard<std::mutex> lk(mu);
  threads.push_back(t);
}

void write_out() {
  if (!on.exchange(false)) return;
  std::lock_guard<std::mutex> lk(mu);
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return;
  fprintf(f, "{\"interval_ms\": 2, \"intervals\": %llu, \"buckets\": [\"<10\", \"<25\", \"<50\", \"<75\", \"<90\", \">=90\"], "
          "\"threads\": [", static_cast<unsigned long long>(intervals));
  for (size_t i = 0; i < threads.size(); i++) {
    const Th& t = threads[i];
    fprintf(f, "%s{\"tag\": %d, \"busy_s\": %.3f, \"hist\": [", i ? ", " : "", t.tag, double(t.busy_ns) / 1e9);
    for (int b = 0; b < kBuckets; b++) fprintf(f, "%s%u", b ? ", " : "", t.hist[b]);
    fprintf(f, "]}");
  }
  fprintf(f, "]}\n");
  fclose(f);
}

void run() {
  pthread_setname_np(pthread_self(), "p2pt-timeline");
  sigset_t mask;
  sigfillset(&mask);
  pthread_sigmask(SIG_BLOCK, &mask, nullptr);
  constexpr uint64_t kIntervalNs = 2000000;
  while (on.load(std::memory_order_relaxed)) {
    std::this_thread::sleep_for(std::chrono::nanoseconds(kIntervalNs));
    std::lock_guard<std::mutex> lk(mu);
    intervals++;
    for (auto& t : threads) {
      if (t.dead) continue;
      bool ok;
      const uint64_t now = cpu_ns(t.cid, &ok);
      if (!ok) {  // the thread has exited
        t.dead = true;
        continue;
      }
      const uint64_t d = now - t.last_ns;
      t.last_ns = now;
      t.busy_ns += d;
      const double u = double(d) / double(kIntervalNs);
      const int b = u < 0.10 ? 0 : u < 0.25 ? 1 : u < 0.50 ? 2 : u < 0.75 ? 3 : u < 0.90 ? 4 : 5;
      t.hist[b]++;
    }
  }
}
}  // namespace timeline

bool start_timeline_from_env() {
  const char* p = getenv("TUNNEL_THREAD_TIMELINE");
  if (!p || !*p || timeline::on.load()) return false;
  timeline::path = p;
  if (size_t at = timeline::path.find("%p"); at != std::string::npos)
    timeline::path.replace(at, 2, std::to_string(getpid()));
  timeline::on.store(true);
  timeline::add_self(0);
  std::thread(timeline::run).detach();
  atexit(timeline::write_out);
  return true;
}

void register_thread(int tag) {
  t_tag = uint64_t(tag);
  if (tag != 0) affinity::pin_this_thread(tag);
  if (timeline::on.load(std::memory_order_relaxed)) timeline::add_self(tag);
  pthread_attr_t attr;
  if (pthread_getattr_np(pthread_self(), &attr) == 0) {
    void* lo = nullptr;
    size_t sz = 0;
    pthread_attr_getstack(&attr, &lo, &sz);
    t_stack_lo = reinterpret_cast<uintptr_t>(lo);
    t_stack_hi = t_stack_lo + sz;
    pthread_attr_destroy(&attr);
  }
  t_timer.arm();
}

bool start_from_env() {
  const char* p = getenv("TUNNEL_PROFILE");
  if (!p || !*p) return false;
  g_path = p;
  int hz = 2000;
  if (size_t at = g_path.rfind('@'); at != std::string::npos) {  // PATH@HZ
    hz = std::min(20000, std::max(10, atoi(g_path.c_str() + at + 1)));
    g_path.resize(at);
  }
  if (size_t at = g_path.find("%p"); at != std::string::npos) g_path.replace(at, 2, std::to_string(getpid()));
  g_slots = new Slot[kSlots];
  // Resolve dladdr's lazy state before the first signal.
  Dl_info di;
  dladdr(reinterpret_cast<void*>(&start_from_env), &di);
  struct sigaction sa = {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  g_hz = hz;
  register_thread(0);  // the main reactor; other threads arm theirs in register_thread()
  atexit(dump);
  return true;
}

void dump() {
  if (!g_slots || g_dumped.exchange(true)) return;
  g_hz = 0;  // late samples still land in the table; the dump below reads it once
  FILE* f = fopen(g_path.c_str(), "w");
  if (!f) return;
  fprintf(f, "# samples %llu dropped %llu\n", static_cast<unsigned long long>(g_samples.load()),
          static_cast<unsigned long long>(g_dropped.load()));
  for (size_t i = 0; i < kSlots; i++) {
    Slot& s = g_slots[i];
    if (!s.hash.load()) continue;
    fprintf(f, "%llu T%llu", static_cast<unsigned long long>(s.count.load()), static_cast<unsigned long long>(s.tag));
    for (int k = 0; k < kDepth && (k < 2 || s.pcs[k]); k++) resolve(f, s.pcs[k]);
    fputc('\n', f);
  }
  fclose(f);
}

}  // namespace p2pt::profiler
