#include "tunnel/workers.h"

#include "core/affinity.h"

#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <future>

#include "core/profiler.h"

namespace p2pt {

WorkerThread::WorkerThread(int index, uint64_t busy_poll_us, const char* name_prefix, int tag) : index_(index) {
  std::promise<Reactor*> ready;
  auto fut = ready.get_future();
  // The reactor is created on its own thread so thread-affine state (the
  // thread_local current reactor) belongs to that thread.
  th_ = std::thread([this, &ready, busy_poll_us, name_prefix, tag] {
    // Process signals (Ctrl-C, SIGTERM) belong to the main reactor's signalfd;
    // a worker must never take them with the default action. SIGPROF stays
    // open so the sampling profiler sees worker time too.
    sigset_t mask;
    sigemptyset(&mask);
    for (int sig : {SIGINT, SIGTERM, SIGHUP, SIGQUIT, SIGUSR1, SIGUSR2, SIGPIPE}) sigaddset(&mask, sig);
    pthread_sigmask(SIG_BLOCK, &mask, nullptr);
    auto r = std::make_unique<Reactor>();
    r->set_busy_poll_us(busy_poll_us);
    Reactor* rp = r.get();
    r_ = std::move(r);
    char name[16];
    snprintf(name, sizeof name, "%s%d", name_prefix, index_);
    pthread_setname_np(pthread_self(), name);
    profiler::register_thread(tag < 0 ? index_ : tag);
    ready.set_value(rp);
    rp->run();
  });
  fut.get();
}

WorkerThread::~WorkerThread() {
  Reactor* r = r_.get();
  r->post_threadsafe([r] { r->stop(); });
  th_.join();
  // Work posted by sessions torn down in the meantime (their last references
  // to worker-side state) still has to run: drain it here.
  r_->run_until([] { return false; }, 20);
}

// Half the CPUs the process may use less one (the association thread, the
// TX seal and send stages and the socket reader take the rest), 1..4:
// measured on the MI355X host (bench/bench_node.py, profiles/node_r02/), 4
// workers carried 1024 1 ms-token streams at direct speed while 8 lost to
// contention with the association thread. One worker per 4 CPUs (round 3)
// gave a process pinned to 6 CPUs a single worker, which then saturated on
// the 64 x 1 MB echo (all 64 upstream sockets' I/O; profiles/r04/flow_ab).
int WorkerPool::auto_count() {
  long n = affinity::process_cpu_count();  // the set from before this thread pinned itself to one CPU
  if (n <= 0) n = sysconf(_SC_NPROCESSORS_ONLN);
  // One CPU per thread (affinity.h): the association thread, the socket
  // reader, the RX lane and the two TX stages take five, from 8 CPUs the two
  // open lanes two more, the workers the rest. On 6 CPUs one worker beat two
  // on the 64 x 1 MB echo (1916 vs 1633 req/s at 1200 MTU, 1920 vs 1876
  // jumbo, same box; profiles/r04/w24).
  if (affinity::enabled()) return int(std::clamp<long>(n >= 8 ? n - 7 : n - 5, 1, 4));
  return int(std::clamp<long>(n / 2 - 1, 1, 4));
}

WorkerPool::WorkerPool(int n, uint64_t busy_poll_us) {
  if (n < 0) n = auto_count();
  for (int i = 0; i < n; i++) threads_.push_back(std::make_unique<WorkerThread>(i + 1, busy_poll_us));
}

WorkerPool::~WorkerPool() = default;

}  // namespace p2pt
