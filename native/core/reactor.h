// Single-threaded run-to-completion epoll reactor.
//
// Replaces tokio (reference tunnel/Cargo.toml:7) and the reference's web of
// spawned tasks + unbounded mpsc channels (reference proxy.rs:106-172,
// :391-419; serve.rs:68-80, :131-137): every connection, stream and timer is
// a callback on one thread, so the tunnel hot path has no locks and no
// cross-thread hand-offs.
//
// Flush hooks run once after every batch of ready events, before the next
// epoll_wait. Transports use them to coalesce everything produced in one
// batch (SCTP bundling, sendmmsg, SACK-per-batch) without adding latency.
#pragma once

#include <cstdint>
#include <deque>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace p2pt {

using Fn = std::function<void()>;

class Reactor {
 public:
  using IoFn = std::function<void(uint32_t events)>;
  using TimerId = uint64_t;

  Reactor();
  ~Reactor();
  Reactor(const Reactor&) = delete;
  Reactor& operator=(const Reactor&) = delete;

  // The reactor that is running on this thread (or nullptr).
  static Reactor* current();

  // fd registration; events are EPOLLIN/EPOLLOUT/... masks.
  void add(int fd, uint32_t events, IoFn cb);
  void modify(int fd, uint32_t events);
  void remove(int fd);
  bool watching(int fd) const { return fds_.count(fd) != 0; }

  // Timers (monotonic microseconds).
  TimerId call_at(uint64_t when_us, Fn fn);
  TimerId call_later_ms(uint64_t ms, Fn fn) { return call_at(now_us() + ms * 1000, std::move(fn)); }
  TimerId call_later_us(uint64_t us, Fn fn) { return call_at(now_us() + us, std::move(fn)); }
  void cancel(TimerId id);

  // Deferred work on this thread (runs before the next epoll_wait).
  void post(Fn fn);
  // Thread-safe variant (wakes the loop through an eventfd).
  void post_threadsafe(Fn fn);
  // Hook that runs after each event batch; returns an id for removal.
  uint64_t add_flush_hook(Fn fn);
  void remove_flush_hook(uint64_t id);
  // Latency-critical work was just queued (a request, the start of a
  // response): run posted work and the flush hooks as soon as the current
  // callback returns instead of after the rest of this turn's events — on a
  // loaded loop a turn of token work took 0.5-1.8 ms (profiles/r05/b13).
  // flushing_soon(): inside such an early flush (transports send what they
  // hold instead of coalescing it). Only while the loop is not saturated
  // (lightly_loaded()): a saturated loop would pay a flush's syscalls per
  // request, and the node row's job then spent more time throttled at its CPU
  // quota than it saved (profiles/r05/b14/node).
  void flush_soon() {
    if (lightly_loaded()) flush_soon_ = true;
  }
  // Below half busy over the last load window: latency shortcuts (early
  // flushes, urgent hand-offs, busy polling) pay for themselves.
  static constexpr double kLightLoad = 0.5;
  bool lightly_loaded() const { return load() < kLightLoad; }
  bool flushing_soon() const { return soon_active_; }

  // SIGINT/SIGTERM etc. delivered via signalfd on the loop thread.
  void on_signal(int signo, Fn fn);

  void run();
  // Run until pred() is true or the timeout passes; returns pred().
  bool run_until(const std::function<bool()>& pred, uint64_t timeout_ms);
  void stop() { stop_ = true; }
  bool stopped() const { return stop_; }
  // Adaptive busy polling: after any I/O event keep polling epoll without
  // sleeping for `us` microseconds before blocking again, within a budget of
  // 10 % of a core. Cuts the wake-up latency out of each hop of a token's
  // path (0 = always block).
  void set_busy_poll_us(uint64_t us) { busy_poll_us_ = us; }
  // Share of wall time this loop spent outside epoll_wait over the last
  // window of >= 2 ms (0..1): lets a transport move work off a saturated loop.
  // Any thread may read it (the "assoc" router compares associations' loops).
  double load() const { return load_.load(std::memory_order_relaxed); }

  static uint64_t now_us();
  static uint64_t now_ms() { return now_us() / 1000; }
  // Virtual time (tests of emulated links): while on, now_us() reads a
  // process-wide virtual clock, and a loop with nothing ready and nothing
  // posted jumps that clock to its next timer (or run_until deadline) instead
  // of sleeping. An in-process link emulator driven by timers then runs
  // deterministically, at any machine load, and faster than real time. Only
  // for single-threaded test reactors without real I/O to wait for.
  static void set_virtual_time(bool on);
  static bool virtual_time();

 private:
  void run_once(int64_t timeout_us);
  int64_t next_timeout_us() const;
  void run_timers();
  void run_posted();
  void run_flush();
  void maybe_flush_soon() {
    if (!flush_soon_) return;
    flush_soon_ = false;
    soon_active_ = true;
    run_posted();
    run_flush();
    soon_active_ = false;
  }

  struct FdEntry {
    uint64_t gen;
    std::shared_ptr<IoFn> cb;
  };
  int epfd_ = -1;
  int evfd_ = -1;
  int sigfd_ = -1;
  bool stop_ = false;
  uint64_t busy_poll_us_ = 0;
  uint64_t last_io_us_ = 0;
  uint64_t win_start_us_ = 0, win_busy_us_ = 0, wake_us_ = 0;
  bool idle_turn_ = false;  // the last turn was an empty busy-polling one
  bool flush_soon_ = false, soon_active_ = false;
  // Busy polling may use at most kSpinBudgetUs of every kSpinWindowUs (10 % of
  // a core): sparse traffic (a token every few ms) polls through every gap
  // that matters, dense traffic sleeps between events as without polling.
  static constexpr uint64_t kSpinWindowUs = 10000, kSpinBudgetUs = 1000;
  uint64_t spin_win_start_us_ = 0, spin_win_used_us_ = 0;
  std::atomic<double> load_{0.0};
  uint64_t gen_ = 1;
  std::unordered_map<int, FdEntry> fds_;
  std::multimap<uint64_t, TimerId> timer_order_;
  std::unordered_map<TimerId, std::pair<uint64_t, Fn>> timers_;
  TimerId next_timer_ = 1;
  std::deque<Fn> posted_;
  std::mutex ts_mu_;
  std::vector<Fn> ts_posted_;
  // post_threadsafe() skips the eventfd write while this loop is awake: it
  // looks at ts_pending_ itself before it sleeps and after every wait. Both
  // flags are sequentially consistent (poster: set pending, read sleeping;
  // loop: set sleeping, read pending), so one of the two sides always sees
  // the other and no post is left waiting behind a sleep.
  std::atomic<bool> sleeping_{false}, ts_pending_{false};
  void run_threadsafe_posts();
  std::vector<std::pair<uint64_t, Fn>> flush_hooks_;
  uint64_t next_hook_ = 1;
  std::unordered_map<int, Fn> signals_;
};

}  // namespace p2pt
