#include "core/reactor.h"

#include <signal.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/signalfd.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace p2pt {

namespace {
thread_local Reactor* t_current = nullptr;
constexpr uint64_t kWakeTag = ~uint64_t(0);
constexpr uint64_t kSigTag = ~uint64_t(0) - 1;
}  // namespace

Reactor* Reactor::current() { return t_current; }

Reactor::Reactor() {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  if (epfd_ < 0) throw std::runtime_error("epoll_create1 failed");
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = kWakeTag;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
}

Reactor::~Reactor() {
  if (sigfd_ >= 0) close(sigfd_);
  if (evfd_ >= 0) close(evfd_);
  if (epfd_ >= 0) close(epfd_);
  if (t_current == this) t_current = nullptr;
}

namespace {
std::atomic<uint64_t> g_virtual_us{0};  // 0: real time

uint64_t real_now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000u + uint64_t(ts.tv_nsec) / 1000u;
}
}  // namespace

uint64_t Reactor::now_us() {
  const uint64_t v = g_virtual_us.load(std::memory_order_relaxed);
  return v ? v : real_now_us();
}

void Reactor::set_virtual_time(bool on) { g_virtual_us.store(on ? real_now_us() : 0, std::memory_order_relaxed); }

bool Reactor::virtual_time() { return g_virtual_us.load(std::memory_order_relaxed) != 0; }

// epoll data carries (generation << 32 | fd) so an event queued for an fd that
// was removed (and possibly reused) within the same batch is ignored.
void Reactor::add(int fd, uint32_t events, IoFn cb) {
  uint64_t g = gen_++;
  fds_[fd] = FdEntry{g, std::make_shared<IoFn>(std::move(cb))};
  epoll_event ev{};
  ev.events = events;
  ev.data.u64 = (g << 32) | uint32_t(fd);
  if (epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev) < 0) {
    if (errno == EEXIST) epoll_ctl(epfd_, EPOLL_CTL_MOD, fd, &ev);
    else throw std::runtime_error(std::string("epoll_ctl add: ") + strerror(errno));
  }
}

void Reactor::modify(int fd, uint32_t events) {
  auto it = fds_.find(fd);
  if (it == fds_.end()) return;
  epoll_event ev{};
  ev.events = events;
  ev.data.u64 = (it->second.gen << 32) | uint32_t(fd);
  epoll_ctl(epfd_, EPOLL_CTL_MOD, fd, &ev);
}

void Reactor::remove(int fd) {
  if (fds_.erase(fd)) epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr);
}

Reactor::TimerId Reactor::call_at(uint64_t when_us, Fn fn) {
  TimerId id = next_timer_++;
  timers_.emplace(id, std::make_pair(when_us, std::move(fn)));
  timer_order_.emplace(when_us, id);
  return id;
}

void Reactor::cancel(TimerId id) {
  auto it = timers_.find(id);
  if (it == timers_.end()) return;
  auto range = timer_order_.equal_range(it->second.first);
  for (auto o = range.first; o != range.second; ++o) {
    if (o->second == id) {
      timer_order_.erase(o);
      break;
    }
  }
  timers_.erase(it);
}

void Reactor::post(Fn fn) { posted_.push_back(std::move(fn)); }

void Reactor::post_threadsafe(Fn fn) {
  bool wake;
  {
    std::lock_guard<std::mutex> lk(ts_mu_);
    // The loop drains the eventfd before it takes the whole queue, so only the
    // push into an empty queue needs to wake it: posts that land while a batch
    // is still waiting ride along without a syscall.
    wake = ts_posted_.empty();
    ts_posted_.push_back(std::move(fn));
    ts_pending_.store(true, std::memory_order_seq_cst);
  }
  // A loop that is awake picks the queue up before it sleeps (run_once): no
  // eventfd write (a syscall per hand-off between busy threads: 8 % of the
  // proxy's association thread on the 1200-MTU download, profiles/r05/b11).
  if (!wake || !sleeping_.load(std::memory_order_seq_cst)) return;
  uint64_t one = 1;
  ssize_t r = write(evfd_, &one, sizeof one);
  (void)r;
}

void Reactor::run_threadsafe_posts() {
  std::vector<Fn> fns;
  {
    std::lock_guard<std::mutex> lk(ts_mu_);
    fns.swap(ts_posted_);
    ts_pending_.store(false, std::memory_order_relaxed);
  }
  for (auto& f : fns) {
    f();
    maybe_flush_soon();
  }
}

uint64_t Reactor::add_flush_hook(Fn fn) {
  uint64_t id = next_hook_++;
  flush_hooks_.emplace_back(id, std::move(fn));
  return id;
}

void Reactor::remove_flush_hook(uint64_t id) {
  for (auto& h : flush_hooks_)
    if (h.first == id) h.second = nullptr;  // compacted in run_flush
}

void Reactor::on_signal(int signo, Fn fn) {
  signals_[signo] = std::move(fn);
  sigset_t mask;
  sigemptyset(&mask);
  for (auto& s : signals_) sigaddset(&mask, s.first);
  sigprocmask(SIG_BLOCK, &mask, nullptr);
  if (sigfd_ < 0) {
    sigfd_ = signalfd(-1, &mask, SFD_NONBLOCK | SFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kSigTag;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, sigfd_, &ev);
  } else {
    signalfd(sigfd_, &mask, SFD_NONBLOCK | SFD_CLOEXEC);
  }
}

int64_t Reactor::next_timeout_us() const {
  if (!posted_.empty()) return 0;
  if (timer_order_.empty()) return 1000000;
  uint64_t now = now_us();
  uint64_t when = timer_order_.begin()->first;
  if (when <= now) return 0;
  return int64_t(std::min<uint64_t>(when - now, 1000000));
}

void Reactor::run_timers() {
  uint64_t now = now_us();
  while (!timer_order_.empty() && timer_order_.begin()->first <= now) {
    TimerId id = timer_order_.begin()->second;
    timer_order_.erase(timer_order_.begin());
    auto it = timers_.find(id);
    if (it == timers_.end()) continue;
    Fn fn = std::move(it->second.second);
    timers_.erase(it);
    fn();
  }
}

void Reactor::run_posted() {
  // Bounded: work posted by posted work runs in the next iteration.
  size_t n = posted_.size();
  for (size_t i = 0; i < n && !posted_.empty(); i++) {
    Fn fn = std::move(posted_.front());
    posted_.pop_front();
    fn();
  }
}

void Reactor::run_flush() {
  // Hooks may register/remove hooks; iterate by index over a stable count.
  size_t n = flush_hooks_.size();
  for (size_t i = 0; i < n; i++) {
    if (flush_hooks_[i].second) {
      Fn f = flush_hooks_[i].second;  // copy: hook may remove itself
      f();
    }
  }
  size_t w = 0;
  for (size_t i = 0; i < flush_hooks_.size(); i++)
    if (flush_hooks_[i].second) flush_hooks_[w++] = std::move(flush_hooks_[i]);
  flush_hooks_.resize(w);
}

// Microsecond timeouts (epoll_pwait2): a timer due in 50 us must not sleep
// for epoll_wait's whole millisecond.
static int wait_events(int epfd, epoll_event* evs, int max, int64_t timeout_us) {
  static bool pwait2 = true;
  if (timeout_us > 0 && pwait2) {
    timespec ts{time_t(timeout_us / 1000000), long(timeout_us % 1000000) * 1000};
    int n = epoll_pwait2(epfd, evs, max, &ts, nullptr);
    if (n >= 0 || errno != ENOSYS) return n;
    pwait2 = false;
  }
  return epoll_wait(epfd, evs, max, timeout_us <= 0 ? 0 : int((timeout_us + 999) / 1000));
}

// Ready descriptors taken per turn. 64 (shorter turns, earlier flushes and
// hand-offs) looked better on one box's node row (profiles/r05/b27) and worse
// on two others (b28, b29: 1024-stream p99 11.2 -> 15.6 ms, download 0.235 ->
// 0.203 of direct).
constexpr int kMaxEvents = 256;

void Reactor::run_once(int64_t timeout_us) {
  epoll_event evs[kMaxEvents];
  bool spin = false;
  const uint64_t t_wait = now_us();
  if (busy_poll_us_) {
    if (t_wait - spin_win_start_us_ >= kSpinWindowUs) {
      spin_win_start_us_ = t_wait;
      spin_win_used_us_ = 0;
    }
    // Within the window's spin budget only: a loop woken every few
    // microseconds (the node row, 1024 streams of 1 ms tokens) would
    // otherwise poll through all its idle time — 4.8 cores per tunnel process
    // against 1.1-1.7 sleeping, and the job's CPU quota throttled
    // (profiles/r05/b07 node).
    // Not on a saturated loop either: it rarely sleeps, so polling buys it
    // little latency, and at node scale its polling turns were CPU the job's
    // quota did not have (profiles/r05/b14/node).
    if (timeout_us > 0 && t_wait - last_io_us_ < busy_poll_us_ && spin_win_used_us_ < kSpinBudgetUs &&
        lightly_loaded()) {
      timeout_us = 0;
      spin = true;
    }
  }
  // An empty polling turn is idle time, not load (a transport reads load() to
  // decide whether to hold small flushes: counting the spin would make every
  // polling loop look half busy).
  if (wake_us_ && !idle_turn_) win_busy_us_ += t_wait - wake_us_;
  if (t_wait - win_start_us_ >= 2000) {
    load_.store(win_start_us_ ? double(win_busy_us_) / double(t_wait - win_start_us_) : 0.0, std::memory_order_relaxed);
    win_start_us_ = t_wait;
    win_busy_us_ = 0;
  }
  if (ts_pending_.load(std::memory_order_acquire)) timeout_us = 0;
  if (timeout_us != 0) {
    sleeping_.store(true, std::memory_order_seq_cst);
    if (ts_pending_.load(std::memory_order_seq_cst)) timeout_us = 0;  // posted as we decided to sleep
  }
  const bool virt = virtual_time();
  int n = wait_events(epfd_, evs, kMaxEvents, virt ? 0 : timeout_us);
  sleeping_.store(false, std::memory_order_relaxed);
  if (virt && n == 0 && timeout_us > 0 && posted_.empty() && !ts_pending_.load(std::memory_order_acquire)) {
    // Nothing to do before the next timer (or the caller's deadline): that
    // much virtual time passes at once.
    g_virtual_us.fetch_add(uint64_t(timeout_us), std::memory_order_relaxed);
  }
  if (n < 0 && errno != EINTR) throw std::runtime_error(std::string("epoll_wait: ") + strerror(errno));
  wake_us_ = now_us();
  if (wake_us_ - win_start_us_ >= 2000 && win_start_us_) {  // a long sleep ends the window idle
    load_.store(double(win_busy_us_) / double(wake_us_ - win_start_us_), std::memory_order_relaxed);
    win_start_us_ = wake_us_;
    win_busy_us_ = 0;
  }
  if (n > 0 && busy_poll_us_) last_io_us_ = now_us();
  // Nothing ready, no timer due and nothing posted: no hook has new work.
  idle_turn_ = spin && n <= 0 && posted_.empty() && !ts_pending_.load(std::memory_order_acquire) &&
               (timer_order_.empty() || timer_order_.begin()->first > wake_us_);
  if (idle_turn_) {
    spin_win_used_us_ += wake_us_ - t_wait;
    return;
  }
  for (int i = 0; i < n; i++) {
    uint64_t tag = evs[i].data.u64;
    if (tag == kWakeTag) {
      uint64_t v;
      ssize_t rd = read(evfd_, &v, sizeof v);  // one read resets the counter
      (void)rd;
      run_threadsafe_posts();
      continue;
    }
    if (tag == kSigTag) {
      signalfd_siginfo si;
      while (read(sigfd_, &si, sizeof si) == sizeof si) {
        auto it = signals_.find(int(si.ssi_signo));
        if (it != signals_.end() && it->second) {
          Fn f = it->second;
          f();
        }
      }
      continue;
    }
    int fd = int(uint32_t(tag));
    uint64_t g = tag >> 32;
    auto it = fds_.find(fd);
    if (it == fds_.end() || it->second.gen != g) continue;
    auto cb = it->second.cb;  // keep alive across the call
    (*cb)(evs[i].events);
    maybe_flush_soon();
  }
  if (ts_pending_.load(std::memory_order_acquire)) run_threadsafe_posts();  // posted while awake: no eventfd
  run_timers();
  run_posted();
  flush_soon_ = false;
  run_flush();
}

void Reactor::run() {
  Reactor* prev = t_current;
  t_current = this;
  stop_ = false;
  while (!stop_) run_once(next_timeout_us());
  t_current = prev;
}

bool Reactor::run_until(const std::function<bool()>& pred, uint64_t timeout_ms) {
  Reactor* prev = t_current;
  t_current = this;
  uint64_t deadline = now_us() + timeout_ms * 1000;
  stop_ = false;
  while (!stop_ && !pred()) {
    uint64_t now = now_us();
    if (now >= deadline) break;
    int64_t t = next_timeout_us();
    int64_t left = int64_t(deadline - now);
    run_once(t < left ? t : left);
  }
  t_current = prev;
  return pred();
}

}  // namespace p2pt
