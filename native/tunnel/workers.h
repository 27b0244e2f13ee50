// Worker threads for the tunnel roles.
//
// The reference runs on tokio's multi-threaded runtime and spawns a task per
// request (reference tunnel/src/main.rs:18, serve.rs:131-137, proxy.rs:196-217),
// so HTTP parsing and socket I/O for many streams spread over all cores. Here
// the association thread owns the one thing that must stay ordered — the data
// channel (ICE/DTLS/SCTP, the frame scheduler, the stream table) — and the
// per-stream HTTP work (upstream calls on serve, client connections on proxy:
// one read or write syscall per SSE token) runs on worker reactors:
//
//   serve:  channel -> [assoc] --Start/Cancel/Pause--> [worker k] -> upstream
//           upstream -> [worker k] --frames (RES_*), Done--> [assoc] -> channel
//   proxy:  client -> [worker k] --Route, frames (REQ_*)--> [assoc] -> channel
//           channel -> [assoc] --RES_* by stream id--> [worker k] -> client
//
// Streams start on the association thread itself (no hand-off latency) and
// only spill onto workers once more than `inline_streams` are active, so low
// concurrency keeps the single-thread TTFT and node-scale load uses the cores.
//
// Threads talk through Pipe<M>: an ordered queue from one reactor's thread to
// another's, batched per event-loop iteration (one lock + one eventfd write per
// batch, whatever the number of frames). Frame payloads are refcounted Bytes
// views, so crossing a thread never copies a body.
#pragma once

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_set>
#include <thread>
#include <vector>

#include "core/buf.h"
#include "core/reactor.h"

namespace p2pt {

// A Reactor running on its own thread until destroyed.
class WorkerThread {
 public:
  // `name`: thread name prefix (index appended); `tag`: profiler / affinity
  // role (core/affinity.h), -1 = the index (an HTTP worker).
  explicit WorkerThread(int index, uint64_t busy_poll_us = 0, const char* name = "p2pt-w", int tag = -1);
  ~WorkerThread();
  Reactor& reactor() { return *r_; }
  int index() const { return index_; }

 private:
  int index_;
  std::unique_ptr<Reactor> r_;
  std::thread th_;
};

// The process's worker threads; they outlive sessions (reconnects reuse them).
class WorkerPool {
 public:
  // n < 0: auto_count(). busy_poll_us: Reactor::set_busy_poll_us of each.
  explicit WorkerPool(int n, uint64_t busy_poll_us = 0);
  ~WorkerPool();
  size_t size() const { return threads_.size(); }
  Reactor& reactor(size_t i) { return threads_[i]->reactor(); }
  static int auto_count();

 private:
  std::vector<std::unique_ptr<WorkerThread>> threads_;
};

// Ordered, batched messages from the thread of `src` to the thread of `dst`.
// push() runs on src's thread; the sink runs on dst's thread, once per message,
// in push order. When src == dst the sink runs synchronously inside push().
// The Pipe itself must be destroyed on src's thread (it owns a flush hook
// there); messages still queued are delivered unless the pipe was close()d.
template <class M>
class Pipe {
 public:
  using Sink = std::function<void(M&)>;
  Pipe(Reactor& src, Reactor& dst, Sink sink)
      : src_(src), dst_(dst), state_(std::make_shared<State>()) {
    state_->sink = std::move(sink);
    if (&src != &dst) {
      std::weak_ptr<State> w = state_;
      Reactor* d = &dst_;
      hook_ = src_.add_flush_hook([w, d] {
        if (auto st = w.lock()) send(st, *d);
      });
    }
  }
  ~Pipe() {
    if (hook_) src_.remove_flush_hook(hook_);
  }
  Pipe(const Pipe&) = delete;
  Pipe& operator=(const Pipe&) = delete;

  // urgent: hand over what is queued now instead of at the end of src's loop
  // turn — a request or the start of a response must not wait behind a loaded
  // thread's whole turn of token work (node row, 1024 streams: 0.5-1.8 ms p50
  // per crossing between the association thread and a worker,
  // profiles/r05/b13/node_trace.json).
  void push(M m, bool urgent = false) {
    if (state_->closed) return;
    if (!hook_) {
      state_->sink(m);
      return;
    }
    state_->buf.push_back(std::move(m));
    if (urgent && src_.lightly_loaded()) send(state_, dst_);  // a saturated src batches (Reactor::flush_soon)
  }
  // A small payload for a message of this pipe, copied into the current
  // batch's own arena (src thread). The arena's reference count is updated by
  // src while the batch fills and by dst after it: one cache-line transfer per
  // batch. A view of a buffer that both threads keep referencing — a slab of
  // token copies the association thread fills while workers release earlier
  // tokens of it — moves that line once per message each way: 1 ms tokens at
  // 1024 streams had the association threads spend ~30 % (proxy) and ~10 %
  // (serve) of their time in such updates (profiles/r05/b11/nodeprof).
  Bytes stage(const Bytes& b) {
    if (!hook_ || b.empty() || b.size() > kStageMax) return b;
    State& st = *state_;
    if (!st.arena || st.arena_off + b.size() > kArena) {
      st.arena = st.arenas.get();
      st.arena_off = 0;
    }
    uint8_t* d = st.arena->data.get() + st.arena_off;
    memcpy(d, b.data(), b.size());
    st.arena_off += (b.size() + 15) & ~size_t(15);
    return Bytes::adopt(st.arena, d, b.size());
  }
  static constexpr size_t kStageMax = 2048, kArena = 32 * 1024;
  // Stop delivering (also batches already posted). src thread only; the flag
  // is read on dst's thread, so it is atomic.
  void close() { state_->closed = true; }
  bool same_thread() const { return hook_ == 0; }
  Reactor& dst() const { return dst_; }

 private:
  struct State;
  static void send(const std::shared_ptr<State>& st, Reactor& d) {
    if (st->buf.empty()) return;
    auto batch = std::make_shared<std::vector<M>>(std::move(st->buf));
    st->buf.clear();
    st->buf.reserve(batch->size());
    st->arena.reset();  // the next batch stages into another one
    d.post_threadsafe([st, batch] {
      if (st->closed) return;
      for (auto& m : *batch) st->sink(m);
    });
  }
  struct State {
    Sink sink;
    std::vector<M> buf;  // src thread only
    std::atomic<bool> closed{false};
    BufPool arenas{kArena, 64};  // stage(): src thread only
    RawBufPtr arena;
    size_t arena_off = 0;
  };
  Reactor& src_;
  Reactor& dst_;
  std::shared_ptr<State> state_;
  uint64_t hook_ = 0;
};

// Picks the thread for a new stream/connection: the association thread
// (index 0) while fewer than `inline_max` are active there, otherwise the
// least-loaded worker (ties round-robin). A stream known to be bulk (a large
// request body) always goes to a worker when there is one: its socket I/O
// would otherwise take the association thread's time from every other stream.
class Placement {
 public:
  static constexpr uint64_t kBulkBytes = 256 * 1024;
  Placement(size_t threads, size_t inline_max) : active_(threads, 0), inline_max_(inline_max) {}
  size_t pick(bool bulk = false) {
    size_t n = active_.size(), best = 0;
    if (n > 1 && (bulk || active_[0] >= inline_max_)) {
      best = 1 + rr_ % (n - 1);
      for (size_t k = 0; k + 1 < n; k++) {
        size_t i = 1 + (rr_ + k) % (n - 1);
        if (active_[i] < active_[best]) best = i;
      }
      rr_ = best;
    }
    active_[best]++;
    return best;
  }
  void release(size_t i) {
    if (i < active_.size() && active_[i]) active_[i]--;
  }
  size_t active(size_t i) const { return active_[i]; }
  size_t threads() const { return active_.size(); }

 private:
  std::vector<size_t> active_;
  size_t inline_max_;
  size_t rr_ = 0;
};

// Routes (method + path, query dropped) whose last response was bulk. A
// download's size is unknown when its request arrives, so Placement cannot
// send it to a worker up front the way it does a large upload; the first
// response of a route teaches it instead, and later requests to that route go
// to a worker (serve) or move their client connection to one (proxy). Streamed
// responses (SSE, NDJSON) never count as bulk, however long: they are the
// interactive traffic the association thread keeps close. One per thread.
class BulkRoutes {
 public:
  static std::string key(std::string_view method, std::string_view path) {
    const size_t q = path.find('?');
    std::string k(method);
    k += ' ';
    k.append(path.substr(0, q));
    return k;
  }
  static bool streaming_type(std::string_view ctype) {
    return ctype.find("event-stream") != std::string_view::npos || ctype.find("ndjson") != std::string_view::npos;
  }
  bool bulk(const std::string& k) const { return !m_.empty() && m_.count(k) != 0; }
  void note(const std::string& k, uint64_t bytes, bool streaming) {
    if (bytes >= Placement::kBulkBytes && !streaming) {
      if (m_.size() >= kMax) m_.clear();
      m_.insert(k);
    } else if (!m_.empty()) {
      m_.erase(k);
    }
  }

 private:
  static constexpr size_t kMax = 256;
  std::unordered_set<std::string> m_;
};

}  // namespace p2pt
