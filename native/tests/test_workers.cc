// Worker-thread plumbing (tunnel/workers.h) and the scheduler's lanes
// (tunnel/scheduler.h).
#include <atomic>
#include <thread>

#include "tests/testing.h"
#include "tunnel/scheduler.h"
#include "tunnel/workers.h"

using namespace p2pt;

// Messages pushed on one reactor thread arrive on another in push order,
// batched per loop iteration, and stop once the pipe is closed.
TEST(pipe_orders_messages_across_threads) {
  WorkerPool pool(1);
  Reactor main;
  std::vector<int> got;
  std::mutex mu;
  std::atomic<int> n{0};
  auto pipe = std::make_unique<Pipe<int>>(main, pool.reactor(0), [&](int& v) {
    std::lock_guard<std::mutex> lk(mu);
    got.push_back(v);
    n++;
  });
  CHECK(!pipe->same_thread());
  int pushed = 0;
  for (int round = 0; round < 50; round++) {
    main.post([&] {
      for (int k = 0; k < 100; k++) pipe->push(pushed++);
    });
    main.run_until([] { return false; }, 1);
  }
  main.run_until([&] { return n.load() == 5000; }, 5000);
  CHECK_EQ(n.load(), 5000);
  {
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < int(got.size()); i++)
      if (got[size_t(i)] != i) {
        CHECK(false);
        break;
      }
  }
  pipe->close();
  main.post([&] { pipe->push(-1); });
  main.run_until([] { return false; }, 20);
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  CHECK_EQ(n.load(), 5000);
  pipe.reset();
}

TEST(pipe_same_thread_is_synchronous) {
  Reactor r;
  int sum = 0;
  Pipe<int> p(r, r, [&](int& v) { sum += v; });
  CHECK(p.same_thread());
  p.push(3);
  p.push(4);
  CHECK_EQ(sum, 7);
}

// Streams stay on the association thread up to the inline limit, then go to
// the least-loaded worker; releases make room again.
TEST(placement_inline_then_least_loaded) {
  Placement pl(4, 2);
  CHECK_EQ(pl.pick(), size_t(0));
  CHECK_EQ(pl.pick(), size_t(0));
  size_t a = pl.pick(), b = pl.pick(), c = pl.pick();
  CHECK(a != 0 && b != 0 && c != 0 && a != b && b != c && a != c);
  size_t d = pl.pick();
  CHECK(d != 0);
  CHECK_EQ(pl.active(d), size_t(2));
  pl.release(0);
  CHECK_EQ(pl.pick(), size_t(0));
  Placement single(1, 0);
  CHECK_EQ(single.pick(), size_t(0));
  CHECK_EQ(single.pick(), size_t(0));
}

namespace {
// A channel that accepts at most `room` bytes until drained by the test.
struct FakeChannel : MessageChannel {
  size_t buffered = 0, room = 0;
  std::vector<std::pair<uint32_t, size_t>> sent;  // (stream, payload bytes)
  bool send(const uint8_t* hdr, size_t, const Bytes& payload) override {
    sent.emplace_back(rd32(hdr + 1), payload.size());
    buffered += 5 + payload.size();
    return true;
  }
  size_t buffered_amount() const override { return buffered; }
  bool is_open() const override { return true; }
  void close() override {}
  std::string describe() const override { return "fake"; }
};
}  // namespace

// With the channel busy, a stream with a small backlog (an SSE token) is
// released before streams with large backlogs, and per-stream order holds.
TEST(scheduler_interactive_lane_goes_first) {
  auto ch = std::make_shared<FakeChannel>();
  FrameScheduler s(ch, 1000);
  ch->buffered = 5000;  // channel full: everything queues
  Bytes big = Bytes::copy(std::string(60000, 'b'));
  for (int i = 0; i < 4; i++) s.send(proto::make_body(proto::MsgType::ResBody, 1, big));
  for (int i = 0; i < 4; i++) s.send(proto::make_body(proto::MsgType::ResBody, 2, big));
  s.send(proto::make_body(proto::MsgType::ResBody, 3, Bytes::copy(std::string(150, 't'))));
  s.send(proto::make_empty(proto::MsgType::Ping, 0));
  CHECK_EQ(s.stream_queued(1), size_t(4 * 60005));
  CHECK_EQ(s.stream_queued(3), size_t(155));
  CHECK(ch->sent.empty());
  ch->buffered = 0;  // the window (1000 B) admits frames until one bulk frame overshoots it
  s.pump();
  CHECK_EQ(ch->sent.size(), size_t(3));
  CHECK_EQ(ch->sent[0].first, 0u);  // control first
  CHECK_EQ(ch->sent[1].first, 3u);  // then the token, ahead of both bulk streams
  CHECK(ch->sent[2].first == 1u || ch->sent[2].first == 2u);
  CHECK_EQ(s.stream_queued(3), size_t(0));
  for (int i = 0; i < 7; i++) {
    ch->buffered = 0;
    s.pump();
  }
  CHECK_EQ(ch->sent.size(), size_t(10));
  for (size_t i = 3; i < 10; i++) CHECK(ch->sent[i].first != ch->sent[i - 1].first);  // bulk streams alternate
  CHECK_EQ(s.queued_bytes(), size_t(0));
}
