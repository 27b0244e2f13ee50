// Worker-thread plumbing (tunnel/workers.h) and the scheduler's lanes
// (tunnel/scheduler.h).
#include <atomic>
#include <mutex>
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
// stage(): small payloads are copied into an arena owned by the batch being
// filled (a later batch gets another), larger ones and same-thread pipes pass
// through untouched; urgent pushes are handed over before the loop turn ends.
TEST(pipe_stage_copies_small_payloads_per_batch_and_urgent_hands_over) {
  WorkerPool pool(1);
  Reactor main;
  struct Msg {
    Bytes b;
    int i = 0;
  };
  std::mutex mu;
  std::vector<std::pair<int, std::string>> got;
  std::atomic<int> n{0};
  Pipe<Msg> pipe(main, pool.reactor(0), [&](Msg& m) {
    std::lock_guard<std::mutex> lk(mu);
    got.emplace_back(m.i, m.b.str());
    n++;
  });
  std::vector<std::string> sent;
  const void* owner1 = nullptr;
  const void* owner2 = nullptr;
  Bytes keep1;  // holds the first batch's arena, so the pool cannot hand it out again
  Bytes big = Bytes::copy(std::string(Pipe<Msg>::kStageMax + 1, 'x'));
  main.post([&] {
    for (int i = 0; i < 10; i++) {
      sent.push_back("token " + std::to_string(i));
      Bytes src = Bytes::copy(sent.back());
      Bytes st = pipe.stage(src);
      CHECK(st.data() != src.data() && st.str() == sent.back());
      if (i == 0) {
        owner1 = st.owner().get();
        keep1 = st;
      }
      CHECK(st.owner().get() == owner1);  // one arena for the batch
      pipe.push(Msg{st, i});
    }
    Bytes kept = pipe.stage(big);
    CHECK(kept.data() == big.data());  // too large: not copied
  });
  main.run_until([&] { return n.load() == 10; }, 2000);
  main.post([&] {
    Bytes st = pipe.stage(Bytes::copy(std::string("next batch")));
    owner2 = st.owner().get();
    pipe.push(Msg{st, 10}, true);
    // Handed over now: the worker may deliver it before this turn ends.
    sent.push_back("next batch");
  });
  main.run_until([&] { return n.load() == 11; }, 2000);
  CHECK_EQ(n.load(), 11);
  CHECK(owner2 != nullptr && owner2 != owner1);  // a new batch stages into another arena
  std::lock_guard<std::mutex> lk(mu);
  for (size_t i = 0; i < got.size(); i++) CHECK(got[i].first == int(i) && got[i].second == sent[i]);
  Reactor same;
  Pipe<Msg> inline_pipe(same, same, [](Msg&) {});
  Bytes src = Bytes::copy(std::string("inline"));
  CHECK(inline_pipe.stage(src).data() == src.data());  // same thread: nothing to stage
}

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

TEST(bulk_routes_learn_downloads_not_streams) {
  BulkRoutes r;
  const std::string dl = BulkRoutes::key("GET", "/bulk?bytes=67108864");
  CHECK(dl == BulkRoutes::key("GET", "/bulk?bytes=1"));  // the query does not split a route
  CHECK(!r.bulk(dl));
  r.note(dl, 64u << 20, false);
  CHECK(r.bulk(dl));
  CHECK(!r.bulk(BulkRoutes::key("POST", "/bulk")));  // the method is part of the route
  // A long SSE / NDJSON response is interactive however many bytes it carried.
  const std::string chat = BulkRoutes::key("POST", "/v1/chat/completions");
  CHECK(BulkRoutes::streaming_type("text/event-stream; charset=utf-8"));
  CHECK(BulkRoutes::streaming_type("application/x-ndjson"));
  r.note(chat, 8u << 20, true);
  CHECK(!r.bulk(chat));
  // A small answer on a learnt route unlearns it.
  r.note(dl, 1000, false);
  CHECK(!r.bulk(dl));
  // Bounded: past 256 routes the table starts over.
  for (int i = 0; i < 300; i++) r.note(BulkRoutes::key("GET", "/f" + std::to_string(i)), 1u << 20, false);
  CHECK(r.bulk(BulkRoutes::key("GET", "/f299")));
  CHECK(!r.bulk(BulkRoutes::key("GET", "/f0")));
}

namespace {
// A channel that accepts at most `room` bytes until drained by the test.
struct FakeChannel : MessageChannel {
  size_t buffered = 0, room = 0;
  std::vector<std::pair<uint32_t, size_t>> sent;  // (stream, payload bytes)
  size_t urgent = 0;  // messages that came through send_urgent
  bool send(const uint8_t* hdr, size_t, const Bytes& payload) override {
    sent.emplace_back(rd32(hdr + 1), payload.size());
    buffered += 5 + payload.size();
    return true;
  }
  bool send_urgent(const uint8_t* hdr, size_t hlen, const Bytes& payload) override {
    urgent++;
    return send(hdr, hlen, payload);
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
  CHECK_EQ(ch->sent[2].first, 1u);  // then the oldest bulk stream
  CHECK_EQ(s.stream_queued(3), size_t(0));
  for (int i = 0; i < 7; i++) {
    ch->buffered = 0;
    s.pump();
  }
  CHECK_EQ(ch->sent.size(), size_t(10));
  // Within their first kFifoBytes bulk streams go oldest first: stream 1
  // finishes before stream 2 starts.
  for (size_t i = 3; i < 10; i++) CHECK_EQ(ch->sent[i].first, i < 6 ? 1u : 2u);
  CHECK_EQ(s.queued_bytes(), size_t(0));
}

// Interactive bypass: over its window (but under 4 windows) the channel still
// takes a token-sized frame of a stream with nothing queued, through the
// transport's urgent path; frames of streams with a backlog, big frames and
// everything past 4 windows queue as before.
TEST(scheduler_interactive_bypass) {
  auto ch = std::make_shared<FakeChannel>();
  FrameScheduler s(ch, 1000);
  ch->buffered = 2000;  // over the 1000-byte window
  Bytes big = Bytes::copy(std::string(60000, 'b'));
  Bytes tok = Bytes::copy(std::string(150, 't'));
  s.send(proto::make_body(proto::MsgType::ResBody, 1, big));  // queues
  s.send(proto::make_body(proto::MsgType::ResBody, 1, tok));  // behind stream 1's backlog: queues
  s.send(proto::make_body(proto::MsgType::ResBody, 3, tok));  // nothing queued for stream 3: bypass
  CHECK_EQ(ch->sent.size(), size_t(1));
  CHECK_EQ(ch->sent[0].first, 3u);
  CHECK_EQ(ch->urgent, size_t(0));  // one small frame says nothing yet
  s.send(proto::make_body(proto::MsgType::ResBody, 3, tok));  // the stream's second token: the urgent path
  CHECK_EQ(ch->sent.size(), size_t(2));
  CHECK_EQ(ch->urgent, size_t(1));
  s.send(proto::make_empty(proto::MsgType::ResEnd, 3));  // an end frame bypasses, not urgent
  CHECK_EQ(ch->sent.size(), size_t(3));
  CHECK_EQ(ch->urgent, size_t(1));
  CHECK_EQ(s.stream_queued(1), size_t(60005 + 155));
  ch->buffered = 5000;  // past 4 windows: a token queues too
  s.send(proto::make_body(proto::MsgType::ResBody, 4, tok));
  CHECK_EQ(ch->sent.size(), size_t(3));
  CHECK_EQ(s.stream_queued(4), size_t(155));
  ch->buffered = 0;
  for (int i = 0; i < 4; i++) {
    s.pump();
    ch->buffered = 0;
  }
  CHECK_EQ(ch->sent.size(), size_t(6));
  CHECK_EQ(s.queued_bytes(), size_t(0));
  // Stream 1's frames stayed in order.
  size_t i1 = 0;
  for (auto& f : ch->sent)
    if (f.first == 1u) CHECK_EQ(f.second, i1++ == 0 ? size_t(60000) : size_t(150));
}

// Past kFifoBytes a stream drops to round-robin: a newer stream's first
// kFifoBytes go ahead of it, then the two alternate.
TEST(scheduler_bulk_fifo_then_round_robin) {
  auto ch = std::make_shared<FakeChannel>();
  FrameScheduler s(ch, 1000);
  ch->buffered = 5000;
  Bytes big = Bytes::copy(std::string(60000, 'b'));
  const int n = 45;  // 2.7 MB per stream
  for (int i = 0; i < n; i++) s.send(proto::make_body(proto::MsgType::ResBody, 7, big));
  for (int i = 0; i < n; i++) s.send(proto::make_body(proto::MsgType::ResBody, 9, big));
  for (int i = 0; i < 2 * n; i++) {
    ch->buffered = 0;
    s.pump();
  }
  CHECK_EQ(ch->sent.size(), size_t(2 * n));
  const size_t fifo_frames = (FrameScheduler::kFifoBytes + 60004) / 60005;
  const size_t share = (FrameScheduler::kBulkShareBytes + 60004) / 60005;  // oldest-first frames per bulk turn
  size_t i = 0;
  for (; i < fifo_frames; i++) CHECK_EQ(ch->sent[i].first, 7u);
  // Stream 9's first 2 MB go oldest-first, with stream 7 (now past its
  // kFifoBytes) given one frame after every `share` of them.
  size_t nine = 0, seven = 0, run = 0;
  for (; nine < fifo_frames; i++) {
    if (ch->sent[i].first == 9u) {
      nine++;
      run++;
    } else {
      CHECK_EQ(ch->sent[i].first, 7u);
      CHECK_EQ(run, share);
      run = 0;
      seven++;
    }
  }
  CHECK_EQ(seven, (fifo_frames - 1) / share);
  // Then round-robin: stream 7's remaining frames never go back to back.
  size_t rest7 = 0;
  for (size_t k = i; k < ch->sent.size(); k++) {
    if (ch->sent[k].first != 7u) continue;
    rest7++;
    CHECK(k + 1 >= ch->sent.size() || ch->sent[k + 1].first == 9u);
  }
  CHECK_EQ(rest7, size_t(n) - fifo_frames - seven);
  CHECK_EQ(s.queued_bytes(), size_t(0));
}

// A transfer past kFifoBytes keeps making progress while new streams keep the
// oldest-first lane busy (advice r3: a 32 MB download under a steady load of
// 1 MB requests got no turns).
TEST(scheduler_long_stream_not_starved_by_new_fifo_streams) {
  auto ch = std::make_shared<FakeChannel>();
  FrameScheduler s(ch, 1000);
  Bytes big = Bytes::copy(std::string(60000, 'b'));
  ch->buffered = 5000;
  const int long_frames = 32 * 1048576 / 60000;
  for (int i = 0; i < long_frames; i++) s.send(proto::make_body(proto::MsgType::ResBody, 1, big));
  // Let stream 1 move past its first 2 MB.
  for (int i = 0; i < 40; i++) {
    ch->buffered = 0;
    s.pump();
  }
  size_t long_sent = 0;
  for (auto& e : ch->sent) long_sent += e.first == 1u;
  CHECK_EQ(long_sent, size_t(40));
  // A steady load: a new 1 MB stream arrives every turn, always with queued
  // frames ahead in the oldest-first lane.
  uint32_t next = 2;
  const size_t before = ch->sent.size();
  for (int turn = 0; turn < 400; turn++) {
    if (turn % 2 == 0) {
      for (int k = 0; k < 18; k++) s.send(proto::make_body(proto::MsgType::ReqBody, next, big));
      s.send(proto::make_empty(proto::MsgType::ReqEnd, next));
      next++;
    }
    ch->buffered = 0;
    s.pump();
  }
  size_t long_now = 0, total = 0;
  for (size_t k = before; k < ch->sent.size(); k++) {
    total++;
    long_now += ch->sent[k].first == 1u;
  }
  // The round-robin lane gets about one frame per kBulkShareBytes of
  // oldest-first bytes: well above zero, and the new streams still lead.
  CHECK(long_now * 8 >= total);
  CHECK(long_now * 2 <= total);
}

// A stream whose queue ran dry keeps its attained service: past kFifoBytes it
// stays behind a younger stream's first bytes after producing again; a
// finished stream is forgotten.
TEST(scheduler_fifo_survives_idle_gaps) {
  auto ch = std::make_shared<FakeChannel>();
  FrameScheduler s(ch, 1000);
  Bytes big = Bytes::copy(std::string(60000, 'b'));
  const int n = int(FrameScheduler::kFifoBytes / 60005) + 2;
  for (int i = 0; i < n; i++) {
    s.send(proto::make_body(proto::MsgType::ResBody, 4, big));
    ch->buffered = 0;
  }
  CHECK_EQ(ch->sent.size(), size_t(n));
  CHECK_EQ(s.queued_bytes(), size_t(0));
  ch->buffered = 5000;
  for (int i = 0; i < 3; i++) s.send(proto::make_body(proto::MsgType::ResBody, 4, big));
  for (int i = 0; i < 3; i++) s.send(proto::make_body(proto::MsgType::ResBody, 6, big));
  for (int i = 0; i < 6; i++) {
    ch->buffered = 0;
    s.pump();
  }
  CHECK_EQ(ch->sent.size(), size_t(n + 6));
  for (size_t i = 0; i < 3; i++) CHECK_EQ(ch->sent[n + i].first, 6u);  // the younger stream's first bytes
  for (size_t i = 3; i < 6; i++) CHECK_EQ(ch->sent[n + i].first, 4u);
  CHECK_EQ(s.queued_bytes(), size_t(0));
}
