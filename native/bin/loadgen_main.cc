// `tunnel-loadgen` — native streamed-completion load generator.
//
// S client connections (keep-alive when the server allows it) each issue K
// back-to-back requests (default `POST /v1/chat/completions {"stream": true}`);
// a "step" is one request on every connection of a thread, all in flight
// together (the multiplexing dimension of the tunnel).
//
// Measured per request: TTFT = time from writing the request to the first
// body byte; per streamed event (SSE "\n\n"-terminated, NDJSON "\n"-terminated)
// its arrival time, from which the inter-token latency (ITL: gap between
// consecutive events of one response) is derived — the number that shows
// head-of-line blocking behind other streams' bulk frames.
//
// --threads T spreads the streams over T reactor threads (one node-scale
// client must not be the bottleneck it measures); --target takes a comma-
// separated list (stream i uses target i mod n: the direct baseline against
// several upstreams). Runs on the reactor (no interpreter jitter), so µs-scale
// tunnel overhead is visible. Output: one JSON object on stdout.
#include <signal.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "core/net.h"
#include "core/reactor.h"
#include "http/http.h"

using namespace p2pt;

namespace {

struct Target {
  std::string host = "127.0.0.1";
  uint16_t port = 8000;
};

struct Opts {
  std::vector<Target> targets{Target{}};
  int streams = 8;
  int steps = 10;
  int warmup = 1;
  int threads = 1;
  bool warm_conns = false;
  // --hold 1: after the warm-up steps print "READY" and wait for a line on
  // stdin before the timed steps (one thread): a caller times exactly the
  // timed steps, on connections the warm-up already opened.
  bool hold = false;
  std::string method = "POST";
  std::string path = "/v1/chat/completions";
  std::string body = R"({"model": "test-model", "stream": true, "messages": [{"role": "user", "content": "hi"}]})";
  size_t post_bytes = 0;  // >0: POST /echo with this many bytes instead
  char event_sep = 0;     // 0: auto from content-type (SSE "\n\n", NDJSON "\n"); 'n' none
  uint64_t read_rate = 0; // >0: read at most this many body bytes/s per stream (slow client)
  uint64_t duration_us = 0;  // >0: repeat timed steps for this long (--duration-s)
};

struct Result {
  std::vector<double> ttft_us, total_us, itl_us;
  int errors = 0;
  uint64_t body_bytes = 0;
  uint64_t events = 0;
  std::vector<uint64_t> step_end;
  std::vector<double> step_ttft_max_us;  // per step: the slowest first byte (thread 0)
  size_t step_base = 0;                  // ttft_us entries before the current step
  uint64_t t_start = 0, t_end = 0;
};

// LOADGEN_TRACE=path: step boundaries of thread 0 as JSON lines in the
// tunnel's trace format (CLOCK_MONOTONIC us), so a waterfall can place the
// tunnel's per-request stamps inside the client's steps.
FILE* step_trace() {
  static FILE* f = [] () -> FILE* {
    const char* p = getenv("LOADGEN_TRACE");
    FILE* o = p && *p ? fopen(p, "a") : nullptr;
    if (o) setvbuf(o, nullptr, _IOLBF, 1 << 16);  // whole lines per write: the tunnel appends to the same file
    return o;
  }();
  return f;
}

void trace_step(int first, int step, const char* ev) {
  FILE* f = step_trace();
  if (!f || first != 0) return;
  fprintf(f, "{\"t_us\":%llu,\"role\":\"loadgen\",\"sid\":%d,\"ev\":\"%s\"}\n",
          static_cast<unsigned long long>(Reactor::now_us()), step, ev);
}

// The step thread 0 is in (for connection stamps: a step that opens new
// connections records when the last of them completed, as "connected").
std::atomic<int> g_step{0};

class Stream : public std::enable_shared_from_this<Stream> {
 public:
  Stream(Reactor& r, const Opts& o, const Target& t, Result* res) : r_(r), o_(o), t_(t), res_(res) {}
  std::function<void()> on_done;  // one request finished
  void set_result(Result* r) { res_ = r; }

  void request() {
    if (!conn_ || conn_->closed()) {
      auto self = shared_from_this();
      TcpConn::connect(r_, t_.host, t_.port, false, [self](std::shared_ptr<TcpConn> c, std::string err) {
        if (!c) {
          self->res_->errors++;
          self->finish();
          return;
        }
        self->conn_ = c;
        trace_step(0, g_step.load(std::memory_order_relaxed), "connected");
        std::weak_ptr<Stream> w = self;
        c->on_data([w](const uint8_t* p, size_t n) {
          if (auto s = w.lock()) s->on_data(p, n);
        });
        c->on_close([w](const std::string&) {
          if (auto s = w.lock()) s->on_close();
        });
        self->send();
      });
      return;
    }
    send();
  }

 private:
  // The request body, built once per process and shared by every request
  // (a refcounted buffer written zero-copy): building a 1 MB string per
  // request cost the single client thread ~0.4 ms each, 26 ms before the
  // last of 64 uploads could start.
  const Bytes& body_bytes() {
    static const Bytes b = [this] {
      std::string body = o_.post_bytes ? std::string(o_.post_bytes, 'x') : (o_.method == "GET" ? "" : o_.body);
      return Bytes::copy(body);
    }();
    return b;
  }

  void send() {
    const Bytes& body = body_bytes();
    std::string path = o_.post_bytes ? "/echo" : o_.path;
    std::string method = o_.post_bytes ? "POST" : o_.method;
    std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + t_.host + ":" + std::to_string(t_.port) + "\r\n";
    if (method != "GET") req += "Content-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
    req += "\r\n";
    buf_.clear();
    head_done_ = false;
    first_ = 0;
    last_ev_ = 0;
    sep_run_ = 0;
    active_ = true;
    t0_ = Reactor::now_us();
    conn_->write(std::move(req));
    if (!body.empty()) conn_->write(body);
  }

  // Event boundaries inside the decoded body bytes; records ITL gaps.
  void scan_events(const uint8_t* d, size_t k, uint64_t now) {
    if (sep_ == 'n') return;
    for (size_t i = 0; i < k; i++) {
      if (d[i] == '\n') {
        sep_run_++;
        if ((sep_ == 'l' && sep_run_ >= 1) || (sep_ == 's' && sep_run_ == 2)) {
          res_->events++;
          if (last_ev_) res_->itl_us.push_back(double(now - last_ev_));
          last_ev_ = now;
          if (sep_ == 'l') sep_run_ = 0;
        }
      } else if (d[i] != '\r') {
        sep_run_ = 0;
      }
    }
  }

  void on_data(const uint8_t* p, size_t n) {
    if (!active_) return;
    if (head_done_ && buf_.empty()) {  // body bytes straight from the socket buffer (no staging copy)
      uint64_t now = Reactor::now_us();
      size_t used = body_.feed(p, n, [&](const uint8_t* d, size_t k) {
        if (!first_ && k) first_ = now;
        res_->body_bytes += k;
        got_ += k;
        scan_events(d, k, now);
      });
      if (used == SIZE_MAX) {
        fail();
        return;
      }
      if (body_.done()) {
        complete();
        return;
      }
      if (used < n) buf_.append(reinterpret_cast<const char*>(p + used), n - used);
      throttle(now);
      return;
    }
    buf_.append(reinterpret_cast<const char*>(p), n);
    if (!head_done_) {
      size_t used = 0;
      auto rs = http::parse_response_head(buf_, head_, used, nullptr);
      if (rs == http::ParseResult::Incomplete) return;
      if (rs == http::ParseResult::Error || head_.status != 200) {
        fail();
        return;
      }
      buf_.erase(0, used);
      uint64_t len = 0;
      auto mode = http::response_body_mode(head_, o_.post_bytes ? "POST" : o_.method.c_str(), len);  // sets len
      body_.reset(mode, len);
      keep_ = head_.version_minor >= 1 && !head_.has_token("connection", "close") &&
              body_.mode() != http::BodyDecoder::Mode::UntilClose;
      head_done_ = true;
      sep_ = o_.event_sep;
      if (!sep_) {
        const std::string* ct = head_.get("content-type");
        if (ct && ct->find("event-stream") != std::string::npos) sep_ = 's';
        else if (ct && ct->find("ndjson") != std::string::npos) sep_ = 'l';
        else sep_ = 'n';
      }
    }
    uint64_t now = Reactor::now_us();
    size_t used = body_.feed(reinterpret_cast<const uint8_t*>(buf_.data()), buf_.size(), [&](const uint8_t* d, size_t k) {
      if (!first_ && k) first_ = now;
      res_->body_bytes += k;
      got_ += k;
      scan_events(d, k, now);
    });
    if (used == SIZE_MAX) {
      fail();
      return;
    }
    buf_.erase(0, used);
    if (body_.done()) {
      complete();
      return;
    }
    throttle(now);
  }

  // Slow client: stop reading once ahead of read_rate, resume when due.
  void throttle(uint64_t now) {
    if (!o_.read_rate || !conn_ || conn_->closed()) return;
    uint64_t due_us = t0_ + got_ * 1000000 / o_.read_rate;
    if (due_us <= now) return;
    conn_->pause_reading();
    std::weak_ptr<Stream> w = shared_from_this();
    r_.call_at(due_us, [w] {
      if (auto s = w.lock())
        if (s->conn_ && !s->conn_->closed()) s->conn_->resume_reading();
    });
  }

  void on_close() {
    if (active_ && head_done_ && body_.on_eof()) {
      keep_ = false;
      complete();
      return;
    }
    if (active_) {
      res_->errors++;
      active_ = false;
      finish();
    }
  }

  // An error response or a malformed body: counted, the connection dropped,
  // and the stream goes on to its next request (it used to stop here, and a
  // step waiting for it never ended: a 502 from a failed association hung the
  // run).
  void fail() {
    res_->errors++;
    active_ = false;
    if (conn_) {
      conn_->on_close(nullptr);
      conn_->close();
      conn_.reset();
    }
    finish();
  }

  void complete() {
    active_ = false;
    got_ = 0;
    uint64_t now = Reactor::now_us();
    res_->ttft_us.push_back(double((first_ ? first_ : now) - t0_));
    res_->total_us.push_back(double(now - t0_));
    if (!keep_ && conn_) {
      conn_->on_close(nullptr);
      conn_->close();
      conn_.reset();
    }
    finish();
  }

  void finish() {
    auto self = shared_from_this();
    r_.post([self] {
      if (self->on_done) self->on_done();
    });
  }

  Reactor& r_;
  const Opts& o_;
  Target t_;
  Result* res_;
  std::shared_ptr<TcpConn> conn_;
  std::string buf_;
  http::Head head_;
  http::BodyDecoder body_;
  bool head_done_ = false, keep_ = false, active_ = false;
  uint64_t t0_ = 0, first_ = 0, last_ev_ = 0, got_ = 0;
  char sep_ = 0;
  int sep_run_ = 0;
};

// One reactor thread driving streams [first, first + count).
void run_thread(const Opts& o, int first, int count, Result& res, Result& warm_res) {
  Reactor r;
  int total_steps = o.warmup + o.steps;
  int step = 0, pending = 0;
  std::vector<std::shared_ptr<Stream>> live, warmers;
  for (int i = first; i < first + count; i++) {
    const Target& t = o.targets[size_t(i) % o.targets.size()];
    live.push_back(std::make_shared<Stream>(r, o, t, &res));
    warmers.push_back(std::make_shared<Stream>(r, o, t, &warm_res));
  }
  // Warmup steps run on their own connections (results discarded); the timed
  // steps reuse one keep-alive connection per stream when the server allows.
  // --warm-conns 1 warms up on the timed connections instead, so connection
  // setup stays out of the timed steps (steady-state keep-alive serving).
  if (o.warm_conns)
    for (auto& s : live) s->set_result(&warm_res);
  std::function<void()> launch = [&] {
    auto& set = step < o.warmup && !o.warm_conns ? warmers : live;
    if (step == o.warmup && o.hold) {
      printf("READY\n");
      fflush(stdout);
      char line[64];
      if (!fgets(line, sizeof line, stdin)) {  // the caller went away: run anyway
      }
    }
    if (step == o.warmup) {
      res.t_start = Reactor::now_us();
      if (o.warm_conns)
        for (auto& s : live) s->set_result(&res);
    }
    pending = count;
    if (first == 0) g_step.store(step, std::memory_order_relaxed);
    trace_step(first, step, "step_start");
    for (auto& s : set) s->request();
  };
  for (auto* set : {&warmers, &live})
    for (auto& s : *set)
      s->on_done = [&] {
        if (--pending == 0) {
          trace_step(first, step, "step_end");
          if (step >= o.warmup) {
            res.step_end.push_back(Reactor::now_us());
            double mx = 0;
            for (size_t k = res.step_base; k < res.ttft_us.size(); k++) mx = std::max(mx, res.ttft_us[k]);
            res.step_ttft_max_us.push_back(mx);
            res.step_base = res.ttft_us.size();
          }
          step++;
          // --duration-s: timed steps repeat until the duration has passed
          // (the step in progress finishes), whatever --steps says.
          const bool done = o.duration_us ? step > o.warmup && Reactor::now_us() - res.t_start >= o.duration_us
                                          : step >= total_steps;
          if (done) {
            res.t_end = Reactor::now_us();
            r.stop();
            return;
          }
          launch();
        }
      };
  if (o.warmup == 0) res.t_start = Reactor::now_us();
  if (count == 0) return;
  launch();
  r.run();
}

double pct(std::vector<double>& v, double q) {
  if (v.empty()) return 0;
  size_t k = size_t(q / 100.0 * double(v.size() - 1) + 0.5);
  std::nth_element(v.begin(), v.begin() + long(std::min(k, v.size() - 1)), v.end());
  return v[std::min(k, v.size() - 1)];
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i], v = argv[i + 1];
    if (a == "--target") {
      o.targets.clear();
      for (size_t s = 0; s <= v.size();) {
        size_t e = v.find(',', s);
        if (e == std::string::npos) e = v.size();
        std::string hp = v.substr(s, e - s);
        s = e + 1;
        if (hp.empty()) continue;
        size_t c = hp.rfind(':');
        Target t;
        t.host = hp.substr(0, c);
        t.port = uint16_t(atoi(hp.c_str() + c + 1));
        o.targets.push_back(t);
      }
      if (o.targets.empty()) o.targets.push_back(Target{});
    } else if (a == "--streams") o.streams = atoi(v.c_str());
    else if (a == "--steps") o.steps = atoi(v.c_str());
    else if (a == "--warmup") o.warmup = atoi(v.c_str());
    else if (a == "--hold") {  // --hold 1
      o.hold = v != "0";
      if (o.hold) o.warm_conns = true;
    }
    else if (a == "--threads") o.threads = std::max(1, atoi(v.c_str()));
    else if (a == "--method") o.method = v;
    else if (a == "--path") {
      o.path = v;
      if (v == "/api/generate") o.body = R"({"model": "test-model", "prompt": "hi", "stream": true})";
    } else if (a == "--body") o.body = v;
    else if (a == "--post-bytes") o.post_bytes = size_t(strtoull(v.c_str(), nullptr, 10));
    else if (a == "--warm-conns") o.warm_conns = v == "1";
    else if (a == "--events") o.event_sep = v == "sse" ? 's' : v == "ndjson" ? 'l' : v == "none" ? 'n' : 0;
    else if (a == "--read-rate") o.read_rate = strtoull(v.c_str(), nullptr, 10);
    else if (a == "--duration-s") o.duration_us = uint64_t(atof(v.c_str()) * 1e6);
  }
  signal(SIGPIPE, SIG_IGN);
  int T = std::min(o.threads, std::max(1, o.streams));
  std::vector<Result> res(static_cast<size_t>(T)), warm(static_cast<size_t>(T));
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) {
    int first = o.streams * t / T, last = o.streams * (t + 1) / T;
    th.emplace_back(run_thread, std::cref(o), first, last - first, std::ref(res[size_t(t)]), std::ref(warm[size_t(t)]));
  }
  for (auto& x : th) x.join();
  Result all;
  int warm_errors = 0;
  all.t_start = UINT64_MAX;
  for (int t = 0; t < T; t++) {
    auto& r = res[size_t(t)];
    all.ttft_us.insert(all.ttft_us.end(), r.ttft_us.begin(), r.ttft_us.end());
    all.total_us.insert(all.total_us.end(), r.total_us.begin(), r.total_us.end());
    all.itl_us.insert(all.itl_us.end(), r.itl_us.begin(), r.itl_us.end());
    all.errors += r.errors;
    all.body_bytes += r.body_bytes;
    all.events += r.events;
    warm_errors += warm[size_t(t)].errors;
    if (r.t_start && r.t_start < all.t_start) all.t_start = r.t_start;
    all.t_end = std::max(all.t_end, r.t_end);
  }
  if (all.t_start == UINT64_MAX) all.t_start = all.t_end;
  double secs = double(all.t_end - all.t_start) / 1e6;
  // Per-step durations (thread 0's steps; every thread runs the same count).
  std::string steps_ms, step_ttft;
  for (size_t i = 0; i < res[0].step_ttft_max_us.size(); i++) {
    char b[32];
    snprintf(b, sizeof b, "%s%.3f", i ? ", " : "", res[0].step_ttft_max_us[i] / 1e3);
    step_ttft += b;
  }
  auto& se = res[0].step_end;
  for (size_t i = 0; i < se.size(); i++) {
    char b[32];
    snprintf(b, sizeof b, "%s%.3f", i ? ", " : "", double(se[i] - (i ? se[i - 1] : res[0].t_start)) / 1e3);
    steps_ms += b;
  }
  double mean = 0;
  for (double x : all.ttft_us) mean += x;
  if (!all.ttft_us.empty()) mean /= double(all.ttft_us.size());
  double itl_max = all.itl_us.empty() ? 0 : *std::max_element(all.itl_us.begin(), all.itl_us.end());
  printf("{\"streams\": %d, \"steps\": %d, \"threads\": %d, \"requests\": %zu, \"errors\": %d, \"seconds\": %.6f, "
         "\"req_s\": %.4f, \"p50_ttft_ms\": %.4f, \"p90_ttft_ms\": %.4f, \"p99_ttft_ms\": %.4f, \"mean_ttft_ms\": %.4f, "
         "\"p50_total_ms\": %.4f, \"body_bytes\": %llu, \"MBps\": %.2f, \"events\": %llu, \"events_s\": %.1f, "
         "\"p50_itl_ms\": %.4f, \"p90_itl_ms\": %.4f, \"p99_itl_ms\": %.4f, \"p999_itl_ms\": %.4f, \"max_itl_ms\": %.4f, "
         "\"step_ms\": [%s], \"step_max_ttft_ms\": [%s]}\n",
         o.streams, o.steps, T, all.ttft_us.size(), all.errors + warm_errors, secs,
         secs > 0 ? double(all.ttft_us.size()) / secs : 0.0, pct(all.ttft_us, 50) / 1e3, pct(all.ttft_us, 90) / 1e3,
         pct(all.ttft_us, 99) / 1e3, mean / 1e3, pct(all.total_us, 50) / 1e3,
         static_cast<unsigned long long>(all.body_bytes), secs > 0 ? double(all.body_bytes) / secs / 1e6 : 0.0,
         static_cast<unsigned long long>(all.events), secs > 0 ? double(all.events) / secs : 0.0,
         pct(all.itl_us, 50) / 1e3, pct(all.itl_us, 90) / 1e3, pct(all.itl_us, 99) / 1e3, pct(all.itl_us, 99.9) / 1e3,
         itl_max / 1e3, steps_ms.c_str(), step_ttft.c_str());
  return all.errors + warm_errors ? 1 : 0;
}
