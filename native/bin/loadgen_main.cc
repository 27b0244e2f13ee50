// `tunnel-loadgen` — native streamed-completion load generator.
//
// S client connections (keep-alive when the server allows it) each issue K
// back-to-back `POST /v1/chat/completions {"stream": true}` requests; a
// "step" is one request on every connection, all in flight together (the
// multiplexing dimension of the tunnel). TTFT = time from
// writing the request to the first byte of the first `data:` event. Runs on
// the reactor (no interpreter jitter), so µs-scale tunnel overhead is visible.
// Output: one JSON object on stdout.
#include <signal.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "core/net.h"
#include "core/reactor.h"
#include "http/http.h"

using namespace p2pt;

namespace {

struct Opts {
  std::string host = "127.0.0.1";
  uint16_t port = 8000;
  int streams = 8;
  int steps = 10;
  std::string path = "/v1/chat/completions";
  std::string body = R"({"model": "test-model", "stream": true, "messages": [{"role": "user", "content": "hi"}]})";
  size_t post_bytes = 0;  // >0: POST /echo with this many bytes instead
};

struct Result {
  std::vector<double> ttft_us, total_us;
  int errors = 0;
  uint64_t body_bytes = 0;
};

class Stream : public std::enable_shared_from_this<Stream> {
 public:
  Stream(Reactor& r, const Opts& o, Result& res) : r_(r), o_(o), res_(res) {}
  std::function<void()> on_done;  // one request finished

  void request() {
    if (!conn_ || conn_->closed()) {
      auto self = shared_from_this();
      TcpConn::connect(r_, o_.host, o_.port, false, [self](std::shared_ptr<TcpConn> c, std::string err) {
        if (!c) {
          self->res_.errors++;
          self->finish();
          return;
        }
        self->conn_ = c;
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
  void send() {
    std::string body = o_.post_bytes ? std::string(o_.post_bytes, 'x') : o_.body;
    std::string path = o_.post_bytes ? "/echo" : o_.path;
    std::string req = "POST " + path + " HTTP/1.1\r\nHost: " + o_.host + ":" + std::to_string(o_.port) +
                      "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) +
                      "\r\n\r\n" + body;
    buf_.clear();
    head_done_ = false;
    first_ = 0;
    active_ = true;
    t0_ = Reactor::now_us();
    conn_->write(std::move(req));
  }

  void on_data(const uint8_t* p, size_t n) {
    if (!active_) return;
    buf_.append(reinterpret_cast<const char*>(p), n);
    if (!head_done_) {
      size_t used = 0;
      auto rs = http::parse_response_head(buf_, head_, used, nullptr);
      if (rs == http::ParseResult::Incomplete) return;
      if (rs == http::ParseResult::Error || head_.status != 200) {
        res_.errors++;
        active_ = false;
        conn_->close();
        return;
      }
      buf_.erase(0, used);
      uint64_t len = 0;
      auto mode = http::response_body_mode(head_, "POST", len);  // sets len: evaluate before reset()
      body_.reset(mode, len);
      keep_ = head_.version_minor >= 1 && !head_.has_token("connection", "close") &&
              body_.mode() != http::BodyDecoder::Mode::UntilClose;
      head_done_ = true;
    }
    size_t used = body_.feed(reinterpret_cast<const uint8_t*>(buf_.data()), buf_.size(), [&](const uint8_t* d, size_t k) {
      if (!first_ && k) first_ = Reactor::now_us();
      res_.body_bytes += k;
    });
    if (used == SIZE_MAX) {
      res_.errors++;
      active_ = false;
      conn_->close();
      return;
    }
    buf_.erase(0, used);
    if (body_.done()) complete();
  }

  void on_close() {
    if (active_ && head_done_ && body_.on_eof()) {
      keep_ = false;
      complete();
      return;
    }
    if (active_) {
      res_.errors++;
      active_ = false;
      finish();
    }
  }

  void complete() {
    active_ = false;
    uint64_t now = Reactor::now_us();
    res_.ttft_us.push_back(double((first_ ? first_ : now) - t0_));
    res_.total_us.push_back(double(now - t0_));
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
  Result& res_;
  std::shared_ptr<TcpConn> conn_;
  std::string buf_;
  http::Head head_;
  http::BodyDecoder body_;
  bool head_done_ = false, keep_ = false, active_ = false;
  uint64_t t0_ = 0, first_ = 0;
};

double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  size_t k = size_t(q / 100.0 * double(v.size() - 1) + 0.5);
  return v[std::min(k, v.size() - 1)];
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  int warmup = 1;
  bool warm_conns = false;  // --warm-conns 1: warmup on the timed steps' own connections
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i], v = argv[i + 1];
    if (a == "--target") {
      size_t c = v.rfind(':');
      o.host = v.substr(0, c);
      o.port = uint16_t(atoi(v.c_str() + c + 1));
    } else if (a == "--streams") o.streams = atoi(v.c_str());
    else if (a == "--steps") o.steps = atoi(v.c_str());
    else if (a == "--warmup") warmup = atoi(v.c_str());
    else if (a == "--path") {
      o.path = v;
      if (v == "/api/generate") o.body = R"({"model": "test-model", "prompt": "hi", "stream": true})";
    } else if (a == "--body") o.body = v;
    else if (a == "--post-bytes") o.post_bytes = size_t(strtoull(v.c_str(), nullptr, 10));
    else if (a == "--warm-conns") warm_conns = v == "1";
  }
  signal(SIGPIPE, SIG_IGN);
  Reactor r;
  Result warm_res, res;
  int total_steps = warmup + o.steps;
  int step = 0, pending = 0;
  uint64_t t_start = 0, t_end = 0;
  std::function<void()> launch;
  // Warmup steps run on their own connections (results discarded); the timed
  // steps reuse one keep-alive connection per stream when the server allows.
  // --warm-conns 1 warms up on the timed connections instead, so connection
  // setup stays out of the timed steps (steady-state keep-alive serving).
  std::vector<std::shared_ptr<Stream>> live, warmers;
  for (int i = 0; i < o.streams; i++) {
    live.push_back(std::make_shared<Stream>(r, o, res));
    warmers.push_back(std::make_shared<Stream>(r, o, warm_res));
  }
  std::vector<uint64_t> step_end;  // timed steps' completion times (per-step durations in the output)
  launch = [&] {
    auto& set = step < warmup && !warm_conns ? warmers : live;
    if (step == warmup) {
      t_start = Reactor::now_us();
      if (warm_conns) {  // drop what the warmup recorded on the live streams
        warm_res.errors += res.errors;
        res = Result{};
      }
    }
    pending = o.streams;
    for (auto& s : set) s->request();
  };
  for (auto* set : {&warmers, &live})
    for (auto& s : *set)
      s->on_done = [&] {
        if (--pending == 0) {
          if (step >= warmup) step_end.push_back(Reactor::now_us());
          step++;
          if (step >= total_steps) {
            t_end = Reactor::now_us();
            r.stop();
            return;
          }
          launch();
        }
      };
  if (warmup == 0) t_start = Reactor::now_us();
  launch();
  r.run();
  double secs = double(t_end - t_start) / 1e6;
  std::string steps_ms;
  for (size_t i = 0; i < step_end.size(); i++) {
    char b[32];
    snprintf(b, sizeof b, "%s%.3f", i ? ", " : "", double(step_end[i] - (i ? step_end[i - 1] : t_start)) / 1e3);
    steps_ms += b;
  }
  printf("{\"streams\": %d, \"steps\": %d, \"requests\": %zu, \"errors\": %d, \"seconds\": %.6f, \"req_s\": %.4f, "
         "\"p50_ttft_ms\": %.4f, \"p90_ttft_ms\": %.4f, \"p99_ttft_ms\": %.4f, \"mean_ttft_ms\": %.4f, "
         "\"p50_total_ms\": %.4f, \"body_bytes\": %llu, \"MBps\": %.2f, \"step_ms\": [%s]}\n",
         o.streams, o.steps, res.ttft_us.size(), res.errors + warm_res.errors, secs,
         secs > 0 ? double(res.ttft_us.size()) / secs : 0.0, pct(res.ttft_us, 50) / 1e3, pct(res.ttft_us, 90) / 1e3,
         pct(res.ttft_us, 99) / 1e3,
         res.ttft_us.empty() ? 0.0 : [&] { double s = 0; for (double x : res.ttft_us) s += x; return s / double(res.ttft_us.size()) / 1e3; }(),
         pct(res.total_us, 50) / 1e3, static_cast<unsigned long long>(res.body_bytes),
         secs > 0 ? double(res.body_bytes) / secs / 1e6 : 0.0, steps_ms.c_str());
  return res.errors ? 1 : 0;
}
