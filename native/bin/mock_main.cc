// `tunnel-mock` — native implementation of the benchmark upstream.
//
// Same workload as the reference's tmp/mock_llm.py (and our Python
// p2p_llm_tunnel_amd/utils/mock_llm.py): GET /v1/models, GET /health,
// POST /v1/chat/completions with {"stream":true} -> 5 SSE token events written
// --interval-ms apart (default 100), then a finish_reason:"stop" event and
// "data: [DONE]"; HTTP/1.0 responses, no Content-Length on SSE, connection
// closed at the end. Extras: POST /echo, GET /bulk?bytes=N. Written on the
// reactor so it adds no GIL/thread-scheduling jitter to TTFT measurements.
#include <signal.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "core/net.h"
#include "core/reactor.h"
#include "http/http.h"

using namespace p2pt;

namespace {

const char* kTokens[] = {"Hello", " from", " the", " tunnel", "!"};

std::string chunk_event(const char* tok) {
  std::string delta = tok ? std::string("{\"content\": \"") + tok + "\"}" : "{}";
  std::string fin = tok ? "null" : "\"stop\"";
  return "data: {\"id\": \"chatcmpl-test\", \"object\": \"chat.completion.chunk\", \"choices\": [{\"index\": 0, "
         "\"delta\": " + delta + ", \"finish_reason\": " + fin + "}]}\n\n";
}

// Ollama /api/generate stream: one NDJSON object per token, then a done record.
std::string ollama_line(const char* tok) {
  if (!tok)
    return "{\"model\": \"test-model\", \"created_at\": \"2026-01-01T00:00:00Z\", \"response\": \"\", \"done\": true, "
           "\"done_reason\": \"stop\", \"eval_count\": 5}\n";
  return std::string("{\"model\": \"test-model\", \"created_at\": \"2026-01-01T00:00:00Z\", \"response\": \"") + tok +
         "\", \"done\": false}\n";
}

struct Server {
  Reactor& r;
  uint64_t interval_us;
  int tokens;
  bool trace;
  std::map<TcpConn*, std::shared_ptr<TcpConn>> conns;

  void respond(const std::shared_ptr<TcpConn>& c, int status, const std::string& ctype, const std::string& body) {
    std::string out = "HTTP/1.0 " + std::to_string(status) + " " + http::reason_phrase(status) +
                      "\r\nServer: p2pt-mock\r\nDate: " + http::http_date_now() + "\r\nContent-Type: " + ctype +
                      "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
    c->write(std::move(out));
    c->close_after_flush();
  }

  // Token stream: SSE chat-completion chunks, or Ollama NDJSON when `ollama`.
  void sse(const std::shared_ptr<TcpConn>& c, bool ollama = false) {
    c->write(std::string("HTTP/1.0 200 OK\r\nServer: p2pt-mock\r\nDate: ") + http::http_date_now() +
             (ollama ? "\r\nContent-Type: application/x-ndjson\r\n\r\n"
                     : "\r\nContent-Type: text/event-stream\r\nCache-Control: no-cache\r\n\r\n"));
    auto step = std::make_shared<std::function<void(int)>>();
    std::weak_ptr<TcpConn> w = c;
    Reactor* rp = &r;
    uint64_t iv = interval_us;
    int n = tokens;
    // The pending timer owns the step; the step refers to itself weakly.
    std::weak_ptr<std::function<void(int)>> ws = step;
    *step = [w, rp, iv, n, ws, ollama](int i) {
      auto conn = w.lock();
      if (!conn || conn->closed()) return;
      if (i < n) {
        const char* tok = i < 5 ? kTokens[i] : " tok";
        conn->write(ollama ? ollama_line(tok) : chunk_event(tok));
        if (auto s = ws.lock()) rp->call_later_us(iv, [s, i] { (*s)(i + 1); });
        return;
      }
      conn->write(ollama ? ollama_line(nullptr) : chunk_event(nullptr) + "data: [DONE]\n\n");
      conn->close_after_flush();
    };
    (*step)(0);
  }

  void handle(const std::shared_ptr<TcpConn>& c, const http::Head& h, const std::string& body) {
    std::string path = h.target.substr(0, h.target.find('?'));
    if (h.method == "GET" && (path == "/v1/models" || path == "/models")) {
      respond(c, 200, "application/json", R"({"object": "list", "data": [{"id": "test-model", "object": "model"}]})");
    } else if (h.method == "GET" && path == "/health") {
      respond(c, 200, "text/plain", "ok");
    } else if (h.method == "GET" && path == "/bulk") {
      size_t n = 1 << 20;
      size_t q = h.target.find("bytes=");
      if (q != std::string::npos) n = size_t(strtoull(h.target.c_str() + q + 6, nullptr, 10));
      // The body (bytes i & 0xFF) is built once per size and shared by every
      // response as a zero-copy view: a 64 MB download costs the reactor no
      // fill loop, so it never delays other connections' token timers.
      static thread_local std::map<size_t, Bytes> cache;
      auto it = cache.find(n);
      if (it == cache.end()) {
        std::vector<uint8_t> b(n);
        for (size_t i = 0; i < n; i++) b[i] = uint8_t(i & 0xFF);
        it = cache.emplace(n, Bytes::take(std::move(b))).first;
      }
      c->write("HTTP/1.0 200 OK\r\nServer: p2pt-mock\r\nDate: " + http::http_date_now() +
               "\r\nContent-Type: application/octet-stream\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
      c->write(it->second);
      c->close_after_flush();
    } else if (h.method == "POST" && (path == "/v1/chat/completions" || path == "/chat/completions")) {
      bool stream = body.find("\"stream\": true") != std::string::npos || body.find("\"stream\":true") != std::string::npos;
      if (stream) sse(c);
      else
        respond(c, 200, "application/json",
                R"({"id": "chatcmpl-test", "object": "chat.completion", "choices": [{"index": 0, "message": {"role": "assistant", "content": "Hello from the tunnel!"}, "finish_reason": "stop"}], "usage": {"prompt_tokens": 10, "completion_tokens": 5, "total_tokens": 15}})");
    } else if (h.method == "GET" && path == "/api/tags") {
      respond(c, 200, "application/json", R"({"models": [{"name": "test-model", "model": "test-model"}]})");
    } else if (h.method == "POST" && path == "/api/generate") {
      // Ollama streams unless the request says "stream": false.
      bool stream = body.find("\"stream\": false") == std::string::npos && body.find("\"stream\":false") == std::string::npos;
      if (stream) sse(c, true);
      else
        respond(c, 200, "application/json",
                R"({"model": "test-model", "response": "Hello from the tunnel!", "done": true, "done_reason": "stop"})");
    } else if (h.method == "POST" && path == "/echo") {
      respond(c, 200, "application/octet-stream", body);
    } else {
      respond(c, 404, "text/plain", "not found");
    }
  }

  void accept(int fd) {
    auto c = TcpConn::adopt(r, fd);
    conns[c.get()] = c;
    auto buf = std::make_shared<std::string>();
    auto done = std::make_shared<bool>(false);
    std::weak_ptr<TcpConn> w = c;
    // POST /sink: the body is consumed as it arrives (counted and checksummed,
    // never held), then {"bytes": N, "wsum": S} with S = sum of (i+1)*byte[i]
    // mod 2^64 (order-sensitive) — for bounded-memory upload tests of
    // gigabyte bodies.
    struct Sink {
      bool on = false;
      http::BodyDecoder body;
      uint64_t bytes = 0, wsum = 0;
      void eat(const uint8_t* d, size_t k) {
        for (size_t i = 0; i < k; i++) wsum += (bytes + i + 1) * d[i];
        bytes += k;
      }
      std::string json() const {
        return "{\"bytes\": " + std::to_string(bytes) + ", \"wsum\": " + std::to_string(wsum) + "}";
      }
    };
    auto sink = std::make_shared<Sink>();
    c->on_data([this, w, buf, done, sink](const uint8_t* p, size_t n) {
      if (*done) return;
      if (sink->on) {
        size_t used = sink->body.feed(p, n, [&](const uint8_t* d, size_t k) { sink->eat(d, k); });
        if (used == SIZE_MAX || sink->body.done()) {
          *done = true;
          if (auto s = w.lock()) respond(s, used == SIZE_MAX ? 400 : 200, "application/json", sink->json());
        }
        return;
      }
      buf->append(reinterpret_cast<const char*>(p), n);
      http::Head h;
      size_t used = 0;
      if (http::parse_request_head(*buf, h, used, nullptr) != http::ParseResult::Done) return;
      uint64_t len = 0;
      std::string err;
      auto mode = http::request_body_mode(h, len, &err);
      if (h.method == "POST" && h.target == "/sink") {
        sink->on = true;
        sink->body.reset(mode, len);
        std::string rest = buf->substr(used);
        buf->clear();
        if (auto s = w.lock()) {
          if (rest.empty() && !sink->body.done()) return;
          // Feed what arrived with the head through the same path.
          size_t u = sink->body.feed(reinterpret_cast<const uint8_t*>(rest.data()), rest.size(),
                                     [&](const uint8_t* d, size_t k) { sink->eat(d, k); });
          if (u == SIZE_MAX || sink->body.done()) {
            *done = true;
            respond(s, u == SIZE_MAX ? 400 : 200, "application/json", sink->json());
          }
        }
        return;
      }
      if (buf->size() - used < len) return;
      *done = true;
      if (trace) fprintf(stderr, "mock_req %llu %s\n", static_cast<unsigned long long>(Reactor::now_us()), h.method.c_str());
      if (auto s = w.lock()) handle(s, h, buf->substr(used, size_t(len)));
    });
    TcpConn* key = c.get();
    c->on_close([this, key](const std::string&) { r.post([this, key] { conns.erase(key); }); });
  }
};

}  // namespace

int main(int argc, char** argv) {
  std::string listen = "127.0.0.1:3001";
  uint64_t interval_us = 100000;
  int tokens = 5;
  int threads = 1;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "--listen") listen = argv[i + 1];
    else if (a == "--port") listen = "127.0.0.1:" + std::string(argv[i + 1]);
    else if (a == "--interval-ms") interval_us = strtoull(argv[i + 1], nullptr, 10) * 1000;
    else if (a == "--interval-us") interval_us = strtoull(argv[i + 1], nullptr, 10);
    else if (a == "--tokens") tokens = atoi(argv[i + 1]);
    else if (a == "--threads") threads = std::max(1, atoi(argv[i + 1]));
  }
  signal(SIGPIPE, SIG_IGN);
  // Accepts on one listener; with --threads N, accepted sockets are handed
  // round-robin to N reactor threads (a node-scale upstream that is not itself
  // the bottleneck of a many-stream benchmark).
  std::vector<std::unique_ptr<Reactor>> rs;
  std::vector<std::unique_ptr<Server>> servers;
  for (int t = 0; t < threads; t++) {
    rs.push_back(std::make_unique<Reactor>());
    servers.push_back(std::make_unique<Server>(Server{*rs.back(), interval_us, tokens, getenv("MOCK_TRACE") != nullptr, {}}));
  }
  Reactor& r = *rs[0];
  std::string err;
  size_t next = 0;
  auto l = TcpListener::bind(
      r, listen,
      [&](int fd, SockAddr) {
        size_t k = next++ % servers.size();
        if (k == 0) servers[0]->accept(fd);
        else {
          Server* sv = servers[k].get();
          rs[k]->post_threadsafe([sv, fd] { sv->accept(fd); });
        }
      },
      &err);
  if (!l) {
    fprintf(stderr, "mock: %s\n", err.c_str());
    return 1;
  }
  printf("Mock LLM server running on %s\n", l->local_addr().str().c_str());
  fflush(stdout);
  r.on_signal(SIGINT, [&] { r.stop(); });
  r.on_signal(SIGTERM, [&] { r.stop(); });
  std::vector<std::thread> th;
  for (int t = 1; t < threads; t++) th.emplace_back([&rs, t] { rs[size_t(t)]->run(); });
  r.run();
  for (int t = 1; t < threads; t++) rs[size_t(t)]->post_threadsafe([&rs, t] { rs[size_t(t)]->stop(); });
  for (auto& x : th) x.join();
  return 0;
}
