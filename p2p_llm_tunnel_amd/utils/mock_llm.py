"""Mock OpenAI/Ollama-compatible upstream used by tests and benchmarks.

Workload parity with the reference's ``tmp/mock_llm.py``:
  * ``GET /v1/models`` -> ``{"object":"list","data":[{"id":"test-model",...}]}``
  * ``GET /health`` -> ``ok``
  * ``POST /v1/chat/completions`` with ``"stream": true`` -> 5 SSE token events
    ("Hello", " from", " the", " tunnel", "!") written 100 ms apart, then a
    final ``finish_reason: stop`` event and ``data: [DONE]``
    (reference tmp/mock_llm.py:43-69); non-streaming returns one JSON body.
  * HTTP/1.0, no Content-Length on SSE (reference tmp/mock_llm.py:97).

Extensions for the benchmark matrix:
  * ``--threaded`` serves requests concurrently (the reference mock is
    single-threaded, which caps streaming at ~2 req/s whatever the concurrency);
  * ``--tokens`` / ``--interval-ms`` change the token count and cadence;
  * ``POST /echo`` returns the request body (1 MB POST config);
  * ``GET /bulk?bytes=N`` streams N bytes;
  * ``GET /api/tags`` and ``POST /api/generate`` speak Ollama's NDJSON stream;
  * ``GET /drop`` sends headers + one event, then closes the socket (mid-stream
    upstream failure path, reference serve.rs:278-284).
"""
from __future__ import annotations

import argparse
import http.server
import json
import socket
import socketserver
import sys
import threading
import time
import urllib.parse

TOKENS = ["Hello", " from", " the", " tunnel", "!"]


def _chunk(token: str | None) -> dict:
    delta = {"content": token} if token is not None else {}
    return {
        "id": "chatcmpl-test",
        "object": "chat.completion.chunk",
        "choices": [{"index": 0, "delta": delta, "finish_reason": None if token is not None else "stop"}],
    }


class MockHandler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.0"
    tokens: list[str] = TOKENS
    interval_s: float = 0.1

    def log_message(self, fmt, *args):  # quiet
        pass

    # -- helpers -------------------------------------------------------
    def _json(self, obj, status=200):
        body = json.dumps(obj).encode()
        self.send_response(status)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _read_body(self) -> bytes:
        n = int(self.headers.get("Content-Length", 0) or 0)
        return self.rfile.read(n) if n > 0 else b""

    # -- routes --------------------------------------------------------
    def do_GET(self):
        url = urllib.parse.urlparse(self.path)
        if url.path in ("/v1/models", "/models"):
            self._json({"object": "list", "data": [{"id": "test-model", "object": "model"}]})
        elif url.path == "/health":
            self.send_response(200)
            self.send_header("Content-Type", "text/plain")
            self.end_headers()
            self.wfile.write(b"ok")
        elif url.path == "/api/tags":
            self._json({"models": [{"name": "test-model:latest", "model": "test-model:latest"}]})
        elif url.path == "/bulk":
            q = urllib.parse.parse_qs(url.query)
            n = int(q.get("bytes", ["1048576"])[0])
            self.send_response(200)
            self.send_header("Content-Type", "application/octet-stream")
            self.send_header("Content-Length", str(n))
            self.end_headers()
            block = bytes(range(256)) * 256
            left = n
            while left > 0:
                k = min(left, len(block))
                self.wfile.write(block[:k])
                left -= k
        elif url.path == "/drop":
            self.send_response(200)
            self.send_header("Content-Type", "text/event-stream")
            self.send_header("Content-Length", "100000")
            self.end_headers()
            self.wfile.write(f"data: {json.dumps(_chunk('partial'))}\n\n".encode())
            self.wfile.flush()
            self.connection.shutdown(socket.SHUT_RDWR)
        elif url.path == "/headers":
            self._json({k.lower(): v for k, v in self.headers.items()})
        elif url.path == "/slow-headers":
            time.sleep(float(urllib.parse.parse_qs(url.query).get("s", ["2"])[0]))
            self._json({"ok": True})
        else:
            self.send_response(404)
            self.send_header("Content-Type", "text/plain")
            self.end_headers()
            self.wfile.write(b"not found")

    def do_POST(self):
        self.server.posts = getattr(self.server, "posts", 0) + 1  # test hook: requests served (approximate)
        url = urllib.parse.urlparse(self.path)
        body = self._read_body()
        if url.path in ("/v1/chat/completions", "/chat/completions"):
            try:
                req = json.loads(body) if body else {}
            except ValueError:
                req = {}
            if req.get("stream", False):
                self._sse()
            else:
                self._json({
                    "id": "chatcmpl-test",
                    "object": "chat.completion",
                    "choices": [{"index": 0, "message": {"role": "assistant", "content": "".join(self.tokens)},
                                 "finish_reason": "stop"}],
                    "usage": {"prompt_tokens": 10, "completion_tokens": len(self.tokens),
                              "total_tokens": 10 + len(self.tokens)},
                })
        elif url.path == "/api/generate":
            self._ollama()
        elif url.path == "/echo":
            self.send_response(200)
            self.send_header("Content-Type", self.headers.get("Content-Type", "application/octet-stream"))
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
        else:
            self.send_response(404)
            self.end_headers()
            self.wfile.write(b"not found")

    def _sse(self):
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.send_header("Cache-Control", "no-cache")
        self.end_headers()
        for tok in self.tokens:
            self.wfile.write(f"data: {json.dumps(_chunk(tok))}\n\n".encode())
            self.wfile.flush()
            time.sleep(self.interval_s)
        self.wfile.write(f"data: {json.dumps(_chunk(None))}\n\n".encode())
        self.wfile.write(b"data: [DONE]\n\n")
        self.wfile.flush()

    def _ollama(self):
        self.send_response(200)
        self.send_header("Content-Type", "application/x-ndjson")
        self.end_headers()
        for tok in self.tokens:
            self.wfile.write((json.dumps({"model": "test-model", "response": tok, "done": False}) + "\n").encode())
            self.wfile.flush()
            time.sleep(self.interval_s)
        self.wfile.write((json.dumps({"model": "test-model", "response": "", "done": True}) + "\n").encode())
        self.wfile.flush()


class _Threaded(socketserver.ThreadingMixIn, socketserver.TCPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 1024


class _Single(socketserver.TCPServer):
    allow_reuse_address = True
    request_queue_size = 1024


def make_server(host: str = "127.0.0.1", port: int = 0, threaded: bool = True, tokens: int | None = None,
                interval_ms: float = 100.0):
    toks = TOKENS if tokens is None else [f" tok{i}" if i else "Hello" for i in range(tokens)]
    handler = type("Handler", (MockHandler,), {"tokens": toks, "interval_s": interval_ms / 1000.0})
    cls = _Threaded if threaded else _Single
    return cls((host, port), handler)


def start_in_thread(**kw):
    """Start a mock server on a daemon thread; returns (server, port)."""
    srv = make_server(**kw)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    return srv, srv.server_address[1]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=3001)
    ap.add_argument("--threaded", action="store_true")
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--interval-ms", type=float, default=100.0)
    a = ap.parse_args(argv)
    srv = make_server(a.host, a.port, a.threaded, a.tokens, a.interval_ms)
    print(f"Mock LLM server running on :{srv.server_address[1]}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
