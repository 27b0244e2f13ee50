"""The inference endpoint's serving path (asyncio HTTP front-end, batched
token delivery, continuous batching with chunked prefill) on the CPU, with a
deterministic stand-in for the GPU model; the GPU model itself is covered by
tests/test_gpu_model.py."""
import http.client
import json
import socket
import threading
import time
from types import SimpleNamespace

import torch

from p2p_llm_tunnel_amd.models.server import Engine, Request, start_server


class FakeModel:
    """decode_step surface of TinyLlama: next = (31 * token + pos + 7) % vocab."""

    def __init__(self, max_batch=4, vocab=1000, max_seq=256, delay_s=0.0):
        self.cfg = SimpleNamespace(vocab=vocab, max_seq=max_seq)
        self.device = torch.device("cpu")
        self.scratch_slot = max_batch
        self.delay_s = delay_s
        self.calls = 0

    def decode_step(self, tokens, pos, pos_range, slots=None):
        self.calls += 1
        if self.delay_s:
            time.sleep(self.delay_s)
        return (tokens * 31 + pos.to(torch.int64) + 7) % self.cfg.vocab


def expected(prompt: bytes, n: int, vocab=1000):
    ids = list(prompt) or [1]
    last, pos = ids[-1] % vocab, len(ids) - 1
    out = []
    for _ in range(n):
        last = (last * 31 + pos + 7) % vocab
        out.append(last)
        pos += 1
    return out


def _server(**kw):
    eng = Engine(max_batch=4, model=FakeModel(**kw))
    srv, port, _ = start_server(port=0, engine=eng, model_name="fake")
    return srv, port, eng


def _post(port, path, body, conn=None):
    c = conn or http.client.HTTPConnection("127.0.0.1", port, timeout=20)
    c.request("POST", path, body=json.dumps(body), headers={"content-type": "application/json"})
    r = c.getresponse()
    return r.status, r.getheader("content-type"), r.read(), c


def test_sse_chat_stream_and_json_agree():
    srv, port, eng = _server()
    try:
        body = {"stream": True, "max_tokens": 6, "messages": [{"role": "user", "content": "hello"}]}
        st, ct, data, c = _post(port, "/v1/chat/completions", body)
        assert st == 200 and ct == "text/event-stream"
        events = [l[6:] for l in data.split(b"\n") if l.startswith(b"data: ")]
        assert events[-1] == b"[DONE]" and len(events) == 8
        objs = [json.loads(e) for e in events[:-1]]
        assert all(o["object"] == "chat.completion.chunk" for o in objs)
        text = "".join(o["choices"][0]["delta"].get("content", "") for o in objs)
        assert text == "".join(f" t{t}" for t in expected(b"hello", 6))
        assert objs[-1]["choices"][0]["finish_reason"] == "length"
        # same connection (keep-alive), non-streamed
        st, ct, data, _ = _post(port, "/v1/chat/completions", dict(body, stream=False), c)
        j = json.loads(data)
        assert st == 200 and j["choices"][0]["message"]["content"] == text
        assert j["usage"]["completion_tokens"] == 6
    finally:
        srv.shutdown()
        eng.stop()


def test_completions_and_ollama_and_gets():
    srv, port, eng = _server()
    try:
        st, _, data, _ = _post(port, "/v1/completions", {"stream": True, "max_tokens": 3, "prompt": "abc"})
        objs = [json.loads(l[6:]) for l in data.split(b"\n") if l.startswith(b"data: {")]
        assert "".join(o["choices"][0]["text"] for o in objs) == "".join(f" t{t}" for t in expected(b"abc", 3))
        st, ct, data, _ = _post(port, "/api/generate", {"prompt": "abc", "num_predict": 4})
        lines = [json.loads(l) for l in data.splitlines() if l]
        assert ct == "application/x-ndjson" and lines[-1]["done"] is True and len(lines) == 5
        assert "".join(l["response"] for l in lines) == "".join(f" t{t}" for t in expected(b"abc", 4))
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        for path, want in (("/health", b"ok"), ("/v1/models", b'"fake"'), ("/api/tags", b'"fake"')):
            c.request("GET", path)
            r = c.getresponse()
            assert r.status == 200 and want in r.read()
        c.request("GET", "/nope")
        r = c.getresponse()
        assert r.status == 404 and r.read()
        c.request("HEAD", "/health")
        r = c.getresponse()
        assert r.status == 200 and r.read() == b""
    finally:
        srv.shutdown()
        eng.stop()


def test_concurrent_streams_are_batched_and_independent():
    srv, port, eng = _server(delay_s=0.002)
    try:
        prompts = [b"x" * n for n in (1, 17, 40, 5, 9, 33, 2, 64)]  # 8 streams > 4 slots: queueing too
        results = [None] * len(prompts)

        def run(i):
            _, _, data, _ = _post(port, "/v1/chat/completions",
                                  {"stream": True, "max_tokens": 10,
                                   "messages": [{"role": "user", "content": prompts[i].decode()}]})
            objs = [json.loads(l[6:]) for l in data.split(b"\n") if l.startswith(b"data: {")]
            results[i] = "".join(o["choices"][0]["delta"].get("content", "") for o in objs)

        ts = [threading.Thread(target=run, args=(i,)) for i in range(len(prompts))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(30)
        for p, r in zip(prompts, results):
            assert r == "".join(f" t{t}" for t in expected(p, 10))
        assert eng.model.calls < sum(len(p) + 10 for p in prompts)  # rows were shared across requests
    finally:
        srv.shutdown()
        eng.stop()


def test_single_token_requests_with_multibyte_prompts():
    """max_tokens=1 finishes a request on its prompt's sampling row, which the
    step plan orders before that prompt's other rows; the engine must survive
    it (stream and non-stream), and bad/edge max_tokens values get answers."""
    srv, port, eng = _server(max_seq=64)
    try:
        for stream in (True, False):
            for mt in (1, 0, -5, None):
                body = {"stream": stream, "prompt": "hello world", "max_tokens": mt}
                st, _, data, _ = _post(port, "/v1/completions", body)
                assert st == 200, data
                if stream:
                    objs = [json.loads(l[6:]) for l in data.split(b"\n") if l.startswith(b"data: {")]
                    text = "".join(o["choices"][0]["text"] for o in objs)
                else:
                    text = json.loads(data)["choices"][0]["text"]
                n = 16 if mt is None else 1
                assert text == "".join(f" t{t}" for t in expected(b"hello world", n)), (stream, mt, text)
        assert eng.thread.is_alive()
        # max_tokens beyond the context: clamped, the prompt's tail is kept
        st, _, data, _ = _post(port, "/v1/completions", {"stream": False, "prompt": "abc", "max_tokens": 1000})
        assert st == 200 and json.loads(data)["choices"][0]["text"].count(" t") == 62
        for bad in ("lots", [3], {"x": 1}):
            st, _, data, _ = _post(port, "/v1/completions", {"prompt": "a", "max_tokens": bad})
            assert st == 400 and b"max_tokens" in data
        st, _, data, _ = _post(port, "/v1/completions", {"stream": False, "prompt": "ok", "max_tokens": 2})
        assert st == 200 and eng.thread.is_alive()
    finally:
        srv.shutdown()
        eng.stop()


def test_client_disconnect_frees_the_slot():
    srv, port, eng = _server(delay_s=0.005)
    try:
        s = socket.create_connection(("127.0.0.1", port), timeout=10)
        body = json.dumps({"stream": True, "max_tokens": 1000, "messages": [{"role": "user", "content": "hi"}]})
        s.sendall(b"POST /v1/chat/completions HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s"
                  % (len(body), body.encode()))
        assert s.recv(4096).startswith(b"HTTP/1.1 200")
        s.close()
        deadline = time.time() + 10
        while any(eng.slots) and time.time() < deadline:
            time.sleep(0.02)
        assert not any(eng.slots)
        assert eng.tokens_out < 1000
        st, _, data, _ = _post(port, "/v1/chat/completions", {"stream": False, "max_tokens": 2, "prompt": "a"})
        assert st == 200
    finally:
        srv.shutdown()
        eng.stop()


def test_chunked_request_body_and_queue_consumers():
    srv, port, eng = _server()
    try:
        s = socket.create_connection(("127.0.0.1", port), timeout=10)
        body = json.dumps({"stream": False, "max_tokens": 2, "prompt": "zz"}).encode()
        s.sendall(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n"
                  b"%x\r\n%s\r\n0\r\n\r\n" % (len(body), body))
        data = b""
        while (d := s.recv(65536)):
            data += d
        assert data.startswith(b"HTTP/1.1 200") and b'"text_completion"' in data
        # direct Engine users (no front-end batching) still get a token queue
        r = eng.submit(Request(list(b"qq"), 3))
        assert list(iter(r.out.get, None)) == expected(b"qq", 3)
    finally:
        srv.shutdown()
        eng.stop()


def test_through_the_tunnel():
    from p2p_llm_tunnel_amd.utils.procs import Tunnel
    srv, port, eng = _server()
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport="tcp") as t:
            for _ in range(3):  # upstream keep-alive reuse through serve's pool
                st, _, data, _ = _post(t.proxy_port, "/v1/chat/completions",
                                       {"stream": True, "max_tokens": 4, "messages": [{"role": "user", "content": "yo"}]})
                assert st == 200 and data.count(b"data: ") == 6
    finally:
        srv.shutdown()
        eng.stop()
