"""OpenAI/Ollama-compatible streaming endpoint backed by ``TinyLlama`` on a HIP device.

This is the "local inference endpoint on the MI355X node" that ``tunnel serve
--upstream`` fronts (BASELINE.json configs #2/#5). One engine thread owns the
GPU and runs iteration-level (continuous) batching: every step advances each
active slot by one token — a prompt token while prefilling, the last sampled
token while decoding — so new requests join without waiting for others.

One asyncio thread serves HTTP/1.1 (keep-alive, chunked) for every
connection. The engine hands each step's tokens to it in ONE batch
(``call_soon_threadsafe``) and the I/O thread writes them from pre-rendered
byte templates, so a step costs one thread hand-off instead of one per
stream, and the engine waits for the GPU with the GIL released (event sync on
a pinned output buffer) while the I/O thread writes the previous step's
tokens. (The thread-per-connection server this replaces spent ~1.3 ms of
GIL ping-pong per 8-stream step around a 0.18 ms GPU step;
profiles/bench_gpu_upstream_r01.json.)

  GET  /v1/models, /health, /api/tags
  POST /v1/chat/completions  (SSE when "stream": true; JSON otherwise)
  POST /v1/completions       (same, "prompt" instead of "messages")
  POST /api/generate         (Ollama NDJSON stream)

Tokenisation is byte-level (prompt bytes mod vocab); generated ids are
rendered as `` t<id>`` pieces — the model is random-init, the point is the
serving path, not the text.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import queue
import socket
import threading
import time
import uuid

import torch


class Request:
    """A generation request. Tokens go to ``out`` (a queue ending with None)
    unless ``batched`` is set: then the engine's ``deliver`` hook receives them
    together with every other batched request's tokens of the same step."""

    def __init__(self, prompt_ids: list[int], max_new: int, batched: bool = False):
        self.prompt = prompt_ids
        self.max_new = max_new
        self.out: queue.Queue = queue.Queue()
        self.generated = 0
        self.cancelled = False
        self.batched = batched
        self.state = None  # front-end bookkeeping for batched requests


class Engine:
    """Continuous batching with chunked prefill over the fused decode step.

    Every step packs up to ``rows`` (16) token rows: first one decode row per
    generating sequence, then prompt chunks of prefilling sequences, each row
    tagged with its cache slot and position (``TinyLlama.decode_step(slots=)``).
    A 512-byte prompt is thus prefilled in 32 steps instead of 512, while
    generating sequences keep emitting a token every step. Padding rows point
    at the model's scratch slot. The step is replayed from one hipGraph whose
    inputs arrive in one pinned host->device copy and whose sampled ids leave
    through one pinned device->host copy; the engine waits on an event with
    the GIL released.

    ``model`` injects a model object (tests use a CPU stand-in with the same
    ``decode_step`` / ``cfg`` / ``scratch_slot`` / ``device`` surface).
    """

    def __init__(self, device="cuda:0", config="tiny", max_batch=8, seed=0, use_graph=True, rows=16, model=None):
        if model is None:
            from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
            model = TinyLlama(config, device=device, max_batch=max_batch, seed=seed, fused=True)
        else:
            use_graph = False
        self.model = model
        self.device = self.model.device
        self.rows = rows
        self.use_graph = use_graph
        if use_graph:
            self.model.capture_graph(rows=rows)
            self._h_in = torch.zeros((3, rows), dtype=torch.int64, pin_memory=True)
            self._h_in_np = self._h_in.numpy()
            self._d_in = torch.zeros((3, rows), dtype=torch.int64, device=self.device)
            self._h_out = torch.zeros(rows, dtype=torch.int64, pin_memory=True)
            self._ev = torch.cuda.Event()
        self.max_batch = max_batch
        self.pending: queue.Queue = queue.Queue()
        self.slots: list[dict | None] = [None] * max_batch
        self.deliver = None  # callable(list[(Request, int | None)]) for batched requests
        self._wake = threading.Event()
        self._stop = threading.Event()
        self.steps = 0
        self.tokens_out = 0
        self.prefill_tokens = 0
        self.thread = threading.Thread(target=self._loop, daemon=True, name="engine")
        self.thread.start()

    def submit(self, req: Request) -> Request:
        self.pending.put(req)
        self._wake.set()
        return req

    def stop(self):
        self._stop.set()
        self._wake.set()
        self.thread.join(timeout=10)

    def _admit(self):
        for i in range(self.max_batch):
            if self.slots[i] is None:
                try:
                    req = self.pending.get_nowait()
                except queue.Empty:
                    return
                ids = req.prompt[: self.model.cfg.max_seq - req.max_new - 1] or [0]
                self.slots[i] = {"req": req, "pos": 0, "ids": ids, "last": None}

    def _plan(self):
        """Rows for this step: [(slot, token, pos, emits)]."""
        V = self.model.cfg.vocab
        rows = []
        for i, s in enumerate(self.slots):  # decode rows first: one token each
            if s is not None and s["pos"] >= len(s["ids"]):
                rows.append((i, s["last"], s["pos"], True))
        for i, s in enumerate(self.slots):  # then prompt chunks
            if s is None or s["pos"] >= len(s["ids"]):
                continue
            take = min(self.rows - len(rows), len(s["ids"]) - s["pos"])
            for p in range(s["pos"], s["pos"] + take):
                rows.append((i, s["ids"][p] % V, p, p == len(s["ids"]) - 1))
            if len(rows) >= self.rows:
                break
        return rows

    def _run(self, rows) -> list[int]:
        n = len(rows)
        if self.use_graph:
            h = self._h_in_np
            h[0, :n] = [r[1] for r in rows]
            h[1, :n] = [r[2] for r in rows]
            h[2, :n] = [r[0] for r in rows]
            if n < self.rows:  # padding rows -> scratch slot
                h[0, n:] = 0
                h[1, n:] = 0
                h[2, n:] = self.model.scratch_slot
            self._d_in.copy_(self._h_in, non_blocking=True)
            ids = self.model.graph_step(self._d_in[0], self._d_in[1], self._d_in[2])
            self._h_out.copy_(ids, non_blocking=True)
            self._ev.record()
            self._ev.synchronize()  # GIL released: the I/O thread writes meanwhile
            return self._h_out[:n].tolist()
        tok = torch.tensor([r[1] for r in rows], dtype=torch.int64).to(self.device)
        pos = torch.tensor([r[2] for r in rows], dtype=torch.int32).to(self.device)
        sl = torch.tensor([r[0] for r in rows], dtype=torch.int32).to(self.device)
        lo, hi = min(r[2] for r in rows), max(r[2] for r in rows)
        return self.model.decode_step(tok, pos, (lo, hi), slots=sl).tolist()

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while not self._stop.is_set():
            self._admit()
            rows = self._plan()
            if not rows:
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            out = self._run(rows)
            self.steps += 1
            batch = []
            for (i, _, _, emits), nxt in zip(rows, out):
                s = self.slots[i]
                s["pos"] += 1
                if not emits:
                    self.prefill_tokens += 1
                    continue
                req = s["req"]
                s["last"] = nxt
                if req.cancelled:
                    self._emit(req, None, batch)
                    self.slots[i] = None
                    continue
                self._emit(req, nxt, batch)
                req.generated += 1
                self.tokens_out += 1
                if req.generated >= req.max_new or s["pos"] >= self.model.cfg.max_seq - 1:
                    self._emit(req, None, batch)
                    self.slots[i] = None
            if batch:
                self.deliver(batch)

    def _emit(self, req: Request, tok, batch: list):
        if req.batched and self.deliver is not None:
            batch.append((req, tok))
        else:
            req.out.put(tok)


def _prompt_ids(body: dict) -> list[int]:
    if "messages" in body:
        text = "\n".join(str(m.get("content", "")) for m in body.get("messages", []))
    else:
        text = str(body.get("prompt", ""))
    return list(text.encode("utf-8"))[:512] or [1]


def _chunk(data: bytes) -> bytes:
    return b"%x\r\n%s\r\n" % (len(data), data)


class _Stream:
    """Per-request output state on the I/O thread: the writer and the byte
    template around each token piece (token ids render as " t<id>": no JSON
    escaping needed)."""
    __slots__ = ("writer", "stream", "kind", "rid", "pre", "post", "toks", "done")

    def __init__(self, writer, stream, kind, rid, model):
        self.writer = writer
        self.stream = stream
        self.kind = kind  # "chat" | "text" | "ollama"
        self.rid = rid
        self.toks = []
        self.done = asyncio.get_running_loop().create_future()
        m = json.dumps(model)
        if kind == "chat":
            self.pre = ('data: {"id": "%s", "object": "chat.completion.chunk", "model": %s, "choices": '
                        '[{"index": 0, "delta": {"content": "' % (rid, m)).encode()
            self.post = b'"}, "finish_reason": null}]}\n\n'
        elif kind == "text":
            self.pre = ('data: {"id": "%s", "object": "text_completion", "model": %s, "choices": '
                        '[{"index": 0, "text": "' % (rid, m)).encode()
            self.post = b'", "finish_reason": null}]}\n\n'
        else:
            self.pre = ('{"model": %s, "response": "' % m).encode()
            self.post = b'", "done": false}\n'


class FrontEnd:
    """HTTP/1.1 server on one asyncio thread (see the module docstring)."""

    def __init__(self, engine: Engine, host: str, port: int, model_name: str):
        self.engine = engine
        self.model_name = model_name
        self.loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._err = None
        self.thread = threading.Thread(target=self._run, args=(host, port), daemon=True, name="http")
        self.thread.start()
        self._ready.wait(30)
        if self._err:
            raise self._err
        engine.deliver = lambda batch: self.loop.call_soon_threadsafe(self._on_batch, batch)

    # ---------------------------------------------------------------- lifecycle
    def _run(self, host, port):
        asyncio.set_event_loop(self.loop)
        try:
            self.server = self.loop.run_until_complete(
                asyncio.start_server(self._conn, host, port, backlog=1024, limit=1 << 20))
            self.server_address = self.server.sockets[0].getsockname()[:2]
        except Exception as e:  # noqa: BLE001 - re-raised by the constructor
            self._err = e
            self._ready.set()
            return
        self._ready.set()
        self.loop.run_forever()

    def shutdown(self):
        def stop():
            self.server.close()
            self.loop.stop()
        self.loop.call_soon_threadsafe(stop)
        self.thread.join(timeout=10)

    # ---------------------------------------------------------------- tokens
    def _on_batch(self, batch):
        for req, tok in batch:
            st = req.state
            if st is None or st.done.done():
                continue
            if st.writer.transport.is_closing():  # client went away: free the slot
                req.cancelled = True
                st.done.set_result(False)
                continue
            if tok is None:
                self._finish(req, st)
            elif st.stream:
                st.writer.write(_chunk(b"%s t%d%s" % (st.pre, tok, st.post)))
            else:
                st.toks.append(tok)

    def _finish(self, req, st):
        w = st.writer
        if st.stream:
            if st.kind == "ollama":
                tail = _chunk((json.dumps({"model": self.model_name, "response": "", "done": True}) + "\n").encode())
            else:
                fin = {"index": 0, "delta": {}, "finish_reason": "length"} if st.kind == "chat" else \
                    {"index": 0, "text": "", "finish_reason": "length"}
                obj = {"id": st.rid, "object": "chat.completion.chunk" if st.kind == "chat" else "text_completion",
                       "choices": [fin]}
                tail = _chunk(f"data: {json.dumps(obj)}\n\n".encode()) + _chunk(b"data: [DONE]\n\n")
            w.write(tail + b"0\r\n\r\n")
        else:
            text = "".join(f" t{t}" for t in st.toks)
            if st.kind == "ollama":
                obj = {"model": self.model_name, "response": text, "done": True}
            elif st.kind == "chat":
                obj = {"id": st.rid, "object": "chat.completion", "model": self.model_name,
                       "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                    "finish_reason": "length"}],
                       "usage": {"prompt_tokens": len(req.prompt), "completion_tokens": len(st.toks),
                                 "total_tokens": len(req.prompt) + len(st.toks)}}
            else:
                obj = {"id": st.rid, "object": "text_completion", "model": self.model_name,
                       "choices": [{"index": 0, "text": text, "finish_reason": "length"}]}
            w.write(self._json_response(obj))
        st.done.set_result(True)

    # ---------------------------------------------------------------- HTTP
    @staticmethod
    def _response(status: int, ctype: str, body: bytes, reason: str = "OK") -> bytes:
        return (b"HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n\r\n"
                % (status, reason.encode(), ctype.encode(), len(body))) + body

    def _json_response(self, obj, status=200) -> bytes:
        return self._response(status, "application/json", json.dumps(obj).encode(),
                              "OK" if status == 200 else "Not Found")

    async def _conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        sock = writer.get_extra_info("socket")
        if sock is not None:
            try:  # one small write per token: never hold it back for an ACK
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        try:
            while True:
                try:
                    head = await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ConnectionError):
                    break
                lines = head.decode("latin-1").split("\r\n")
                parts = lines[0].split(" ")
                if len(parts) != 3:
                    writer.write(self._response(400, "text/plain", b"bad request", "Bad Request"))
                    break
                method, target, version = parts
                hdrs = {}
                for line in lines[1:]:
                    if ":" in line:
                        k, v = line.split(":", 1)
                        hdrs[k.strip().lower()] = v.strip()
                try:
                    if "chunked" in hdrs.get("transfer-encoding", "").lower():
                        body = await self._read_chunked(reader)
                    else:
                        n = int(hdrs.get("content-length", "0") or 0)
                        body = await reader.readexactly(n) if n else b""
                except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ValueError, ConnectionError):
                    break
                conn = hdrs.get("connection", "").lower()
                keep = (version == "HTTP/1.1" and conn != "close") or (version == "HTTP/1.0" and conn == "keep-alive")
                ok = await self._dispatch(method, target.split("?")[0], body, writer)
                if not ok or not keep:
                    break
                await writer.drain()
        except ConnectionError:
            pass
        finally:
            try:
                writer.close()
            except RuntimeError:
                pass

    @staticmethod
    async def _read_chunked(reader) -> bytes:
        out = bytearray()
        while True:
            size = int((await reader.readuntil(b"\r\n")).split(b";")[0].strip() or b"0", 16)
            if size == 0:
                while (await reader.readuntil(b"\r\n")) != b"\r\n":  # trailers
                    pass
                return bytes(out)
            out += await reader.readexactly(size)
            await reader.readexactly(2)

    async def _dispatch(self, method, path, body, writer) -> bool:
        name = self.model_name
        if method in ("GET", "HEAD"):
            if path in ("/v1/models", "/models"):
                resp = self._json_response({"object": "list", "data": [
                    {"id": name, "object": "model", "owned_by": "p2p_llm_tunnel_amd"}]})
            elif path == "/health":
                resp = self._response(200, "text/plain", b"ok")
            elif path == "/api/tags":
                resp = self._json_response({"models": [{"name": name, "model": name}]})
            else:
                resp = self._json_response({"error": "not found"}, 404)
            if method == "HEAD":
                resp = resp[: resp.index(b"\r\n\r\n") + 4]
            writer.write(resp)
            return True
        if method != "POST" or path not in ("/v1/chat/completions", "/chat/completions", "/v1/completions",
                                            "/api/generate"):
            writer.write(self._json_response({"error": "not found"}, 404))
            return True
        try:
            req_body = json.loads(body or b"{}")
            if not isinstance(req_body, dict):
                req_body = {}
        except ValueError:
            req_body = {}
        max_new = int(req_body.get("max_tokens", req_body.get("num_predict", 16)) or 16)
        ollama = path == "/api/generate"
        kind = "ollama" if ollama else ("chat" if "chat" in path else "text")
        stream = bool(req_body.get("stream", ollama))
        rid = ("chatcmpl-" if kind == "chat" else "cmpl-") + uuid.uuid4().hex[:12]
        req = Request(_prompt_ids(req_body), max(1, min(max_new, 1024)), batched=True)
        st = _Stream(writer, stream, kind, rid, name)
        req.state = st
        if stream:
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: %s\r\nCache-Control: no-cache\r\n"
                         b"Transfer-Encoding: chunked\r\n\r\n"
                         % (b"application/x-ndjson" if ollama else b"text/event-stream"))
        self.engine.submit(req)
        return await st.done


def start_server(host="127.0.0.1", port=0, device="cuda:0", config="tiny", max_batch=8, model_name=None,
                 engine: Engine | None = None):
    """Engine + HTTP front-end; returns (server, port, engine). ``server.shutdown()``
    stops the HTTP side, ``engine.stop()`` the GPU side."""
    engine = engine or Engine(device=device, config=config, max_batch=max_batch)
    srv = FrontEnd(engine, host, port, model_name or f"p2pt-{config}")
    return srv, srv.server_address[1], engine


def _replicas(a) -> int:
    """--gpus N: one endpoint process per GPU on ports port..port+N-1 (data-
    parallel replicas: the model fits one MI355X many times over, so replicas
    scale throughput with no cross-GPU traffic). `tunnel serve --upstream`
    takes the printed comma-separated list and balances requests over them by
    fewest in flight. Each child is a fresh interpreter pinned to its device;
    the parent never touches the GPU and exits with the first child that dies."""
    import subprocess
    import sys
    base = a.port
    procs = []
    for i in range(a.gpus):
        cmd = [sys.executable, "-m", "p2p_llm_tunnel_amd.models.server", "--host", a.host, "--port", str(base + i),
               "--device", f"cuda:{i}", "--config", a.config, "--max-batch", str(a.max_batch)]
        procs.append(subprocess.Popen(cmd))
    ups = ",".join(f"http://{a.host}:{base + i}" for i in range(a.gpus))
    print(f"{a.gpus} inference endpoints; use: tunnel serve --upstream {ups}", flush=True)
    try:
        while True:
            for p in procs:
                rc = p.poll()
                if rc is not None:
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
                    return rc
            time.sleep(0.5)
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()
        return 0


def main(argv=None):
    ap = argparse.ArgumentParser(description="GPU-backed OpenAI/Ollama-compatible endpoint")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=11434)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--max-batch", type=int, default=8)
    ap.add_argument("--gpus", type=int, default=0,
                    help="spawn one endpoint per GPU (cuda:0..N-1) on consecutive ports instead of serving here")
    a = ap.parse_args(argv)
    if a.gpus > 0:
        raise SystemExit(_replicas(a))
    srv, port, engine = start_server(a.host, a.port, a.device, a.config, a.max_batch)
    print(f"inference endpoint on http://{a.host}:{port} ({a.config}, {a.device})", flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        engine.stop()


if __name__ == "__main__":
    main()
