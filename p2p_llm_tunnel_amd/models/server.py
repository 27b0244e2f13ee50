"""OpenAI/Ollama-compatible streaming endpoint backed by ``TinyLlama`` on a HIP device.

This is the "local inference endpoint on the MI355X node" that ``tunnel serve
--upstream`` fronts (BASELINE.json configs #2/#5). One engine thread owns the
GPU and runs iteration-level (continuous) batching: every step advances each
active slot by one token — a prompt token while prefilling, the last sampled
token while decoding — so new requests join without waiting for others.
HTTP handler threads stream tokens as they are produced:

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
import http.server
import json
import queue
import socketserver
import threading
import time
import uuid

import torch

from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama


class Request:
    def __init__(self, prompt_ids: list[int], max_new: int):
        self.prompt = prompt_ids
        self.max_new = max_new
        self.out: queue.Queue = queue.Queue()
        self.generated = 0
        self.cancelled = False


class Engine:
    """Continuous batching with chunked prefill over the fused decode step.

    Every step packs up to ``rows`` (16) token rows: first one decode row per
    generating sequence, then prompt chunks of prefilling sequences, each row
    tagged with its cache slot and position (``TinyLlama.decode_step(slots=)``).
    A 512-byte prompt is thus prefilled in 32 steps instead of 512, while
    generating sequences keep emitting a token every step. Padding rows point
    at the model's scratch slot. The step is replayed from one hipGraph.
    """

    def __init__(self, device="cuda:0", config="tiny", max_batch=8, seed=0, use_graph=True, rows=16):
        self.model = TinyLlama(config, device=device, max_batch=max_batch, seed=seed, fused=True)
        self.device = self.model.device
        self.rows = rows
        self.use_graph = use_graph
        if use_graph:
            self.model.capture_graph(rows=rows)
        self.max_batch = max_batch
        self.pending: queue.Queue = queue.Queue()
        self.slots: list[dict | None] = [None] * max_batch
        self._stop = threading.Event()
        self.steps = 0
        self.tokens_out = 0
        self.prefill_tokens = 0
        self.thread = threading.Thread(target=self._loop, daemon=True, name="engine")
        self.thread.start()

    def submit(self, req: Request) -> Request:
        self.pending.put(req)
        return req

    def stop(self):
        self._stop.set()
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

    def _loop(self):
        torch.cuda.set_device(self.device)
        while not self._stop.is_set():
            self._admit()
            rows = self._plan()
            if not rows:
                time.sleep(0.0005)
                continue
            n = len(rows)
            pad = self.rows - n if self.use_graph else 0
            slot = [r[0] for r in rows] + [self.model.scratch_slot] * pad
            tok = [r[1] for r in rows] + [0] * pad
            pos = [r[2] for r in rows] + [0] * pad
            t = torch.tensor(tok, dtype=torch.int64).to(self.device, non_blocking=True)
            p = torch.tensor(pos, dtype=torch.int32).to(self.device, non_blocking=True)
            sl = torch.tensor(slot, dtype=torch.int32).to(self.device, non_blocking=True)
            if self.use_graph:
                out = self.model.graph_step(t, p, sl)[:n].tolist()
            else:
                out = self.model.decode_step(t, p, (min(pos), max(pos)), slots=sl).tolist()
            self.steps += 1
            for (i, _, _, emits), nxt in zip(rows, out):
                s = self.slots[i]
                s["pos"] += 1
                if not emits:
                    self.prefill_tokens += 1
                    continue
                req = s["req"]
                s["last"] = nxt
                if req.cancelled:
                    req.out.put(None)
                    self.slots[i] = None
                    continue
                req.out.put(nxt)
                req.generated += 1
                self.tokens_out += 1
                if req.generated >= req.max_new or s["pos"] >= self.model.cfg.max_seq - 1:
                    req.out.put(None)
                    self.slots[i] = None


def _prompt_ids(body: dict) -> list[int]:
    if "messages" in body:
        text = "\n".join(str(m.get("content", "")) for m in body.get("messages", []))
    else:
        text = str(body.get("prompt", ""))
    return list(text.encode("utf-8"))[:512] or [1]


def make_handler(engine: Engine, model_name: str):
    class H(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"
        # Tokens leave as small chunked writes every decode step; with Nagle on,
        # each would wait for the peer's (delayed) ACK of the previous one.
        disable_nagle_algorithm = True

        def log_message(self, *a):
            pass

        def _send_json(self, obj, status=200):
            b = json.dumps(obj).encode()
            self.send_response(status)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            if self.path in ("/v1/models", "/models"):
                self._send_json({"object": "list", "data": [{"id": model_name, "object": "model",
                                                             "owned_by": "p2p_llm_tunnel_amd"}]})
            elif self.path == "/health":
                b = b"ok"
                self.send_response(200)
                self.send_header("Content-Type", "text/plain")
                self.send_header("Content-Length", "2")
                self.end_headers()
                self.wfile.write(b)
            elif self.path == "/api/tags":
                self._send_json({"models": [{"name": model_name, "model": model_name}]})
            else:
                self._send_json({"error": "not found"}, 404)

        def _body(self):
            n = int(self.headers.get("Content-Length", 0) or 0)
            raw = self.rfile.read(n) if n else b"{}"
            try:
                return json.loads(raw or b"{}")
            except ValueError:
                return {}

        def _chunk(self, data: bytes):
            self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
            self.wfile.flush()

        def do_POST(self):
            body = self._body()
            path = self.path.split("?")[0]
            if path not in ("/v1/chat/completions", "/chat/completions", "/v1/completions", "/api/generate"):
                self._send_json({"error": "not found"}, 404)
                return
            max_new = int(body.get("max_tokens", body.get("num_predict", 16)) or 16)
            req = engine.submit(Request(_prompt_ids(body), max(1, min(max_new, 1024))))
            rid = "chatcmpl-" + uuid.uuid4().hex[:12]
            chat = "chat" in path
            ollama = path == "/api/generate"
            stream = body.get("stream", ollama)
            if not stream:
                toks = []
                while (t := req.out.get()) is not None:
                    toks.append(t)
                text = "".join(f" t{t}" for t in toks)
                if ollama:
                    self._send_json({"model": model_name, "response": text, "done": True})
                elif chat:
                    self._send_json({"id": rid, "object": "chat.completion", "model": model_name,
                                     "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                                  "finish_reason": "length"}],
                                     "usage": {"prompt_tokens": len(req.prompt), "completion_tokens": len(toks),
                                               "total_tokens": len(req.prompt) + len(toks)}})
                else:
                    self._send_json({"id": rid, "object": "text_completion", "model": model_name,
                                     "choices": [{"index": 0, "text": text, "finish_reason": "length"}]})
                return
            self.send_response(200)
            self.send_header("Content-Type", "application/x-ndjson" if ollama else "text/event-stream")
            self.send_header("Cache-Control", "no-cache")
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            try:
                while (t := req.out.get()) is not None:
                    piece = f" t{t}"
                    if ollama:
                        self._chunk((json.dumps({"model": model_name, "response": piece, "done": False}) + "\n").encode())
                    else:
                        delta = {"content": piece} if chat else None
                        choice = {"index": 0, "delta": delta, "finish_reason": None} if chat else \
                            {"index": 0, "text": piece, "finish_reason": None}
                        obj = {"id": rid, "object": "chat.completion.chunk" if chat else "text_completion",
                               "model": model_name, "choices": [choice]}
                        self._chunk(f"data: {json.dumps(obj)}\n\n".encode())
                if ollama:
                    self._chunk((json.dumps({"model": model_name, "response": "", "done": True}) + "\n").encode())
                else:
                    fin = {"index": 0, "delta": {}, "finish_reason": "length"} if chat else \
                        {"index": 0, "text": "", "finish_reason": "length"}
                    self._chunk(f"data: {json.dumps({'id': rid, 'object': 'chat.completion.chunk', 'choices': [fin]})}\n\n".encode())
                    self._chunk(b"data: [DONE]\n\n")
                self.wfile.write(b"0\r\n\r\n")
                self.wfile.flush()
            except (BrokenPipeError, ConnectionResetError):
                req.cancelled = True

    return H


class _Server(socketserver.ThreadingMixIn, http.server.HTTPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 1024  # the default backlog of 5 drops SYNs of a connection burst (1 s retry)


def start_server(host="127.0.0.1", port=0, device="cuda:0", config="tiny", max_batch=8, model_name=None):
    engine = Engine(device=device, config=config, max_batch=max_batch)
    srv = _Server((host, port), make_handler(engine, model_name or f"p2pt-{config}"))
    threading.Thread(target=srv.serve_forever, daemon=True).start()
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
