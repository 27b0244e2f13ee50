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

Sampling: temperature / top_p / seed (and the common top_k extension) from an
OpenAI request, or "options" of an Ollama one, drawn on device after the LM
head (ops.sample_, sample.hip: top-k and top-p by radix select, Gumbel-max
draw); temperature 0 — the default unless --default-temperature — keeps the
fused LM head's greedy argmax. Stop sequences (OpenAI "stop": a string or up
to 4; Ollama "options.stop") end a completion at the first match in the
detokenised text, which is left out (finish_reason "stop"); a streamed
response holds back only a tail that could still begin one. Parameters that
would change the output and are not implemented (n > 1, penalties,
logit_bias, logprobs, Ollama's repeat_penalty, mirostat, ...) are answered
with 400, as is sampling on an engine without the captured HIP step.

Two model sources:

* random-init (``--config tiny|small|micro``, the benchmark default): byte-level
  prompts (bytes mod vocab), generated ids rendered as `` t<id>`` pieces;
* a Hugging Face Llama-architecture checkpoint (``--checkpoint DIR``: config.json,
  safetensors, tokenizer.json; loaded weights-only by ``checkpoint.py``): prompts
  go through the checkpoint's tokenizer and chat template, tokens are
  detokenised incrementally, and generation stops at the EOS token
  (finish_reason "stop").
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import queue
import socket
import sys
import threading
import time
import uuid

import torch


class Sampling:
    """How a request picks its tokens: temperature (0 = greedy argmax, the
    fused LM head's own result), then top-k (0 = off) and top-p (1 = off),
    drawn on device by ``ops.sample_`` (sample.hip) from a per-request seed
    and the token's index, so a fixed seed replays the same completion."""
    __slots__ = ("temperature", "top_k", "top_p", "seed")

    def __init__(self, temperature: float = 0.0, top_k: int = 0, top_p: float = 1.0, seed: int | None = None):
        self.temperature = float(temperature)
        self.top_k = int(top_k)
        self.top_p = float(top_p)
        self.seed = int.from_bytes(os.urandom(8), "little") >> 1 if seed is None else int(seed) & ((1 << 63) - 1)

    @property
    def greedy(self) -> bool:
        return not self.temperature >= 1e-4 or self.top_k == 1  # the kernel's own greedy rule (+ top-1)

    def column(self, counter: int) -> list[int]:
        from p2p_llm_tunnel_amd.ops import pack_sampling
        return pack_sampling(0.0 if self.greedy else self.temperature, self.top_k, self.top_p, self.seed, counter)


class SamplingError(ValueError):
    """A request asks for sampling this server does not implement (answered with 400)."""


def _number(src: dict, key: str, lo: float, hi: float, default, integer=False, lo_open=False):
    v = src.get(key)
    if v is None:
        return default
    if isinstance(v, bool) or not isinstance(v, (int, float)) or (integer and isinstance(v, float) and not v.is_integer()):
        raise SamplingError(f"{key} must be {'an integer' if integer else 'a number'}, got {v!r}")
    if not (lo < v if lo_open else lo <= v) or v > hi:
        raise SamplingError(f"{key} must be in {'(' if lo_open else '['}{lo}, {hi}], got {v!r}")
    return int(v) if integer else float(v)


# Parameters that would change which tokens come out and that this server
# does not implement: neutral values pass, anything else is refused instead of
# being silently ignored.
_OPENAI_NEUTRAL = {"n": (1,), "best_of": (1,), "presence_penalty": (0, 0.0), "frequency_penalty": (0, 0.0),
                   "logprobs": (False, 0), "top_logprobs": (0,), "logit_bias": ({},)}
_OLLAMA_NEUTRAL = {"repeat_penalty": (1, 1.0), "presence_penalty": (0, 0.0), "frequency_penalty": (0, 0.0),
                   "mirostat": (0,), "tfs_z": (1, 1.0), "typical_p": (1, 1.0), "min_p": (0, 0.0)}
_MAX_STOPS = 4  # the OpenAI API's limit


def sampling_params(body: dict, ollama: bool, default_temperature: float = 0.0) -> Sampling:
    """Sampling of an OpenAI request (top-level temperature / top_p / seed, and
    the common top_k extension) or an Ollama one ("options"). Raises
    SamplingError for values out of range or parameters not implemented."""
    src = body.get("options", {}) if ollama else body
    if src is None:
        src = {}
    if not isinstance(src, dict):
        raise SamplingError("options must be an object")
    for key, neutral in (_OLLAMA_NEUTRAL if ollama else _OPENAI_NEUTRAL).items():
        if key in src and src[key] is not None and not any(src[key] == x and type(src[key]) is type(x)
                                                            for x in neutral):
            raise SamplingError(f"{key}={src[key]!r} is not supported by this server")
    t = _number(src, "temperature", 0.0, 100.0, default_temperature)
    top_p = _number(src, "top_p", 0.0, 1.0, 1.0, lo_open=True)
    top_k = _number(src, "top_k", 0, 1 << 30, 0, integer=True)
    seed = _number(src, "seed", -(1 << 63), (1 << 64) - 1, None, integer=True)
    return Sampling(t, top_k, top_p, seed)


def stop_sequences(body: dict, ollama: bool) -> list[str]:
    """Stop sequences of an OpenAI request ("stop": null, a string, or a list
    of up to 4 strings) or an Ollama one ("options.stop": a list of strings).
    Empty strings are dropped (they would match at once); anything else that
    is not a string is refused."""
    src = body.get("options", {}) if ollama else body
    if not isinstance(src, dict):
        return []
    v = src.get("stop")
    if v is None:
        return []
    if isinstance(v, str):
        v = [v]
    if not isinstance(v, list) or not all(isinstance(x, str) for x in v):
        raise SamplingError(f"stop must be a string or a list of strings, got {v!r}")
    if len(v) > _MAX_STOPS and not ollama:
        raise SamplingError(f"stop takes at most {_MAX_STOPS} sequences, got {len(v)}")
    return [x for x in v if x]


class StopMatcher:
    """Finds the first stop sequence in a completion's text as pieces arrive.

    ``push(piece)`` returns the text that is safe to emit and whether a stop
    sequence ended the completion (the text up to the match is emitted, the
    match and everything after it are not). A tail that could still be the
    start of a stop sequence is held back until the next piece decides it;
    ``flush()`` releases it when the completion ends for another reason."""
    __slots__ = ("stops", "buf")

    def __init__(self, stops: list[str]):
        self.stops = stops
        self.buf = ""

    def push(self, piece: str) -> tuple[str, bool]:
        buf = self.buf + piece
        hit = -1
        for s in self.stops:
            i = buf.find(s)
            if i >= 0 and (hit < 0 or i < hit):
                hit = i
        if hit >= 0:
            self.buf = ""
            return buf[:hit], True
        keep = 0
        for s in self.stops:
            for k in range(min(len(s) - 1, len(buf)), keep, -1):
                if buf.endswith(s[:k]):
                    keep = k
                    break
        self.buf = buf[len(buf) - keep:] if keep else ""
        return (buf[:len(buf) - keep] if keep else buf), False

    def flush(self) -> str:
        out, self.buf = self.buf, ""
        return out


class Request:
    """A generation request. Tokens go to ``out`` (a queue ending with None)
    unless ``batched`` is set: then the engine's ``deliver`` hook receives them
    together with every other batched request's tokens of the same step."""

    def __init__(self, prompt_ids: list[int], max_new: int, batched: bool = False, sampling: Sampling | None = None):
        self.prompt = prompt_ids
        self.max_new = max_new
        self.out: queue.Queue = queue.Queue()
        self.generated = 0
        self.cancelled = False
        self.batched = batched
        self.sampling = sampling or Sampling()
        self.state = None  # front-end bookkeeping for batched requests


class _StepBuf:
    """Host staging of one in-flight step (two alternate: step k+1 is planned
    and launched while step k runs). Rows: token (prompt rows), position,
    slot, decode flag, slot to record the sampled id under (scratch for rows
    that emit nothing), then the sampler's column per row (rows 5-9:
    temperature bits, top_k, top_p bits, seed, counter; temperature 0 = greedy)."""

    def __init__(self, rows: int, cuda: bool):
        self.h_in = torch.zeros((10, rows), dtype=torch.int64, pin_memory=cuda)
        self.np = self.h_in.numpy()
        self.h_out = torch.zeros(rows, dtype=torch.int64, pin_memory=cuda)
        self.ev = torch.cuda.Event() if cuda else None
        self.n = 0
        self.emits = []  # (row, req, finished, token index)


class Engine:
    """Continuous batching with chunked prefill over the fused decode step,
    one step in flight ahead of the host.

    Every step packs up to ``rows`` (64) token rows: first one decode row per
    generating sequence, then prompt chunks of prefilling sequences, each row
    tagged with its cache slot and position (``TinyLlama.decode_step(slots=)``).
    A 512-byte prompt is thus prefilled in 8 steps instead of 512, while
    generating sequences keep emitting a token every step. Steps of up to 16
    rows replay a 16-row graph, larger ones a 64-row graph; padding rows point
    at the model's scratch slot.

    The schedule never depends on token values (no stop tokens; lengths are
    known), so the host plans step k+1 while step k runs: a decode row's input
    token is read on the device from ``last[slot]``, which every emitting row
    updates after the step, and the sampled ids come back through a pinned
    buffer and an event per step. The host waits on step k (GIL released, so
    the HTTP thread writes meanwhile) only after step k+1 is queued behind it.
    Each step is one hipGraph replay: input copy from pinned staging, decode
    token gather, the fused step, last-token scatter, ids back to pinned
    memory.

    ``model`` injects a model object (tests use a CPU stand-in with the same
    ``decode_step`` / ``cfg`` / ``scratch_slot`` / ``device`` surface).
    """

    def __init__(self, device="cuda:0", config="tiny", max_batch=8, seed=0, use_graph=True, rows=64, model=None,
                 small_rows=16):
        if model is None:
            from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
            model = TinyLlama(config, device=device, max_batch=max_batch, seed=seed, fused=True)
        # hipGraphs need the real fused model on a HIP device (a loaded
        # checkpoint qualifies; CPU stand-ins in tests run eagerly).
        use_graph = use_graph and model.device.type == "cuda" and hasattr(model, "_decode_impl")
        max_batch = getattr(model, "max_batch", max_batch)
        if not (1 <= max_batch <= rows and 1 <= small_rows <= rows):
            raise ValueError("need 1 <= max_batch <= rows and small_rows <= rows")
        self.model = model
        self.device = self.model.device
        self.rows = rows
        self.small_rows = small_rows
        self.use_graph = use_graph
        cuda = self.device.type == "cuda"
        self._k = 0
        self._d_last = torch.zeros(max_batch + 1, dtype=torch.int64, device=self.device)
        self._graphs = {}
        if use_graph:
            # Two row counts: steps of up to 16 rows replay the 16-row graphs,
            # larger ones (prefill-heavy, or more than 16 generating slots) the
            # 64-row graphs (4 MFMA row tiles), whose LM head covers only the
            # leading rows that sample (at most one per slot: max_batch rows).
            # Each graph holds the whole step: input copy from its pinned
            # staging buffer, decode-row token gather, the fused step, the
            # last-token scatter and the copy of the ids back to pinned memory;
            # one per staging buffer of the pair, so a step is one replay.
            sizes = [small_rows] + ([rows] if rows > small_rows else [])
            self._bufs = {R: [_StepBuf(R, cuda), _StepBuf(R, cuda)] for R in sizes}
            self._d_in = {R: torch.zeros((10, R), dtype=torch.int64, device=self.device) for R in sizes}
            # Steps where some row samples replay a graph with the sampler
            # kernel after the fused step; all-greedy steps one without it.
            for R in sizes:
                for par in (0, 1):
                    for smp in (False, True):
                        self._graphs[(R, par, smp)] = self._capture(self._bufs[R][par], R,
                                                                    0 if R == small_rows else max_batch, smp)
        else:
            self._bufs = {rows: [_StepBuf(rows, cuda), _StepBuf(rows, cuda)]}
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
                # max_new is clamped so prompt + generated rows fit max_seq; a
                # prompt too long for the rest keeps its end (for a chat, the
                # latest turns and the generation prompt).
                max_seq = self.model.cfg.max_seq
                req.max_new = max(1, min(req.max_new, max_seq - 2))
                ids = req.prompt[-(max_seq - req.max_new - 1):] or [0]
                self.slots[i] = {"req": req, "pos": 0, "ids": ids, "gen": 0}

    def _plan(self, batch: list):
        """Rows of the next step [(slot, token, pos, is_decode, emits)], with the
        host-side state advanced past them (it does not depend on the tokens)
        and the emitting rows' (row, req, finished) list."""
        V = self.model.cfg.vocab
        rows, emits = [], []
        for i, s in enumerate(self.slots):  # decode rows first: one token each
            if s is None or s["pos"] < len(s["ids"]):
                continue
            if s["req"].cancelled:
                self._emit(s["req"], None, batch)
                self.slots[i] = None
                continue
            rows.append((i, 0, s["pos"], 1, True))
        for i, s in enumerate(self.slots):  # then prompt chunks
            if s is None or s["pos"] >= len(s["ids"]):
                continue
            take = min(self.rows - len(rows), len(s["ids"]) - s["pos"])
            for p in range(s["pos"], s["pos"] + take):
                rows.append((i, s["ids"][p] % V, p, 0, p == len(s["ids"]) - 1))
            if len(rows) >= self.rows:
                break
        # Rows that sample go first: the 64-row graph's LM head covers only the
        # first max_batch rows (each slot samples at most once per step).
        rows.sort(key=lambda r: not r[4])
        # Advance every row's slot first: after the sort a slot's sampling row
        # can precede its other prompt rows, so slots are only freed once all
        # rows of the step are accounted for.
        max_seq = self.model.cfg.max_seq
        for i, _, _, _, emit in rows:
            self.slots[i]["pos"] += 1
            if not emit:
                self.prefill_tokens += 1
        done = []
        for r, (i, _, _, _, emit) in enumerate(rows):
            if not emit:
                continue
            s = self.slots[i]
            s["gen"] += 1
            fin = s["gen"] >= s["req"].max_new or s["pos"] >= max_seq - 1
            emits.append((r, s["req"], fin, s["gen"] - 1))  # the token's index: the sampler's counter
            if fin:
                done.append(i)
        for i in done:
            self.slots[i] = None
        return rows, emits

    def _step_body(self, b: _StepBuf, R: int, emit_rows: int, sample: bool = False):
        """The captured step: staging -> device, token gather, fused step,
        (the sampler over the emitting rows' logits,) last-token scatter, ids
        -> pinned staging."""
        d = self._d_in[R]
        d.copy_(b.h_in, non_blocking=True)
        tok = torch.where(d[3] != 0, self._d_last[d[2]], d[0])
        S = self.model.cfg.max_seq
        ids, logits = self.model._decode_impl(tok, d[1].to(torch.int32), (0, S - 1), S, d[2].to(torch.int32),
                                              emit_rows)
        if sample:
            from p2p_llm_tunnel_amd import ops
            n = emit_rows or R
            ops.sample_(logits[:n], ids[:n], d[5:10])
        self._d_last.index_copy_(0, d[4], ids)
        b.h_out.copy_(ids, non_blocking=True)

    def _capture(self, b: _StepBuf, R: int, emit_rows: int, sample: bool = False):
        scratch = self.model.scratch_slot
        b.np[:] = 0
        b.np[2, :] = scratch  # warm-up and capture touch the scratch slot only
        b.np[4, :] = scratch
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(2):  # allocator + kernel warm-up outside capture
                self._step_body(b, R, emit_rows, sample)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(graph):
            self._step_body(b, R, emit_rows, sample)
        torch.cuda.synchronize(self.device)
        return graph

    def _launch(self, rows, emits) -> _StepBuf:
        n, scratch = len(rows), self.model.scratch_slot
        if self.use_graph:
            R = self.small_rows if n <= self.small_rows else self.rows
        else:
            R = self.rows
        par = self._k % 2
        self._k += 1
        b = self._bufs[R][par]
        h = b.np
        h[0, :n] = [r[1] for r in rows]
        h[1, :n] = [r[2] for r in rows]
        h[2, :n] = [r[0] for r in rows]
        h[3, :n] = [r[3] for r in rows]
        h[4, :n] = [r[0] if r[4] else scratch for r in rows]
        h[5:10, :] = 0  # greedy unless an emitting row samples
        sample = False
        for r, req, _, ctr in emits:
            if not req.sampling.greedy:
                h[5:10, r] = req.sampling.column(ctr)
                sample = True
        if n < R:  # padding rows: scratch slot, nothing recorded
            h[0:2, n:R] = 0
            h[2, n:R] = scratch
            h[3, n:R] = 0
            h[4, n:R] = scratch
        b.n, b.emits = n, emits
        if self.use_graph:
            self._graphs[(R, par, sample)].replay()
        else:  # injected model (tests): the same step, eagerly, on its n rows
            d = b.h_in.to(self.device)
            tok = torch.where(d[3, :n] != 0, self._d_last[d[2, :n]], d[0, :n])
            lo, hi = min(r[2] for r in rows), max(r[2] for r in rows)
            ids = self.model.decode_step(tok, d[1, :n].to(torch.int32), (lo, hi), slots=d[2, :n].to(torch.int32))
            self._d_last.index_copy_(0, d[4, :n], ids.to(torch.int64))
            b.h_out[:n].copy_(ids)
        if b.ev is not None:
            b.ev.record()
        self.steps += 1
        return b

    def _drain(self, b: _StepBuf, batch: list):
        if b.ev is not None:
            b.ev.synchronize()  # GIL released: the HTTP thread writes meanwhile
        out = b.h_out[: b.n].tolist() if b.emits else []
        for r, req, fin, _ in b.emits:
            if req.cancelled:
                continue
            self._emit(req, out[r], batch)
            req.generated += 1
            self.tokens_out += 1
            if fin:
                self._emit(req, None, batch)

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        inflight: list[_StepBuf] = []
        with torch.no_grad():
            while not self._stop.is_set():
                batch = []
                self._admit()
                rows, emits = self._plan(batch)
                if rows:
                    inflight.append(self._launch(rows, emits))
                if inflight and (len(inflight) >= 2 or not rows):
                    self._drain(inflight.pop(0), batch)
                if batch:
                    self._flush(batch)
                # Hand the GIL over once per step: when the host is the slower
                # side the event wait above returns at once, and the HTTP thread
                # (accepting a burst of new connections, say) would otherwise get
                # the GIL only at the interpreter's forced-switch interval.
                time.sleep(0)
                if not rows and not inflight:
                    self._wake.wait(0.05)
                    self._wake.clear()

    def _emit(self, req: Request, tok, batch: list):
        if req.batched and self.deliver is not None:
            batch.append((req, tok))
        else:
            req.out.put(tok)

    def _flush(self, batch: list):
        if self.deliver is not None:
            self.deliver(batch)


def _prompt_ids(body: dict, tok=None) -> list[int]:
    msgs = body.get("messages")
    if tok is not None:
        if isinstance(msgs, list):
            return tok.chat([m for m in msgs if isinstance(m, dict)]) or [0]
        return tok.encode(str(body.get("prompt", ""))) or [0]
    if "messages" in body:
        text = "\n".join(str(m.get("content", "")) for m in body.get("messages", []) if isinstance(m, dict))
    else:
        text = str(body.get("prompt", ""))
    return list(text.encode("utf-8"))[:512] or [1]


def _piece(text: str) -> bytes:
    """A text piece as the inside of a JSON string."""
    return json.dumps(text, ensure_ascii=False)[1:-1].encode()


def _chunk(data: bytes) -> bytes:
    return b"%x\r\n%s\r\n" % (len(data), data)


class _Stream:
    """Per-request output state on the I/O thread: the writer and the byte
    template around each token piece (token ids render as " t<id>": no JSON
    escaping needed)."""
    __slots__ = ("writer", "stream", "kind", "rid", "pre", "post", "toks", "done", "detok", "reason", "stop",
                 "stop_hit")

    def __init__(self, writer, stream, kind, rid, model, detok=None, stop=None):
        self.writer = writer
        self.stream = stream
        self.kind = kind  # "chat" | "text" | "ollama"
        self.rid = rid
        self.toks = []  # non-streamed: rendered pieces (bytes, JSON-escaped when detokenised)
        self.detok = detok  # checkpoint tokenizer: incremental text of this request
        self.reason = "length"
        self.stop = stop  # StopMatcher, or None without stop sequences
        self.stop_hit = False  # a stop sequence matched (its held-back text is the match, never emitted)
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

    def __init__(self, engine: Engine, host: str, port: int, model_name: str, tokenizer=None,
                 default_temperature: float = 0.0):
        self.engine = engine
        self.model_name = model_name
        # Temperature of requests that give none. 0 (greedy) by default — the
        # OpenAI API's nominal default is 1 — so unparameterised completions
        # stay deterministic; --default-temperature sets it.
        self.default_temperature = default_temperature
        self.tok = tokenizer
        self.eos = tokenizer.eos_ids if tokenizer is not None else frozenset()
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
        # Stopped: cancel the keep-alive connection tasks still parked in a
        # read and let them unwind, so none is destroyed while pending.
        pending = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
        for t in pending:
            t.cancel()
        if pending:
            self.loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))

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
                continue
            if tok in self.eos:  # stop: the engine frees the slot on its next step
                req.cancelled = True
                st.reason = "stop"
                self._finish(req, st)
                continue
            if st.stop is not None:
                piece = st.detok.push(tok) if st.detok is not None else " t%d" % tok
                text, stopped = st.stop.push(piece)
                if text:
                    self._emit_piece(st, _piece(text))
                if stopped:  # the engine frees the slot on its next step
                    req.cancelled = True
                    st.reason = "stop"
                    st.stop_hit = True
                    self._finish(req, st)
                continue
            if st.detok is not None:
                piece = st.detok.push(tok)
                if not piece:
                    continue
                body = _piece(piece)
            else:
                body = b" t%d" % tok
            self._emit_piece(st, body)

    @staticmethod
    def _emit_piece(st, body: bytes):
        if st.stream:
            st.writer.write(_chunk(st.pre + body + st.post))
        else:
            st.toks.append(body)

    def _finish(self, req, st):
        w = st.writer
        if st.stop is not None and not st.stop_hit:
            # A held-back tail that never became a stop sequence: the completion
            # ended otherwise (length, EOS — also finish_reason "stop"), so it is
            # real text.
            held = st.stop.flush()
            if held:
                self._emit_piece(st, _piece(held))
        if st.stream:
            if st.kind == "ollama":
                tail = _chunk((json.dumps({"model": self.model_name, "response": "", "done": True}) + "\n").encode())
            else:
                fin = {"index": 0, "delta": {}, "finish_reason": st.reason} if st.kind == "chat" else \
                    {"index": 0, "text": "", "finish_reason": st.reason}
                obj = {"id": st.rid, "object": "chat.completion.chunk" if st.kind == "chat" else "text_completion",
                       "choices": [fin]}
                tail = _chunk(f"data: {json.dumps(obj)}\n\n".encode()) + _chunk(b"data: [DONE]\n\n")
            w.write(tail + b"0\r\n\r\n")
        else:
            text = json.loads(b'"' + b"".join(st.toks) + b'"')
            if st.kind == "ollama":
                obj = {"model": self.model_name, "response": text, "done": True}
            elif st.kind == "chat":
                obj = {"id": st.rid, "object": "chat.completion", "model": self.model_name,
                       "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                    "finish_reason": st.reason}],
                       "usage": {"prompt_tokens": len(req.prompt), "completion_tokens": req.generated,
                                 "total_tokens": len(req.prompt) + req.generated}}
            else:
                obj = {"id": st.rid, "object": "text_completion", "model": self.model_name,
                       "choices": [{"index": 0, "text": text, "finish_reason": st.reason}]}
            w.write(self._json_response(obj))
        st.done.set_result(True)

    # ---------------------------------------------------------------- HTTP
    @staticmethod
    def _response(status: int, ctype: str, body: bytes, reason: str = "OK") -> bytes:
        return (b"HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n\r\n"
                % (status, reason.encode(), ctype.encode(), len(body))) + body

    def _json_response(self, obj, status=200) -> bytes:
        reason = {200: "OK", 400: "Bad Request", 404: "Not Found"}.get(status, "Error")
        return self._response(status, "application/json", json.dumps(obj).encode(), reason)

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
        raw_max = req_body.get("max_tokens", req_body.get("num_predict", 16))
        try:
            max_new = int(raw_max if raw_max is not None else 16)
        except (TypeError, ValueError):
            writer.write(self._json_response({"error": f"max_tokens must be an integer, got {raw_max!r}"}, 400))
            return True
        ollama = path == "/api/generate"
        kind = "ollama" if ollama else ("chat" if "chat" in path else "text")
        try:
            sampling = sampling_params(req_body, ollama, self.default_temperature)
            stops = stop_sequences(req_body, ollama)
            if not sampling.greedy and not self.engine.use_graph:
                # The eager step (CPU stand-ins, injected models) has no sampler:
                # refuse rather than answer a sampled request greedily.
                raise SamplingError("sampling (temperature > 0) needs the graph-captured HIP step; "
                                    "this engine runs eagerly")
        except SamplingError as e:
            writer.write(self._json_response({"error": {"message": str(e), "type": "invalid_request_error"}}, 400))
            return True
        stream = bool(req_body.get("stream", ollama))
        rid = ("chatcmpl-" if kind == "chat" else "cmpl-") + uuid.uuid4().hex[:12]
        prompt = _prompt_ids(req_body, self.tok)
        req = Request(prompt, max(1, min(max_new, 1024)), batched=True, sampling=sampling)
        st = _Stream(writer, stream, kind, rid, name, self.tok.detokenizer(prompt) if self.tok is not None else None,
                     StopMatcher(stops) if stops else None)
        req.state = st
        if stream:
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: %s\r\nCache-Control: no-cache\r\n"
                         b"Transfer-Encoding: chunked\r\n\r\n"
                         % (b"application/x-ndjson" if ollama else b"text/event-stream"))
        self.engine.submit(req)
        return await st.done


def start_server(host="127.0.0.1", port=0, device="cuda:0", config="tiny", max_batch=8, model_name=None,
                 engine: Engine | None = None, checkpoint: str | None = None, max_seq: int | None = None,
                 tokenizer=None, default_temperature: float = 0.0):
    """Engine + HTTP front-end; returns (server, port, engine). ``server.shutdown()``
    stops the HTTP side, ``engine.stop()`` the GPU side. ``checkpoint``: serve a
    Hugging Face Llama checkpoint directory (weights + tokenizer) instead of
    the random-init ``config``. ``tokenizer`` (a ``checkpoint.Tokenizer``)
    overrides the checkpoint's own or gives an injected engine a text side."""
    sys.setswitchinterval(0.0005)  # two busy threads: bound a GIL wait at 0.5 ms, not 5
    tok = tokenizer
    if checkpoint and engine is None:
        import os
        from p2p_llm_tunnel_amd.models.checkpoint import Tokenizer, load_llama
        model = load_llama(checkpoint, device=device, max_batch=max_batch, max_seq=max_seq)
        tok = tok or Tokenizer.for_checkpoint(checkpoint)
        engine = Engine(device=device, max_batch=max_batch, model=model)
        model_name = model_name or os.path.basename(os.path.normpath(checkpoint))
    engine = engine or Engine(device=device, config=config, max_batch=max_batch)
    srv = FrontEnd(engine, host, port, model_name or f"p2pt-{config}", tokenizer=tok,
                   default_temperature=default_temperature)
    return srv, srv.server_address[1], engine


def _replicas(a) -> int:
    """--gpus N: one endpoint process per GPU on ports port..port+N-1 (data-
    parallel replicas: the model fits one MI355X many times over, so replicas
    scale throughput with no cross-GPU traffic). `tunnel serve --upstream`
    takes the printed comma-separated list and balances requests over them by
    fewest in flight. Each child is a fresh interpreter pinned to its device;
    the parent never touches the GPU and exits with the first child that dies."""
    import subprocess
    base = a.port
    procs = []
    for i in range(a.gpus):
        cmd = [sys.executable, "-m", "p2p_llm_tunnel_amd.models.server", "--host", a.host, "--port", str(base + i),
               "--device", f"cuda:{i}", "--config", a.config, "--max-batch", str(a.max_batch)]
        if a.checkpoint:
            cmd += ["--checkpoint", a.checkpoint] + (["--max-seq", str(a.max_seq)] if a.max_seq else [])
        cmd += ["--default-temperature", str(a.default_temperature)]
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
    ap.add_argument("--checkpoint", default=None,
                    help="Hugging Face Llama checkpoint directory (config.json, *.safetensors, tokenizer.json)")
    ap.add_argument("--max-seq", type=int, default=None, help="KV-cache length per slot (checkpoint default: "
                    "min(max_position_embeddings, 8192))")
    ap.add_argument("--gpus", type=int, default=0,
                    help="spawn one endpoint per GPU (cuda:0..N-1) on consecutive ports instead of serving here")
    ap.add_argument("--default-temperature", type=float, default=0.0,
                    help="temperature of requests that set none (0: greedy; requests may set temperature, top_p, "
                         "top_k, seed)")
    a = ap.parse_args(argv)
    if a.gpus > 0:
        raise SystemExit(_replicas(a))
    srv, port, engine = start_server(a.host, a.port, a.device, a.config, a.max_batch, checkpoint=a.checkpoint,
                                     max_seq=a.max_seq, default_temperature=a.default_temperature)
    print(f"inference endpoint on http://{a.host}:{port} ({a.checkpoint or a.config}, {a.device})", flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        engine.stop()


if __name__ == "__main__":
    main()
