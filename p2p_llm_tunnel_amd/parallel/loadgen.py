"""Asyncio load generator for streamed (SSE) completions.

Each *stream* is one client connection issuing back-to-back
``POST /v1/chat/completions {"stream": true}`` requests (keep-alive), the
multiplexing dimension of the tunnel. A *step* is one
request on every stream, all in flight together; the step ends when the last
response completes. TTFT is measured from just before the request bytes are
written to the arrival of the first ``data:`` line.
"""
from __future__ import annotations

import asyncio
import json
import statistics
import time
from dataclasses import dataclass, field

BODY = json.dumps({"model": "test-model", "stream": True,
                   "messages": [{"role": "user", "content": "hi"}]}).encode()


@dataclass
class StepStats:
    ttft_s: list = field(default_factory=list)
    total_s: list = field(default_factory=list)
    events: int = 0
    errors: int = 0


class SseStream:
    def __init__(self, host: str, port: int, path: str = "/v1/chat/completions", body: bytes = BODY):
        self.host, self.port, self.path, self.body = host, port, path, body
        self.reader = self.writer = None

    async def _connect(self):
        self.reader, self.writer = await asyncio.open_connection(self.host, self.port)

    async def close(self):
        if self.writer:
            self.writer.close()
            try:
                await self.writer.wait_closed()
            except Exception:
                pass
            self.writer = None

    async def request(self, stats: StepStats):
        if self.writer is None:
            await self._connect()
        req = (f"POST {self.path} HTTP/1.1\r\nHost: {self.host}:{self.port}\r\n"
               f"Content-Type: application/json\r\nContent-Length: {len(self.body)}\r\n\r\n").encode() + self.body
        t0 = time.perf_counter()
        self.writer.write(req)
        r = self.reader
        status = await r.readline()
        if not status.startswith(b"HTTP/1.1 200") and not status.startswith(b"HTTP/1.0 200"):
            stats.errors += 1
            await self.close()
            return
        chunked = False
        length = None
        keep = status.startswith(b"HTTP/1.1")
        while True:
            line = await r.readline()
            if line in (b"\r\n", b"\n", b""):
                break
            k, _, v = line.decode("latin-1").partition(":")
            k = k.strip().lower()
            v = v.strip().lower()
            if k == "transfer-encoding" and "chunked" in v:
                chunked = True
            elif k == "content-length":
                length = int(v)
            elif k == "connection" and v == "close":
                keep = False
        first = None
        n_events = 0
        buf = b""

        def scan(data: bytes):
            nonlocal first, n_events, buf
            buf += data
            while b"\n\n" in buf:
                ev, buf = buf.split(b"\n\n", 1)
                if ev.startswith(b"data: "):
                    if first is None:
                        first = time.perf_counter()
                    n_events += 1

        if chunked:
            while True:
                size_line = await r.readline()
                size = int(size_line.split(b";")[0].strip() or b"0", 16)
                if size == 0:
                    await r.readline()
                    break
                data = await r.readexactly(size)
                await r.readexactly(2)
                scan(data)
        elif length is not None:
            scan(await r.readexactly(length))
        else:
            while True:
                d = await r.read(65536)
                if not d:
                    break
                scan(d)
            keep = False
        t1 = time.perf_counter()
        if first is None:
            stats.errors += 1
        else:
            stats.ttft_s.append(first - t0)
            stats.total_s.append(t1 - t0)
            stats.events += n_events
        if not keep:
            await self.close()


async def run_steps(host: str, port: int, streams: int, steps: int, between=None) -> tuple[float, StepStats]:
    """Run `steps` steps of `streams` concurrent requests; returns (seconds, stats)."""
    conns = [SseStream(host, port) for _ in range(streams)]
    stats = StepStats()
    t0 = time.perf_counter()
    for _ in range(steps):
        await asyncio.gather(*(c.request(stats) for c in conns))
    dt = time.perf_counter() - t0
    for c in conns:
        await c.close()
    return dt, stats


def pct(xs, q):
    if not xs:
        return float("nan")
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))
    return xs[k]


def summarize(stats: StepStats) -> dict:
    return {
        "p50_ttft_ms": pct(stats.ttft_s, 50) * 1e3,
        "p99_ttft_ms": pct(stats.ttft_s, 99) * 1e3,
        "mean_ttft_ms": (statistics.fmean(stats.ttft_s) * 1e3) if stats.ttft_s else float("nan"),
        "p50_total_ms": pct(stats.total_s, 50) * 1e3,
        "requests": len(stats.ttft_s),
        "errors": stats.errors,
    }
