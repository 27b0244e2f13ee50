"""Randomised concurrent traffic through one tunnel with worker threads: SSE
streams read fully or abandoned mid-stream, echoed uploads of random size
(some above the 8 MiB streaming threshold), downloads read slowly or dropped,
requests for missing routes, all at once from many clients. Afterwards the
tunnel must still serve, and both sides must have released every stream
(in-flight and paused gauges back to zero) — the state that the worker
hand-offs, per-stream pauses, credit and cancellation all touch.

Run it against sanitizer builds with P2PT_BIN_DIR=build-tsan/bin (or asan)."""
import http.client
import json
import os
import random
import socket
import threading
import time
import urllib.request

import pytest

from p2p_llm_tunnel_amd import binary
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn

DURATION_S = float(os.environ.get("CHAOS_SECONDS", "12"))


def _gauges(port):
    text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    out = {}
    for line in text.splitlines():
        p = line.split()
        if len(p) == 2 and not line.startswith("#"):
            try:
                out[p[0]] = float(p[1])
            except ValueError:
                pass
    return out


def _sse(port, rng, stats):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True, "messages": []}),
              headers={"content-type": "application/json"})
    r = c.getresponse()
    assert r.status == 200
    if rng.random() < 0.4:  # abandon after the first event
        r.read1(64)
        c.sock.shutdown(socket.SHUT_RDWR)
        c.close()
        stats["sse_abandoned"] += 1
        return
    data = r.read()
    assert data.rstrip().endswith(b"data: [DONE]"), data[-200:]
    stats["sse_ok"] += 1


def _echo(port, rng, stats):
    n = rng.choice([0, 1, 1000, 65408, 65409, 300_000, 2_000_000] + ([9_000_000] if rng.random() < 0.08 else []))
    body = rng.randbytes(n)
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", "/echo", body=body)
    r = c.getresponse()
    got = r.read()
    assert r.status == 200 and got == body, (n, len(got))
    c.close()
    stats["echo_ok"] += 1


def _bulk(port, rng, stats):
    n = rng.choice([1 << 16, 1 << 20, 8 << 20])
    s = socket.create_connection(("127.0.0.1", port), timeout=30)
    s.sendall(b"GET /bulk?bytes=%d HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n" % n)
    got, slow, drop_at = 0, rng.random() < 0.3, (n // 3 if rng.random() < 0.3 else None)
    while True:
        if slow:
            time.sleep(0.002)
        d = s.recv(65536)
        if not d:
            break
        got += len(d)
        if drop_at is not None and got > drop_at:
            s.close()
            stats["bulk_dropped"] += 1
            return
    s.close()
    assert got > n, (got, n)  # headers + body
    stats["bulk_ok"] += 1


def _missing(port, rng, stats):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    c.request("GET", "/nope/%d" % rng.randrange(1000))
    r = c.getresponse()
    r.read()
    assert r.status == 404
    stats["missing_ok"] += 1


@pytest.mark.parametrize("workers", ["2", "0"])
def test_chaos_traffic_drains(workers):
    mport = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(mport), "--interval-ms", "20", "--tokens", "20",
                          "--threads", "2"])
    mock.wait_for("Mock LLM server running", 10)
    sm, pm = free_port(), free_port()
    try:
        with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc",
                    serve_extra=[f"--workers={workers}", "--inline-streams=2", "--metrics-listen", f"127.0.0.1:{sm}"],
                    proxy_extra=[f"--workers={workers}", "--inline-streams=2",
                                 "--metrics-listen", f"127.0.0.1:{pm}"]) as t:
            stats = {k: 0 for k in ("sse_ok", "sse_abandoned", "echo_ok", "bulk_ok", "bulk_dropped", "missing_ok")}
            errors = []
            lock = threading.Lock()
            stop = time.time() + DURATION_S

            def client(seed):
                rng = random.Random(seed)
                local = {k: 0 for k in stats}
                while time.time() < stop:
                    op = rng.choices([_sse, _echo, _bulk, _missing], weights=[5, 3, 2, 1])[0]
                    try:
                        op(t.proxy_port, rng, local)
                    except Exception as e:  # noqa: BLE001 - collected and asserted below
                        errors.append(f"{op.__name__}: {e!r}")
                        return
                with lock:
                    for k, v in local.items():
                        stats[k] += v

            ts = [threading.Thread(target=client, args=(i,)) for i in range(24)]
            for th in ts:
                th.start()
            for th in ts:
                th.join(DURATION_S + 120)
            assert not errors, errors[:5]
            assert stats["sse_ok"] > 20 and stats["sse_abandoned"] > 5 and stats["echo_ok"] > 10, stats
            # The tunnel still serves, and every stream is released on both sides.
            st, _, body = (lambda r: (r.status, None, r.read()))(
                urllib.request.urlopen(f"http://127.0.0.1:{t.proxy_port}/health", timeout=10))
            assert st == 200 and body == b"ok"
            deadline = time.time() + 15
            while True:
                g = [_gauges(sm), _gauges(pm)]
                busy = [(x.get("tunnel_streams_inflight"), x.get("tunnel_streams_paused")) for x in g]
                if all(a == 0 and b == 0 for a, b in busy) or time.time() > deadline:
                    break
                time.sleep(0.2)
            assert all(a == 0 and b == 0 for a, b in busy), busy
            assert t.serve.popen.poll() is None and t.proxy.popen.poll() is None
    finally:
        mock.stop()
