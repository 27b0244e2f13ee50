"""Per-stream flow control ("flow" extension) and bounded request bodies.

The reference has no flow control (unbounded queues) and
buffers whole request bodies on serve (reference serve.rs:120-139). Here:

* "flow" is negotiated in HELLO/AGREE like "cancel": with it, each stream and
  direction starts with proto::kFlowWindow (256 KiB) of body credit and the
  receiver hands consumed bytes back in CREDIT frames (type 14); without it
  (a reference peer) nothing changes on the wire;
* a slow HTTP client therefore pauses just its own upstream read on serve,
  and the proxy's memory stays bounded;
* request bodies above 8 MiB stream to the upstream as they arrive (credit
  returned as the upstream takes them), so a 1 GiB upload keeps serve small;
  --max-request-body answers 413.
"""
import http.client
import json
import os
import socket
import struct
import threading
import time
import urllib.request

import numpy as np
import pytest

from p2p_llm_tunnel_amd import binary
from p2p_llm_tunnel_amd.utils import framepeer as fp
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn

WINDOW = 256 * 1024


def _native_mock():
    port = free_port()
    p = spawn("mock", [binary("tunnel-mock"), "--port", str(port)])
    p.wait_for("Mock LLM server running", 10)
    return p, port


def _serve(upstream, extra=(), env=None):
    port = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", upstream,
                           "--transport", f"tcp-listen:127.0.0.1:{port}", "--max-retries", "0", *extra],
                 env=dict({"RUST_LOG": "info"}, **(env or {})))
    proc.wait_for("tcp transport: listening", 10)
    return proc, fp.FramePeer.connect(port)


def _handshake(peer, features):
    peer.send_json(fp.HELLO, 0, {"proto": "httptunnel", "min_version": 1, "max_version": 1, "features": features})
    t, _, p = peer.recv_until(lambda t, s, p: t == fp.AGREE)
    return json.loads(p)


def _drain_body(peer, sid, quiet=0.5):
    """RES_BODY bytes that arrive until the stream goes quiet (or ends)."""
    n, ended = 0, False
    while True:
        try:
            t, s, p = peer.recv_until(lambda t, s, p: s == sid, timeout=quiet)
        except (socket.timeout, TimeoutError):
            return n, ended
        if t == fp.RES_BODY:
            n += len(p)
        elif t == fp.RES_END:
            return n, True


# Sanitizer builds (P2PT_BIN_DIR=build-tsan/bin, ...) carry shadow memory: the
# RSS bounds below are scaled for them, the behaviour checks are not.
RSS_SCALE = 4 if "san" in os.path.basename(os.path.dirname(os.environ.get("P2PT_BIN_DIR", "").rstrip("/"))) else 1


def _rss_kb(pid, field="VmRSS"):
    for line in open(f"/proc/{pid}/status"):
        if line.startswith(field + ":"):
            return int(line.split()[1])
    return 0


@pytest.mark.parametrize("flow", [True, False])
def test_serve_res_body_waits_for_credit(flow):
    mock, mport = _native_mock()
    proc, peer = _serve(f"http://127.0.0.1:{mport}")
    try:
        agree = _handshake(peer, ["sse", "flow"] if flow else ["sse"])
        assert ("flow" in agree["features"]) == flow
        total = 3_000_000
        peer.send_json(fp.REQ_HEADERS, 1, {"stream_id": 1, "method": "GET", "path": f"/bulk?bytes={total}",
                                          "headers": {}})
        peer.send(fp.REQ_END, 1)
        peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
        got, ended = _drain_body(peer, 1)
        if not flow:  # reference behaviour: everything flows, no CREDIT involved
            while not ended:
                n, ended = _drain_body(peer, 1)
                got += n
            assert got == total
            return
        # out of credit after the window (plus at most one upstream read in flight)
        assert WINDOW <= got <= WINDOW + 2 * 65536 and not ended, got
        granted = 0
        while not ended:
            peer.send(fp.CREDIT, 1, struct.pack(">I", 200_000))
            granted += 200_000
            n, ended = _drain_body(peer, 1, quiet=0.3)
            got += n
            assert got <= WINDOW + granted + 2 * 65536
        assert got == total
    finally:
        peer.close()
        proc.stop()
        mock.stop()


def test_serve_streams_large_upload_and_grants_credit():
    mock, mport = _native_mock()
    proc, peer = _serve(f"http://127.0.0.1:{mport}")
    try:
        _handshake(peer, ["sse", "flow"])
        data = np.random.default_rng(1).integers(0, 256, 12 << 20, dtype=np.uint8).tobytes()
        peer.send_json(fp.REQ_HEADERS, 3, {"stream_id": 3, "method": "POST", "path": "/sink",
                                          "headers": {"content-length": str(len(data))}})
        credit, sent = WINDOW, 0
        while sent < len(data):
            while credit <= 0:  # honour serve's credit like our proxy does
                t, s, p = peer.recv_until(lambda t, s, p: t == fp.CREDIT and s == 3, timeout=10)
                credit += struct.unpack(">I", p)[0]
            piece = data[sent:sent + 65408]
            peer.send(fp.REQ_BODY, 3, piece)
            sent += len(piece)
            credit -= len(piece)
        peer.send(fp.REQ_END, 3)
        t, s, p = peer.recv_until(lambda t, s, p: t == fp.RES_BODY and s == 3, timeout=20)
        res = json.loads(p)
        w = np.arange(1, len(data) + 1, dtype=np.uint64) * np.frombuffer(data, dtype=np.uint8).astype(np.uint64)
        assert res["bytes"] == len(data) and res["wsum"] == int(w.sum(dtype=np.uint64))
    finally:
        peer.close()
        proc.stop()
        mock.stop()


def test_serve_413_above_max_request_body(mock_upstream):
    proc, peer = _serve(mock_upstream, extra=("--max-request-body", "100000"))
    try:
        _handshake(peer, ["sse"])
        peer.send_json(fp.REQ_HEADERS, 1, {"stream_id": 1, "method": "POST", "path": "/echo",
                                          "headers": {"content-length": "200000"}})
        t, s, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
        assert json.loads(p)["status"] == 413
        # undeclared length: rejected once the received body passes the limit
        peer.send_json(fp.REQ_HEADERS, 2, {"stream_id": 2, "method": "POST", "path": "/echo", "headers": {}})
        for _ in range(3):
            peer.send(fp.REQ_BODY, 2, b"x" * 60000)
        t, s, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS and s == 2)
        assert json.loads(p)["status"] == 413
        peer.send(fp.REQ_END, 2)
        # a body under the limit still goes through
        peer.send_json(fp.REQ_HEADERS, 3, {"stream_id": 3, "method": "POST", "path": "/echo", "headers": {}})
        peer.send(fp.REQ_BODY, 3, b"y" * 50000)
        peer.send(fp.REQ_END, 3)
        t, s, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS and s == 3)
        assert json.loads(p)["status"] == 200
    finally:
        peer.close()
        proc.stop()


@pytest.fixture
def flow_proxy():
    srv = fp.FramePeer.listen()
    port = srv.getsockname()[1]
    http_port = free_port()
    proc = spawn("proxy", [binary("tunnel"), "proxy", "--room", "x", "--listen", f"127.0.0.1:{http_port}",
                           "--transport", f"tcp-connect:127.0.0.1:{port}"], env={"RUST_LOG": "info"})
    conn, _ = srv.accept()
    peer = fp.FramePeer(conn)
    t, sid, p = peer.recv()
    assert t == fp.HELLO and "flow" in json.loads(p)["features"]
    peer.send_json(fp.AGREE, 0, {"version": 1, "features": ["sse", "cancel", "flow"]})
    proc.wait_for("proxy listening", 5)
    yield peer, proc, http_port
    peer.close()
    proc.stop()
    srv.close()


def test_proxy_upload_waits_for_credit_and_grants_download_credit(flow_proxy):
    peer, proc, port = flow_proxy
    body = bytes(range(256)) * 8192  # 2 MiB
    out = {}

    def run():
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        c.request("POST", "/up", body=body)
        r = c.getresponse()
        out["status"], out["body"] = r.status, r.read()

    th = threading.Thread(target=run)
    th.start()
    peer.recv_until(lambda t, s, p: t == fp.REQ_HEADERS)
    got = b""

    def take(quiet):
        nonlocal got
        while True:
            try:
                t, s, p = peer.recv_until(lambda t, s, p: True, timeout=quiet)
            except (socket.timeout, TimeoutError):
                return False
            if t == fp.REQ_END:
                return True
            assert t == fp.REQ_BODY
            got += p

    assert not take(0.5)
    assert WINDOW <= len(got) <= WINDOW + 2 * 65536, len(got)  # the proxy stopped reading its client
    done = False
    while not done:
        peer.send(fp.CREDIT, 1, struct.pack(">I", 512 * 1024))
        done = take(0.3)
    assert got == body
    # download: the proxy grants RES_BODY credit as its client consumes it
    peer.send_json(fp.RES_HEADERS, 1, {"stream_id": 1, "status": 200, "headers": {}})
    blob = b"z" * 65408
    for _ in range(32):  # 2 MiB, sent regardless of credit (a scripted peer)
        peer.send(fp.RES_BODY, 1, blob)
    granted = 0
    deadline = time.time() + 10
    while granted < 32 * 65408 - 64 * 1024 and time.time() < deadline:
        t, s, p = peer.recv_until(lambda t, s, p: t == fp.CREDIT, timeout=5)
        granted += struct.unpack(">I", p)[0]
    # Consumed bytes come back as credit, plus the window's growth: a reader
    # that takes whole windows fast doubles it (receiver-side autotuning,
    # 256 KiB -> at most 8 MiB), so the grants may exceed what was consumed
    # by at most that growth.
    assert 32 * 65408 - 64 * 1024 <= granted <= 32 * 65408 + (8 << 20) - (256 << 10)
    peer.send(fp.RES_END, 1)
    th.join(10)
    assert out["status"] == 200 and len(out["body"]) == 32 * 65408


@pytest.mark.parametrize("features", [None, "sse,cancel"])
def test_slow_client_bounds_proxy_memory(features):
    """One client stops reading a 96 MB download: with "flow" the proxy holds
    about one window for it; a reference-style peer pair (no "flow") buffers
    the download in the proxy, as the reference would."""
    mock, mport = _native_mock()
    env = {"TUNNEL_FEATURES": features} if features else None
    ms = free_port()
    try:
        with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc", env=env,
                    serve_extra=["--metrics-listen", f"127.0.0.1:{ms}"]) as t:
            base = _rss_kb(t.proxy.popen.pid)
            s = socket.create_connection(("127.0.0.1", t.proxy_port))
            s.sendall(b"GET /bulk?bytes=100000000 HTTP/1.1\r\nHost: x\r\n\r\n")
            head = s.recv(65536)
            assert head.startswith(b"HTTP/1.1 200")
            time.sleep(2.0)  # the client reads nothing
            grown = _rss_kb(t.proxy.popen.pid) - base
            m = urllib.request.urlopen(f"http://127.0.0.1:{ms}/metrics", timeout=5).read().decode()
            stalls = [float(l.split()[1]) for l in m.splitlines() if l.startswith("tunnel_stream_credit_stalls_total")]
            if features is None:
                assert grown < 24 * 1024 * RSS_SCALE, grown  # KiB: a window or so, not the 100 MB download
                assert stalls and stalls[0] >= 1
            else:
                assert grown > 48 * 1024, grown  # no flow control: the proxy buffers for its client
                assert not stalls
            n = len(head) - head.index(b"\r\n\r\n") - 4
            s.settimeout(30)
            while n < 100_000_000:
                d = s.recv(1 << 20)
                assert d
                n += len(d)
            assert n == 100_000_000
            s.close()
    finally:
        mock.stop()


def test_one_gib_upload_keeps_serve_and_proxy_small():
    mock, mport = _native_mock()
    try:
        with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc") as t:
            total = 1 << 30
            chunk = np.random.default_rng(7).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
            s = socket.create_connection(("127.0.0.1", t.proxy_port))
            s.sendall(b"POST /sink HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % total)
            peak = {"serve": 0, "proxy": 0}
            stop = threading.Event()

            def watch():
                while not stop.is_set():
                    for k, p in (("serve", t.serve), ("proxy", t.proxy)):
                        peak[k] = max(peak[k], _rss_kb(p.popen.pid))
                    time.sleep(0.05)

            w = threading.Thread(target=watch)
            w.start()
            for _ in range(total // len(chunk)):
                s.sendall(chunk)
            s.settimeout(60)
            resp = b""
            while b"}" not in resp:
                d = s.recv(65536)
                assert d
                resp += d
            stop.set()
            w.join()
            res = json.loads(resp[resp.index(b"\r\n\r\n") + 4:])
            assert res["bytes"] == total
            per = np.arange(1, len(chunk) + 1, dtype=np.uint64) * np.frombuffer(chunk, dtype=np.uint8).astype(np.uint64)
            a, b = int(per.sum(dtype=np.uint64)), int(np.frombuffer(chunk, dtype=np.uint8).astype(np.uint64).sum())
            k = total // len(chunk)
            # sum over repeats r of (a + r*len*b), mod 2^64
            want = (k * a + len(chunk) * b * (k * (k - 1) // 2)) % (1 << 64)
            assert res["wsum"] == want
            for k_, v in peak.items():
                assert v < 64 * 1024 * RSS_SCALE, (k_, v, peak)  # KiB: RSS stays below 64 MiB for a 1 GiB body
            s.close()
    finally:
        mock.stop()


@pytest.mark.parametrize("chunked", [False, True])
def test_upload_answered_early_with_413_completes(chunked):
    """A client that sends its whole 1 MB body before reading gets the 413
    serve answered early: the proxy drains the rest of the upload once the
    response is done, although serve's credit for the stream never comes
    (the window is 256 KiB), and the connection stays usable."""
    mock, mport = _native_mock()
    try:
        with Tunnel(f"http://127.0.0.1:{mport}", transport="tcp",
                    serve_extra=["--max-request-body", "100000"]) as t:
            body = b"q" * (1 << 20)
            c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=20)
            if chunked:
                c.request("POST", "/sink", body=iter([body[o:o + 65536] for o in range(0, len(body), 65536)]),
                          encode_chunked=True)
            else:
                c.request("POST", "/sink", body=body)
            r = c.getresponse()
            assert r.status == 413
            r.read()
            c.request("GET", "/health")  # same connection: the upload was drained
            r = c.getresponse()
            assert r.status == 200 and r.read()
    finally:
        mock.stop()


def test_slow_client_on_an_extra_association_bounds_proxy_memory():
    """The same stalled 100 MB download, but on an extra association of the
    "assoc" extension: the route is learnt as bulk first, so the download's
    connection moves to another association before it starts; flow credit
    still bounds what the proxy holds for the client."""
    mock, mport = _native_mock()
    ms, mp = free_port(), free_port()
    try:
        with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc",
                    serve_extra=["--metrics-listen", f"127.0.0.1:{ms}", "--assoc", "3"],
                    proxy_extra=["--metrics-listen", f"127.0.0.1:{mp}", "--assoc", "3"],
                    env={"RUST_LOG": "info"}) as t:
            for k in (1, 2):
                t.proxy.wait_for(f"association {k} ready", 20)
            urllib.request.urlopen(t.url + "/bulk?bytes=1000000", timeout=30).read()  # the route is bulk now
            base = _rss_kb(t.proxy.popen.pid)
            s = socket.create_connection(("127.0.0.1", t.proxy_port))
            s.sendall(b"GET /bulk?bytes=100000000 HTTP/1.1\r\nHost: x\r\n\r\n")
            head = s.recv(65536)
            assert head.startswith(b"HTTP/1.1 200")
            time.sleep(2.0)  # the client reads nothing
            grown = _rss_kb(t.proxy.popen.pid) - base
            m = urllib.request.urlopen(f"http://127.0.0.1:{mp}/metrics", timeout=5).read().decode()
            handoffs = [float(l.split()[1]) for l in m.splitlines() if l.startswith("tunnel_assoc_handoffs_total")]
            assert handoffs and handoffs[0] >= 1, m[:200]
            assert grown < 24 * 1024 * RSS_SCALE, grown  # KiB
            n = len(head) - head.index(b"\r\n\r\n") - 4
            s.settimeout(30)
            while n < 100_000_000:
                d = s.recv(1 << 20)
                assert d
                n += len(d)
            assert n == 100_000_000
            s.close()
    finally:
        mock.stop()
