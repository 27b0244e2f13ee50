"""Wire-level conformance of the native roles against a scripted Python peer.

Serve side (reference serve.rs): HELLO->AGREE, PING->PONG, REQ_* lifecycle
keyed by the JSON stream_id, body-for-unknown-stream dropped, 502 synthesis,
ERROR+END mid-stream, and the local fixes for Q3/Q4 (400 instead of killing
the session / hanging the client). Proxy side (reference proxy.rs): HELLO
first, REQ framing (<= 65408-byte bodies), routing by JSON stream_id,
RES_BODY-before-headers dropped, ERROR-before-headers -> 502
"Tunnel error: ...", and CANCEL on client disconnect when negotiated.
"""
import http.client
import json
import socket
import threading
import time

import pytest

from p2p_llm_tunnel_amd.utils import framepeer as fp
from p2p_llm_tunnel_amd.utils.procs import free_port, spawn
from p2p_llm_tunnel_amd import binary


# ------------------------------------------------------------------ serve side

@pytest.fixture
def serve_peer(mock_upstream):
    port = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", mock_upstream,
                           "--transport", f"tcp-listen:127.0.0.1:{port}", "--max-retries", "0"],
                 env={"RUST_LOG": "info,tunnel::serve=debug"})
    proc.wait_for("tcp transport: listening", 10)
    peer = fp.FramePeer.connect(port)
    yield peer, proc
    peer.close()
    proc.stop()


def handshake(peer, features=("sse",)):
    peer.send_json(fp.HELLO, 0, {"proto": "httptunnel", "min_version": 1, "max_version": 1, "features": list(features)})
    t, sid, p = peer.recv()
    assert t == fp.AGREE and sid == 0
    return json.loads(p)


def test_serve_handshake_and_ping(serve_peer):
    peer, proc = serve_peer
    assert handshake(peer) == {"version": 1, "features": ["sse"]}
    # First PING arrives immediately after AGREE (tokio interval first tick).
    t, sid, p = peer.recv()
    assert (t, sid, p) == (fp.PING, 0, b"")
    peer.send(fp.PING, 0)
    assert peer.recv()[:2] == (fp.PONG, 0)
    proc.wait_for("sent AGREE, tunnel ready", 2)


def test_serve_request_lifecycle_keyed_by_json_stream_id(serve_peer):
    peer, _ = serve_peer
    handshake(peer)
    # Frame stream_id 5, JSON stream_id 7: the reference keys by the JSON id.
    peer.send_json(fp.REQ_HEADERS, 5, {"stream_id": 7, "method": "POST", "path": "/echo", "headers": {"x-a": "b"}})
    peer.send(fp.REQ_BODY, 7, b"hello ")
    peer.send(fp.REQ_BODY, 99, b"dropped: unknown stream")
    peer.send(fp.REQ_BODY, 7, b"world")
    peer.send(fp.REQ_END, 7)
    t, sid, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
    h = json.loads(p)
    assert sid == 7 and h["stream_id"] == 7 and h["status"] == 200
    assert all(k == k.lower() for k in h["headers"])
    body = b""
    while True:
        t, sid, p = peer.recv_until(lambda *a: True)
        if t == fp.RES_END:
            break
        assert t == fp.RES_BODY and sid == 7
        body += p
    assert body == b"hello world"


def test_serve_502_on_dead_upstream():
    port = free_port()
    dead = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", f"http://127.0.0.1:{dead}",
                           "--transport", f"tcp-listen:127.0.0.1:{port}"])
    try:
        proc.wait_for("tcp transport: listening", 10)
        peer = fp.FramePeer.connect(port)
        handshake(peer)
        peer.send_json(fp.REQ_HEADERS, 1, {"stream_id": 1, "method": "GET", "path": "/x", "headers": {}})
        peer.send(fp.REQ_END, 1)
        t, _, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
        assert json.loads(p)["status"] == 502 and json.loads(p)["headers"] == {"content-type": "text/plain"}
        t, _, p = peer.recv_until(lambda *a: True)
        assert t == fp.RES_BODY and p.startswith(b"Bad Gateway: ")
        assert peer.recv_until(lambda *a: True)[0] == fp.RES_END
    finally:
        proc.stop()


def test_serve_malformed_headers_and_bad_method_get_400(serve_peer):
    peer, _ = serve_peer
    handshake(peer)
    peer.send(fp.REQ_HEADERS, 3, b"{not json")
    t, sid, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
    assert sid == 3 and json.loads(p)["status"] == 400
    peer.recv_until(lambda t, s, p: t == fp.RES_END)
    peer.send_json(fp.REQ_HEADERS, 4, {"stream_id": 4, "method": "GE T", "path": "/", "headers": {}})
    peer.send(fp.REQ_END, 4)
    t, sid, p = peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
    assert sid == 4 and json.loads(p)["status"] == 400
    peer.recv_until(lambda t, s, p: t == fp.RES_END)
    # session still alive
    peer.send(fp.PING, 0)
    peer.recv_until(lambda t, s, p: t == fp.PONG, skip_pings=False)


def test_serve_midstream_error_then_end(serve_peer):
    peer, _ = serve_peer
    handshake(peer)
    peer.send_json(fp.REQ_HEADERS, 9, {"stream_id": 9, "method": "GET", "path": "/drop", "headers": {}})
    peer.send(fp.REQ_END, 9)
    peer.recv_until(lambda t, s, p: t == fp.RES_HEADERS)
    t, _, p = peer.recv_until(lambda t, s, p: t != fp.RES_BODY)
    assert t == fp.ERROR and p.startswith(b"upstream error: ")
    assert peer.recv_until(lambda *a: True)[0] == fp.RES_END


def test_serve_rejects_wrong_first_frame():
    port = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", "http://127.0.0.1:1",
                           "--transport", f"tcp-listen:127.0.0.1:{port}", "--max-retries", "0"])
    try:
        proc.wait_for("tcp transport: listening", 10)
        peer = fp.FramePeer.connect(port)
        peer.send(fp.PING, 0)
        proc.wait_for("expected HELLO, got Ping", 5)
    finally:
        proc.stop()


def test_serve_rejects_incompatible_version():
    port = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", "http://127.0.0.1:1",
                           "--transport", f"tcp-listen:127.0.0.1:{port}", "--max-retries", "0"])
    try:
        proc.wait_for("tcp transport: listening", 10)
        peer = fp.FramePeer.connect(port)
        peer.send_json(fp.HELLO, 0, {"proto": "httptunnel", "min_version": 5, "max_version": 9, "features": []})
        proc.wait_for(r"handshake failed: no compatible version: peer=\[5,9\], ours=\[1,1\]", 5)
    finally:
        proc.stop()


def test_serve_cancel_aborts_upstream(serve_peer):
    peer, proc = serve_peer
    agree = handshake(peer, ("sse", "cancel"))
    assert agree["features"] == ["sse", "cancel"]
    peer.send_json(fp.REQ_HEADERS, 2, {"stream_id": 2, "method": "POST", "path": "/v1/chat/completions",
                                       "headers": {"content-type": "application/json"}})
    peer.send(fp.REQ_BODY, 2, b'{"stream": true}')
    peer.send(fp.REQ_END, 2)
    peer.recv_until(lambda t, s, p: t == fp.RES_BODY)
    peer.send(fp.CANCEL, 2)
    proc.wait_for("stream 2 cancelled by peer", 5)
    with pytest.raises((socket.timeout, TimeoutError)):
        peer.recv_until(lambda t, s, p: t == fp.RES_END, timeout=1.0)


# ------------------------------------------------------------------ proxy side

@pytest.fixture
def proxy_peer():
    srv = fp.FramePeer.listen()
    port = srv.getsockname()[1]
    http_port = free_port()
    proc = spawn("proxy", [binary("tunnel"), "proxy", "--room", "x", "--listen", f"127.0.0.1:{http_port}",
                           "--transport", f"tcp-connect:127.0.0.1:{port}", "--header-timeout-ms", "3000"],
                 env={"RUST_LOG": "info,tunnel::proxy=debug"})
    conn, _ = srv.accept()
    peer = fp.FramePeer(conn)
    t, sid, p = peer.recv()
    hello = json.loads(p)
    assert t == fp.HELLO and sid == 0 and hello["proto"] == "httptunnel" and "sse" in hello["features"]
    peer.send_json(fp.AGREE, 0, {"version": 1, "features": ["sse", "cancel"]})
    proc.wait_for("proxy listening", 5)
    yield peer, proc, http_port
    peer.close()
    proc.stop()
    srv.close()


def client(port, method, path, body=None, headers=None):
    out = {}

    def run():
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=15)
        c.request(method, path, body=body, headers=headers or {})
        r = c.getresponse()
        out["status"], out["headers"], out["body"] = r.status, dict(r.getheaders()), r.read()
    th = threading.Thread(target=run)
    th.start()
    return th, out


def test_proxy_request_framing(proxy_peer):
    peer, _, port = proxy_peer
    body = b"a" * 150000
    th, out = client(port, "POST", "/v1/x?q=1", body, {"X-Test": "1"})
    t, sid, p = peer.recv_until(lambda t, s, p: t == fp.REQ_HEADERS)
    h = json.loads(p)
    assert sid == 1 and h["stream_id"] == 1 and h["method"] == "POST" and h["path"] == "/v1/x?q=1"
    assert h["headers"]["x-test"] == "1" and h["headers"]["host"].startswith("127.0.0.1:")
    got = b""
    sizes = []
    while True:
        t, s, p = peer.recv_until(lambda *a: True)
        if t == fp.REQ_END:
            break
        assert t == fp.REQ_BODY and s == 1
        sizes.append(len(p))
        got += p
    assert got == body and max(sizes) <= 65408
    peer.send_json(fp.RES_HEADERS, 1, {"stream_id": 1, "status": 201, "headers": {"x-r": "y", "connection": "zzz"}})
    peer.send(fp.RES_BODY, 1, b"par")
    peer.send(fp.RES_BODY, 1, b"tial")
    peer.send(fp.RES_END, 1)
    th.join(10)
    assert out["status"] == 201 and out["body"] == b"partial" and out["headers"]["x-r"] == "y"
    assert out["headers"].get("connection") != "zzz"


def test_proxy_body_before_headers_dropped_and_routing_by_json_id(proxy_peer):
    peer, _, port = proxy_peer
    th, out = client(port, "GET", "/a")
    _, sid, _ = peer.recv_until(lambda t, s, p: t == fp.REQ_END)
    peer.send(fp.RES_BODY, sid, b"early")  # dropped with a warning
    peer.send_json(fp.RES_HEADERS, 777, {"stream_id": sid, "status": 200, "headers": {"content-length": "2"}})
    peer.send(fp.RES_BODY, sid, b"ok")
    peer.send(fp.RES_END, sid)
    th.join(10)
    assert out["status"] == 200 and out["body"] == b"ok"


def test_proxy_error_before_headers_is_502(proxy_peer):
    peer, _, port = proxy_peer
    th, out = client(port, "GET", "/b")
    _, sid, _ = peer.recv_until(lambda t, s, p: t == fp.REQ_END)
    peer.send(fp.ERROR, sid, b"boom")
    peer.send(fp.RES_END, sid)  # ignored: stream already removed
    th.join(10)
    assert out["status"] == 502 and out["body"] == b"Tunnel error: boom"


def test_proxy_end_before_headers_is_502(proxy_peer):
    peer, _, port = proxy_peer
    th, out = client(port, "GET", "/c")
    _, sid, _ = peer.recv_until(lambda t, s, p: t == fp.REQ_END)
    peer.send(fp.RES_END, sid)
    th.join(10)
    assert out["status"] == 502 and out["body"] == b"Tunnel error: response ended before headers"


def test_proxy_header_timeout_504(proxy_peer):
    peer, _, port = proxy_peer
    th, out = client(port, "GET", "/slow")
    peer.recv_until(lambda t, s, p: t == fp.REQ_END)
    th.join(10)
    assert out["status"] == 504 and out["body"] == b"Tunnel response timeout"


def test_proxy_answers_ping_and_sends_cancel_on_disconnect(proxy_peer):
    peer, proc, port = proxy_peer
    peer.send(fp.PING, 0)
    peer.recv_until(lambda t, s, p: t == fp.PONG, skip_pings=False)
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"GET /stream HTTP/1.1\r\nHost: x\r\n\r\n")
    _, sid, _ = peer.recv_until(lambda t, s_, p: t == fp.REQ_END)
    peer.send_json(fp.RES_HEADERS, sid, {"stream_id": sid, "status": 200, "headers": {"content-type": "text/event-stream"}})
    peer.send(fp.RES_BODY, sid, b"data: 1\n\n")
    time.sleep(0.2)
    s.close()
    t, csid, _ = peer.recv_until(lambda t, s_, p: t == fp.CANCEL)
    assert csid == sid


def test_proxy_stream_ids_monotone(proxy_peer):
    peer, _, port = proxy_peer
    ids = []
    for i in range(3):
        th, out = client(port, "GET", f"/{i}")
        _, sid, p = peer.recv_until(lambda t, s, p: t == fp.REQ_HEADERS)
        ids.append(json.loads(p)["stream_id"])
        peer.recv_until(lambda t, s, p: t == fp.REQ_END)
        peer.send_json(fp.RES_HEADERS, sid, {"stream_id": sid, "status": 204, "headers": {}})
        peer.send(fp.RES_END, sid)
        th.join(10)
        assert out["status"] == 204
    assert ids == [1, 2, 3]
