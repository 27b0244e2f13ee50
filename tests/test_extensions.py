"""Opt-in extensions and HTTP edge cases (defaults keep reference behaviour)."""
import http.client
import socket
import time
import urllib.request

import pytest

from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn, start_signal
from p2p_llm_tunnel_amd import binary


def test_listen_early_answers_503_until_ready(mock_upstream):
    sig, sport = start_signal()
    port = free_port()
    proxy = spawn("proxy", [binary("tunnel"), "proxy", "--room", "early", "--listen", f"127.0.0.1:{port}",
                            "--signal", f"ws://127.0.0.1:{sport}", "--stun", "none", "--listen-early"])
    serve = None
    try:
        proxy.wait_for("proxy listening on", 10)
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5)
        assert e.value.code == 503 and e.value.read() == b"Tunnel not ready"
        serve = spawn("serve", [binary("tunnel"), "serve", "--room", "early", "--upstream", mock_upstream,
                                "--signal", f"ws://127.0.0.1:{sport}", "--stun", "none"])
        serve.wait_for("tunnel ready", 20)
        deadline = time.time() + 10
        while True:
            try:
                assert urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5).read() == b"ok"
                break
            except urllib.error.HTTPError:
                if time.time() > deadline:
                    raise
                time.sleep(0.1)
    finally:
        for p in (serve, proxy, sig):
            if p:
                p.stop()


def test_metrics_endpoint(mock_upstream):
    mport = free_port()
    with Tunnel(mock_upstream, proxy_extra=["--metrics-listen", f"127.0.0.1:{mport}"]) as t:
        for _ in range(3):
            urllib.request.urlopen(t.url + "/health", timeout=5).read()
        text = urllib.request.urlopen(f"http://127.0.0.1:{mport}/metrics", timeout=5).read().decode()
    assert 'tunnel_frames_sent_total{type="ReqHeaders"} 3' in text
    assert 'tunnel_frames_received_total{type="ResEnd"} 3' in text
    assert "tunnel_streams_opened_total 3" in text
    assert "tunnel_sctp_cwnd_bytes" in text


def test_oversized_request_headers_431(mock_upstream):
    with Tunnel(mock_upstream, transport="tcp") as t:
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=10)
        hdrs = {f"x-big-{i}": "v" * 1000 for i in range(60)}  # ~61 KB of header JSON > 64 KiB frame
        hdrs.update({f"x-more-{i}": "w" * 1000 for i in range(10)})
        c.request("GET", "/health", headers=hdrs)
        r = c.getresponse()
        assert r.status == 431


def test_head_request_has_no_body(mock_upstream):
    with Tunnel(mock_upstream, transport="tcp") as t:
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=10)
        c.request("HEAD", "/v1/models")
        r = c.getresponse()
        assert r.read() == b""
        c.request("GET", "/health")  # connection still usable
        assert c.getresponse().read() == b"ok"


def test_chunked_request_body_and_expect_continue(mock_upstream):
    with Tunnel(mock_upstream, transport="webrtc") as t:
        s = socket.create_connection(("127.0.0.1", t.proxy_port), timeout=10)
        s.sendall(b"POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\nExpect: 100-continue\r\n\r\n")
        assert s.recv(1024).startswith(b"HTTP/1.1 100 Continue")
        s.sendall(b"5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n")
        data = b""
        while b"hello world" not in data:
            d = s.recv(65536)
            if not d:
                break
            data += d
        s.close()
        assert data.startswith(b"HTTP/1.1 200") and data.endswith(b"hello world")


def test_pipelined_requests(mock_upstream):
    with Tunnel(mock_upstream, transport="tcp") as t:
        s = socket.create_connection(("127.0.0.1", t.proxy_port), timeout=10)
        s.sendall(b"GET /health HTTP/1.1\r\nHost: x\r\n\r\nGET /health HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
        data = b""
        while True:
            d = s.recv(65536)
            if not d:
                break
            data += d
        assert data.count(b"HTTP/1.1 200") == 2 and data.endswith(b"2\r\nok\r\n0\r\n\r\n")


def test_cli_help_version_and_missing_args():
    import subprocess
    out = subprocess.run([binary("tunnel"), "--version"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("tunnel ")
    out = subprocess.run([binary("tunnel"), "serve", "--help"], capture_output=True, text=True)
    assert "--upstream" in out.stdout and "TUNNEL_UPSTREAM" in out.stdout and "--advertise" in out.stdout
    out = subprocess.run([binary("tunnel"), "proxy", "--help"], capture_output=True, text=True)
    assert "127.0.0.1:8000" in out.stdout and "TUNNEL_LISTEN" in out.stdout
    out = subprocess.run([binary("tunnel"), "serve", "--room", "r"], capture_output=True, text=True,
                         env={"PATH": "/usr/bin"})
    assert out.returncode == 2 and "--upstream" in out.stderr
    out = subprocess.run([binary("tunnel"), "proxy"], capture_output=True, text=True,
                         env={"PATH": "/usr/bin", "TUNNEL_ROOM": "r", "TUNNEL_SIGNAL": "ws://127.0.0.1:1",
                              "TUNNEL_MAX_RETRIES": "0"})
    assert "connecting to signaling server: ws://127.0.0.1:1" in out.stdout  # env fallbacks honoured


@pytest.mark.parametrize("args,env,flag,why", [
    (["serve", "--room", "r", "--upstream", "http://x", "--workers", "x"], {}, "--workers", "invalid digit"),
    (["proxy", "--room", "r", "--ping-interval-ms", "x"], {}, "--ping-interval-ms", "invalid digit"),
    (["proxy", "--room", "r", "--ping-interval-ms="], {}, "--ping-interval-ms", "empty string"),
    (["proxy", "--room", "r", "--pong-timeout-ms", "-5"], {}, "--pong-timeout-ms", "invalid digit"),
    (["proxy", "--room", "r", "--header-timeout-ms", "99999999999999999999999"], {}, "--header-timeout-ms",
     "too large"),
    (["serve", "--room", "r", "--upstream", "http://x", "--sctp-mtu", "100"], {}, "--sctp-mtu", "not in 576..65535"),
    (["serve", "--room", "r", "--upstream", "http://x", "--max-request-body", "1k"], {}, "--max-request-body",
     "invalid digit"),
    (["proxy", "--room", "r"], {"TUNNEL_WORKERS": "four"}, "--workers", "invalid digit"),  # env values are checked too
    (["proxy", "--room", "r"], {"TUNNEL_GATHER_TIMEOUT_MS": "5s"}, "--gather-timeout-ms", "invalid digit"),
])
def test_cli_rejects_bad_numbers(args, env, flag, why):
    """Every numeric flag is parsed whole (clap's u64 parser, cli.rs:13-68): exit 2 naming the flag."""
    import os
    import subprocess
    out = subprocess.run([binary("tunnel")] + args, capture_output=True, text=True, timeout=10,
                         env={"PATH": os.environ.get("PATH", "/usr/bin"), **env})
    assert out.returncode == 2, out
    assert f"for '{flag} <VALUE>'" in out.stderr and why in out.stderr, out.stderr


@pytest.mark.parametrize("cmd,flag", [
    ("proxy", ["--max-request-body", "5"]),
    ("proxy", ["--stream-body-threshold", "5"]),
    ("proxy", ["--upstream-prewarm", "0"]),
    ("proxy", ["--upstream-prewarm-ttl-ms=10"]),
    ("proxy", ["--upstream", "http://x"]),
    ("proxy", ["--advertise", "/v1"]),
    ("serve", ["--listen-early"]),
    ("serve", ["--listen", "127.0.0.1:1"]),
])
def test_cli_rejects_flags_of_the_other_subcommand(cmd, flag):
    """clap rejects an argument its subcommand does not define (cli.rs:13-68); so do the extensions."""
    import subprocess
    base = ["--room", "r"] + (["--upstream", "http://x"] if cmd == "serve" else [])
    out = subprocess.run([binary("tunnel"), cmd] + base + flag, capture_output=True, text=True, timeout=10)
    name = flag[0].split("=")[0]
    assert out.returncode == 2 and f"unexpected argument '{name}'" in out.stderr, out
    help_text = subprocess.run([binary("tunnel"), cmd, "--help"], capture_output=True, text=True).stdout
    assert name + " " not in help_text and name + "\n" not in help_text


def test_cli_flag_switch_takes_no_value():
    import subprocess
    out = subprocess.run([binary("tunnel"), "proxy", "--room", "r", "--ipv6=1"], capture_output=True, text=True)
    assert out.returncode == 2 and "'--ipv6'" in out.stderr


def _raw_exchange(port, request: bytes) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.sendall(request)
    data = b""
    while True:
        d = s.recv(65536)
        if not d:
            break
        data += d
    s.close()
    return data


@pytest.mark.parametrize("framing", [
    b"Transfer-Encoding: chunked\r\nContent-Length: 5\r\n",          # TE + CL (RFC 9112 §6.3 smuggling vector)
    b"Content-Length: 5\r\nTransfer-Encoding: chunked\r\n",
    b"Transfer-Encoding: chunked, gzip\r\n",                        # chunked not the final coding
    b"Transfer-Encoding: chunked\r\nTransfer-Encoding: gzip\r\n",  # same, over two field lines
    b"Transfer-Encoding: gzip\r\n",
    b"Transfer-Encoding: gzip, chunked\r\n",                        # a coding serve could not relay
])
def test_request_framing_rejected_with_400_and_close(mock_upstream, framing):
    """Ambiguous or unsupported request framing: 400 and the connection closes
    (RFC 9112 §6.1), so nothing after the head is read as a next request."""
    with Tunnel(mock_upstream, transport="tcp") as t:
        smuggled = b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n"
        data = _raw_exchange(t.proxy_port, b"POST /echo HTTP/1.1\r\nHost: x\r\n" + framing + b"\r\n"
                             b"5\r\nhello\r\n0\r\n\r\n" + smuggled)
        assert data.startswith(b"HTTP/1.1 400"), data[:200]
        assert data.count(b"HTTP/1.1 ") == 1  # closed: the trailing request was never served
        # The proxy itself is fine afterwards.
        assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"


def test_request_chunked_alone_still_accepted(mock_upstream):
    with Tunnel(mock_upstream, transport="tcp") as t:
        data = _raw_exchange(t.proxy_port, b"POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: Chunked\r\n"
                             b"Connection: close\r\n\r\n5\r\nhello\r\n0\r\n\r\n")
        assert data.startswith(b"HTTP/1.1 200") and b"hello" in data


def test_cpu_affinity(mock_upstream):
    """--cpu-affinity pins the reactor thread (NUMA placement next to the NIC)."""
    import os
    import subprocess
    cpu = sorted(os.sched_getaffinity(0))[-1]
    with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--cpu-affinity", str(cpu)]) as t:
        assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"
        status = open(f"/proc/{t.serve.popen.pid}/status").read()
        allowed = [l.split(":", 1)[1].strip() for l in status.splitlines() if l.startswith("Cpus_allowed_list")]
        assert allowed == [str(cpu)]
        assert f"pinned to CPUs {cpu}" in t.serve.text()
    out = subprocess.run([binary("tunnel"), "serve", "--room", "r", "--upstream", "http://x", "--cpu-affinity", "3-1"],
                         capture_output=True, text=True)
    assert out.returncode == 2 and "bad CPU range" in out.stderr


def test_backoff_schedule(native):
    assert [native.backoff_secs(n) for n in range(1, 9)] == [2, 4, 8, 16, 32, 60, 60, 60]
