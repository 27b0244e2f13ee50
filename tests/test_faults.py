"""Fault injection and failure recovery (the reference tests none of this).

* Datagram loss / duplication / reordering on the WebRTC path (built-in
  injector: TUNNEL_FAULT drop / dup / delay_ms) — SCTP must deliver every
  frame intact and in order.
* Peer death: the surviving side detects it (SCTP ABORT on graceful exit,
  ICE consent timeout on kill -9), the supervisor backs off and reconnects,
  and requests work again.
"""
import http.client
import json
import threading
import time
import urllib.request

import pytest

from p2p_llm_tunnel_amd.utils.procs import Tunnel, start_serve


def sse(port):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=20)
    c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
    r = c.getresponse()
    return r.status, [l for l in r.read().split(b"\n") if l.startswith(b"data: ")]


@pytest.mark.parametrize("fault", [
    {"TUNNEL_FAULT": "drop=0.05"},
    {"TUNNEL_FAULT": "drop=0.02,dup=0.05,delay_ms=8"},
], ids=["loss5", "loss2-dup5-reorder"])
def test_lossy_path_integrity(mock_upstream, fault):
    with Tunnel(mock_upstream, transport="webrtc", env=fault) as t:
        body = bytes(range(256)) * 4096 * 2  # 2 MiB
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=60)
        c.request("POST", "/echo", body=body)
        r = c.getresponse()
        assert r.status == 200 and r.read() == body
        results = []
        ths = [threading.Thread(target=lambda: results.append(sse(t.proxy_port))) for _ in range(6)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        for st, ev in results:
            assert st == 200 and len(ev) == 7 and ev[-1] == b"data: [DONE]"


def test_graceful_peer_exit_triggers_fast_reconnect(mock_upstream):
    with Tunnel(mock_upstream, transport="webrtc") as t:
        assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"
        n_ready = t.proxy.count("proxy listening")
        t.serve.stop()  # SIGTERM: SCTP ABORT + DTLS close_notify reach the proxy at once
        t.proxy.wait_for(r"proxy failed \(attempt 1\)", 5)
        serve2 = start_serve(t.room, t.upstream, _signal_port(t))
        t.procs.append(serve2)
        serve2.wait_for("tunnel ready", 30)
        deadline = time.time() + 30
        while t.proxy.count("proxy listening") <= n_ready and time.time() < deadline:
            time.sleep(0.1)
        assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"


def test_hard_kill_detected_by_consent_timeout(mock_upstream):
    extra = ["--ice-timeout-ms", "2000"]
    with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra) as t:
        t.serve.kill()  # SIGKILL: nothing is sent; only liveness can notice
        line = t.proxy.wait_for(r"proxy failed \(attempt 1\)", 10)
        assert "failed" in line
        serve2 = start_serve(t.room, t.upstream, _signal_port(t), extra)
        t.procs.append(serve2)
        serve2.wait_for("tunnel ready", 30)
        t.proxy.wait_for("proxy listening", 30, start=len(t.proxy.lines) - 5)
        deadline = time.time() + 10
        while True:
            try:
                assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"
                break
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.2)


def _signal_port(t):
    # "[signal] listening on ws://127.0.0.1:PORT"
    line = next(l for l in t.signal.lines if "listening on" in l)
    return int(line.rsplit(":", 1)[1])


def test_signal_server_loss_and_restart(mock_upstream):
    """Signalling is only needed to set a session up (reference rtc.rs:463-514):
    an established tunnel keeps serving when the signal server dies; a peer
    that restarts meanwhile backs off until the signal server is back, then
    both sides rendezvous again."""
    with Tunnel(mock_upstream, transport="webrtc") as t:
        sp = _signal_port(t)
        t.signal.stop()
        for _ in range(3):
            st, ev = sse(t.proxy_port)
            assert st == 200 and ev[-1] == b"data: [DONE]"
        n_ready = t.proxy.count("proxy listening")
        t.serve.stop()
        t.proxy.wait_for(r"proxy failed \(attempt 1\)", 10)
        serve2 = start_serve(t.room, t.upstream, sp)
        t.procs.append(serve2)
        time.sleep(1.0)  # serve2 cannot reach the signal server yet
        from p2p_llm_tunnel_amd.utils.procs import start_signal
        sig2, _ = start_signal(sp)
        t.procs.append(sig2)
        serve2.wait_for("tunnel ready", 60)
        deadline = time.time() + 30
        while t.proxy.count("proxy listening") <= n_ready and time.time() < deadline:
            time.sleep(0.1)
        assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"
        st, ev = sse(t.proxy_port)
        assert st == 200 and len(ev) == 7


def test_blackholed_path_fails_and_recovers(mock_upstream):
    """The network path silently drops everything for a while (both peers
    alive): ICE consent freshness declares the session dead, the supervisor
    backs off and re-establishes once packets flow again."""
    extra = ["--ice-timeout-ms", "1500"]
    env = {"TUNNEL_FAULT": "blackhole=3000:4000"}
    with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra, env=env) as t:
        assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"
        t.proxy.wait_for(r"proxy failed \(attempt 1\)", 15)
        t.proxy.wait_for("proxy listening", 40, start=len(t.proxy.lines) - 1)
        deadline = time.time() + 10
        while True:
            try:
                assert urllib.request.urlopen(t.url + "/health", timeout=5).read() == b"ok"
                break
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.2)
