"""The standard 1200-byte SCTP path (what every cross-host WebRTC peer uses,
reference rtc.rs:31-72 via webrtc-rs defaults), forced on loopback with
--no-jumbo-loopback: bulk bodies and SSE stay correct with UDP GSO/GRO on
(runs of equal-size DTLS datagrams leave as one message and arrive
coalesced) and with both switched off (TUNNEL_UDP_OFFLOAD=none)."""
import http.client
import os
import json
import time
import urllib.request

import pytest

from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port

STD = ["--no-jumbo-loopback"]
# One association: the transport gauges checked below are the first
# association's, and with "assoc" the bulk echo would run on an extra one.
ONE = ["--assoc", "1"]


def _metrics(port):
    txt = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    return {l.split()[0]: float(l.split()[1]) for l in txt.splitlines() if l and not l.startswith("#")}


@pytest.mark.parametrize("offload", [True, False])
def test_standard_mtu_bulk_and_sse(mock_upstream, offload):
    ms, mp = free_port(), free_port()
    env = None if offload else {"TUNNEL_UDP_OFFLOAD": "none"}
    with Tunnel(mock_upstream, transport="webrtc", env=env,
                serve_extra=STD + ONE + ["--metrics-listen", f"127.0.0.1:{ms}"],
                proxy_extra=STD + ONE + ["--metrics-listen", f"127.0.0.1:{mp}"]) as t:
        assert "mtu=1200" in t.serve.wait_for("connection established", 5)
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=60)
        body = bytes((i * 7 + 3) & 0xFF for i in range(3 * 1024 * 1024 + 17))
        for _ in range(2):
            c.request("POST", "/echo", body=body)
            r = c.getresponse()
            assert r.status == 200 and r.read() == body
        c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
        r = c.getresponse()
        assert r.status == 200 and r.read().count(b"data: ") == 7
        sm, pm = _metrics(ms), _metrics(mp)
        if offload:
            # the echoed bodies left as GSO runs and arrived GRO-coalesced
            assert sm["tunnel_udp_gso_sends"] > 0 and pm["tunnel_udp_gso_sends"] > 0
            assert sm["tunnel_udp_gro_batches"] > 0 and pm["tunnel_udp_gro_batches"] > 0
        else:
            assert sm["tunnel_udp_gso_sends"] == 0 and sm["tunnel_udp_gro_batches"] == 0
        assert sm["tunnel_sctp_packets_sent"] > 2 * len(body) / 1200


def test_emulated_wan_path_with_loss(mock_upstream):
    """20 ms RTT, 100 Mbit/s bottleneck, 1% loss on both peers' datagrams
    (the ICE agent's WAN shim): bodies and SSE still arrive intact, losses are
    repaired without T3 collapse, and a slow path keeps the scheduler's
    channel window small without stalling it (adaptive window + low-water)."""
    ms = free_port()
    env = {"TUNNEL_FAULT": "rtt_ms=20,rate_mbps=100,loss=0.01"}
    with Tunnel(mock_upstream, transport="webrtc", env=env, serve_extra=STD + ["--metrics-listen", f"127.0.0.1:{ms}"],
                proxy_extra=STD) as t:
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=60)
        body = bytes((i * 13 + 1) & 0xFF for i in range(1024 * 1024 + 3))
        c.request("POST", "/echo", body=body)
        r = c.getresponse()
        assert r.status == 200 and r.read() == body
        for _ in range(3):
            c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
            r = c.getresponse()
            assert r.status == 200 and r.read().count(b"data: ") == 7
        m = _metrics(ms)
        assert m["tunnel_sctp_retransmits"] > 0  # losses happened and were repaired
        assert 15000 <= m["tunnel_sctp_srtt_us"] <= 200000


def test_flow_window_grows_on_a_long_rtt_path(mock_upstream):
    """50 ms RTT, 400 Mbit/s bottleneck with a one-BDP queue, no loss: 12 MiB
    downloads on one keep-alive connection. A fixed 256 KiB "flow" window
    caps a stream at 256 KiB per round trip (measured 4.8 MB/s before the
    autotuning); the proxy's receive-window autotuning doubles it while
    windows are taken within two round trips (measured 16 MB/s)."""
    mp = free_port()
    env = {"TUNNEL_FAULT": "rtt_ms=50,rate_mbps=400,loss=0,queue_kb=2441"}
    n = 12 << 20
    with Tunnel(mock_upstream, transport="webrtc", env=env, serve_extra=STD,
                proxy_extra=STD + ["--metrics-listen", f"127.0.0.1:{mp}"]) as t:
        c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=60)
        c.request("GET", "/bulk?bytes=65536")  # warm the association
        assert len(c.getresponse().read()) == 65536
        rates = []
        for _ in range(2):  # the first also ramps SCTP's congestion window
            t0 = time.time()
            c.request("GET", f"/bulk?bytes={n}")
            r = c.getresponse()
            got = len(r.read())
            rates.append(n / (time.time() - t0) / 1e6)
            assert r.status == 200 and got == n
        m = _metrics(mp)
        assert m.get("tunnel_flow_window_growths_total", 0) >= 3  # 256 KiB -> >= 2 MiB
        if not os.environ.get("P2PT_BIN_DIR"):  # sanitizer builds run several times slower
            assert max(rates) > 8.0, rates
