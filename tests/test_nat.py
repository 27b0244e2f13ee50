"""NAT traversal without two NATs (BASELINE.json config #4: "two hosts behind
separate NATs, public signal server, STUN-only ICE"; SURVEY §4.2 "NAT-style
port rewrite").

Both tunnel peers run with the ICE agent's NAT emulation (TUNNEL_NAT, see
native/rtc/ice.h): every datagram leaves through an emulated external socket,
the private host sockets drop all inbound traffic, and an external socket only
admits datagrams from destinations it has sent to. The test STUN/TURN server
therefore reports the *external* address as the server-reflexive candidate.

* port-restricted cone NATs on both sides: STUN-only ICE connects through the
  srflx candidates by hole punching (each side's checks open its own filter);
* symmetric NATs on both sides: srflx mappings do not carry over to the peer,
  STUN-only ICE fails; with TURN configured the tunnel connects via the relay.

The reference relies on webrtc-rs for this and tests none of it.
"""
import http.client
import json
import re
import time
import urllib.request

from p2p_llm_tunnel_amd.utils.procs import Tunnel, start_proxy, start_serve, start_signal
from p2p_llm_tunnel_amd.utils.turn_server import TurnServer

LOG = {"RUST_LOG": "info,tunnel::ice=debug,tunnel::rtc=debug"}


def _exercise(port):
    assert urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=10).read() == b"ok"
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
    r = c.getresponse()
    assert r.status == 200 and r.read().count(b"data: ") == 7
    body = bytes(range(256)) * 2048
    c.request("POST", "/echo", body=body)
    r = c.getresponse()
    assert r.status == 200 and r.read() == body


def _filtered(text):
    m = re.findall(r"NAT emulation: (\d+) inbound datagrams filtered", text)
    return int(m[-1]) if m else -1


def test_port_restricted_nats_connect_with_stun_only(mock_upstream):
    stun = TurnServer().start()
    try:
        extra = ["--stun", f"stun:127.0.0.1:{stun.port}"]
        env = dict(LOG, TUNNEL_NAT="port-restricted")
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra, env=env) as t:
            _exercise(t.proxy_port)
            sel = [l for l in t.serve.lines if "ICE selected pair" in l]
            assert sel, t.serve.text()[-2000:]
        # srflx candidates came from the STUN server; the peers reached each
        # other through them, and each NAT dropped traffic it had not asked for.
        assert stun.stats["bindings"] >= 2
        for p in (t.serve, t.proxy):
            txt = p.text()
            assert "NAT emulation: port-restricted" in txt
            assert re.search(r"local candidate: candidate:\S+ 1 udp \d+ \S+ \d+ typ srflx", txt), txt[-3000:]
            assert _filtered(txt) > 0
    finally:
        stun.stop()


def test_symmetric_nats_fail_with_stun_only(mock_upstream):
    stun = TurnServer().start()
    signal, sp = start_signal()
    procs = [signal]
    try:
        room = f"nat-sym-{time.time_ns()}"
        extra = ["--stun", f"stun:127.0.0.1:{stun.port}", "--ice-timeout-ms", "3000", "--max-retries", "1"]
        env = dict(LOG, TUNNEL_NAT="symmetric")
        serve = start_serve(room, mock_upstream, sp, extra, env)
        proxy = start_proxy(room, "127.0.0.1:0", sp, extra, env)
        procs += [serve, proxy]
        # Whichever side's ICE timer fires first reports the failure; the other
        # then sees the peer leave (or fails on its own timer). Both give up
        # after --max-retries without ever carrying traffic.
        pat = r"ICE connection failed|peer connection failed"
        deadline = time.time() + 30
        while time.time() < deadline and not (serve.count(pat) or proxy.count(pat)):
            time.sleep(0.1)
        assert serve.count(pat) or proxy.count(pat), serve.text()[-2000:] + "\n----\n" + proxy.text()[-2000:]
        for p in (serve, proxy):
            p.wait_for(r"giving up", 30)
            assert p.popen.wait(10) == 1
        assert proxy.count("proxy listening") == 0
        assert serve.count("tunnel ready") == 0
    finally:
        for p in reversed(procs):
            p.stop()
        stun.stop()


def test_symmetric_nats_connect_through_turn(mock_upstream):
    turn = TurnServer(user="u", password="p").start()
    try:
        extra = ["--turn", turn.url, "--turn-user", "u", "--turn-pass", "p", "--stun", f"stun:127.0.0.1:{turn.port}"]
        env = dict(LOG, TUNNEL_NAT="symmetric")
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra, env=env) as t:
            _exercise(t.proxy_port)
            sel = [l for l in t.serve.lines + t.proxy.lines if "ICE selected pair" in l]
            assert any("relay" in l for l in sel), sel
        assert turn.stats["allocations"] >= 2 and turn.stats["relayed_to_peer"] > 10
    finally:
        turn.stop()
