"""TURN relay path (--turn/--turn-user/--turn-pass; reference cli.rs:30-40,
rtc.rs:54-63). Both peers are forced onto relayed candidates
(--ice-relay-only) so every datagram crosses the test TURN server."""
import http.client
import json
import urllib.request

from p2p_llm_tunnel_amd.utils.procs import Tunnel
from p2p_llm_tunnel_amd.utils.turn_server import TurnServer


def test_tunnel_through_turn_relay(mock_upstream):
    turn = TurnServer(user="alice", password="s3cret").start()
    try:
        extra = ["--turn", turn.url, "--turn-user", "alice", "--turn-pass", "s3cret", "--ice-relay-only"]
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra,
                    env={"RUST_LOG": "info,tunnel::rtc=debug,tunnel::turn=info"}) as t:
            assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"
            c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=30)
            body = b"z" * 300000
            c.request("POST", "/echo", body=body)
            r = c.getresponse()
            assert r.status == 200 and r.read() == body
            c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
            r = c.getresponse()
            assert r.read().count(b"data: ") == 7
            assert "relay:" in t.serve.text() and "TURN server configured" in t.serve.text()
            assert t.serve.count("TURN allocation: relayed") == 1
        assert turn.stats["allocations"] >= 2
        assert turn.stats["relayed_to_peer"] > 50 and turn.stats["relayed_to_client"] > 50
        assert turn.stats["channel_binds"] >= 2
    finally:
        turn.stop()


def test_turn_bad_credentials_fail_gathering_gracefully(mock_upstream):
    turn = TurnServer(user="alice", password="right").start()
    try:
        extra = ["--turn", turn.url, "--turn-user", "alice", "--turn-pass", "wrong"]
        # Without relay-only the host path still works; the failed allocation must not block.
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra) as t:
            assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"
        assert turn.stats["allocations"] == 0
    finally:
        turn.stop()
