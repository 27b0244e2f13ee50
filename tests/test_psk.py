"""Pre-shared-secret authentication (extension "psk", `--secret` /
TUNNEL_SECRET): the reference README lists `--secret` as planned (README.md
"Future options"); the room name is otherwise the only credential.

Both sides prove the secret with an HMAC over a fresh nonce and the channel
binding (both DTLS certificate fingerprints, sorted; empty on the TCP debug
transport), so a proof cannot be replayed on another channel. Without a
secret nothing changes on the wire (reference HELLO/AGREE).
"""
import hashlib
import hmac
import http.client
import json
import os
import time

from p2p_llm_tunnel_amd import binary
from p2p_llm_tunnel_amd.utils import framepeer as fp
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn, start_proxy, start_serve, start_signal


def _sse(port):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=20)
    c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
    r = c.getresponse()
    return r.status, r.read().count(b"data: ")


def test_matching_secrets_connect(mock_upstream):
    env = {"TUNNEL_SECRET": "correct horse battery staple"}
    with Tunnel(mock_upstream, transport="webrtc", env=env) as t:
        assert _sse(t.proxy_port) == (200, 7)
        assert '"psk"' in t.proxy.text() and "psk_mac" in t.serve.text()


def _pair(mock_upstream, serve_env, proxy_env):
    signal, sp = start_signal()
    room = f"psk-{time.time_ns()}"
    extra = ["--max-retries", "1"]
    serve = start_serve(room, mock_upstream, sp, extra, serve_env)
    proxy = start_proxy(room, f"127.0.0.1:{free_port()}", sp, extra, proxy_env)
    return [signal, serve, proxy]


def _stop(procs):
    for p in reversed(procs):
        p.stop()


def test_wrong_or_missing_secret_is_rejected_by_serve(mock_upstream):
    for proxy_env in ({"TUNNEL_SECRET": "wrong"}, None):
        procs = _pair(mock_upstream, {"TUNNEL_SECRET": "right"}, proxy_env)
        try:
            signal, serve, proxy = procs
            serve.wait_for("authentication failed: HELLO without a valid shared-secret proof", 30)
            assert proxy.count("proxy listening") == 0
        finally:
            _stop(procs)


def test_proxy_requires_proof_from_serve(mock_upstream):
    """A proxy with a secret refuses a serve side that cannot prove it (no
    downgrade to the unauthenticated reference handshake)."""
    procs = _pair(mock_upstream, None, {"TUNNEL_SECRET": "s"})
    try:
        signal, serve, proxy = procs
        proxy.wait_for("authentication failed: peer did not prove the shared secret", 30)
        assert proxy.count("proxy listening") == 0
    finally:
        _stop(procs)


def test_psk_wire_format(mock_upstream):
    """Scripted peer over the TCP transport (channel binding ""): HELLO proof
    accepted, AGREE proof verifiable with plain HMAC-SHA256."""
    secret = b"s3cr3t"
    port = free_port()
    proc = spawn("serve", [binary("tunnel"), "serve", "--room", "x", "--upstream", mock_upstream, "--transport",
                           f"tcp-listen:127.0.0.1:{port}", "--max-retries", "0"], env={"TUNNEL_SECRET": secret.decode()})
    try:
        proc.wait_for("tcp transport: listening", 10)
        peer = fp.FramePeer.connect(port)
        nonce = os.urandom(16).hex()
        mac = hmac.new(secret, f"p2pt-psk|hello|{nonce}|".encode(), hashlib.sha256).hexdigest()
        peer.send_json(fp.HELLO, 0, {"proto": "httptunnel", "min_version": 1, "max_version": 1,
                                     "features": ["sse", "psk"], "psk_nonce": nonce, "psk_mac": mac})
        t, sid, p = peer.recv()
        agree = json.loads(p)
        assert t == fp.AGREE and agree["features"] == ["sse", "psk"]
        assert agree["psk_mac"] == hmac.new(secret, f"p2pt-psk|agree|{nonce}|".encode(), hashlib.sha256).hexdigest()
        peer.close()
    finally:
        proc.stop()
