"""TURN relay path (--turn/--turn-user/--turn-pass; reference cli.rs:30-40,
rtc.rs:54-63). Both peers are forced onto relayed candidates
(--ice-relay-only) so every datagram crosses the test TURN server, reached
over UDP, TCP (turn:...?transport=tcp) or TLS (turns:...), the transports a
firewalled network leaves open. URLs the client cannot honour are refused."""
import http.client
import json
import shutil
import ssl
import subprocess
import urllib.request

import pytest

from p2p_llm_tunnel_amd import binary
from p2p_llm_tunnel_amd.utils.procs import Tunnel
from p2p_llm_tunnel_amd.utils.turn_server import TurnServer


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    d = tmp_path_factory.mktemp("turnpki")

    def run(*args):
        subprocess.run(list(args), cwd=d, check=True, capture_output=True)

    run("openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes",
        "-keyout", "ca.key", "-out", "ca.pem", "-days", "2", "-subj", "/CN=p2pt turn test CA")
    (d / "ext.cnf").write_text("subjectAltName=DNS:localhost,IP:127.0.0.1\nbasicConstraints=CA:FALSE\n")
    run("openssl", "req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes",
        "-keyout", "srv.key", "-out", "srv.csr", "-subj", "/CN=localhost")
    run("openssl", "x509", "-req", "-in", "srv.csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial",
        "-out", "srv.pem", "-days", "2", "-extfile", "ext.cnf")
    return d


def _server(transport, pki=None):
    ctx = None
    if transport == "tls":
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(pki / "srv.pem", pki / "srv.key")
    return TurnServer(user="alice", password="s3cret", transport=transport, ssl_ctx=ctx).start()


@pytest.mark.parametrize("transport", ["udp", "tcp", "tls"])
def test_tunnel_through_turn_relay(mock_upstream, transport, request):
    pki = request.getfixturevalue("pki") if transport == "tls" else None
    turn = _server(transport, pki)
    env = {"RUST_LOG": "info,tunnel::rtc=debug,tunnel::turn=info"}
    if pki:
        env["SSL_CERT_FILE"] = str(pki / "ca.pem")  # the relay's certificate is verified, not trusted blindly
    try:
        extra = ["--turn", turn.url, "--turn-user", "alice", "--turn-pass", "s3cret", "--ice-relay-only"]
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra, env=env) as t:
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
            # One allocation per association (the first, plus the "assoc"
            # extension's extra ones on this short path), each relayed.
            assert 1 <= t.serve.count("TURN allocation: relayed") <= 3
        assert turn.stats["allocations"] >= 2
        assert turn.stats["relayed_to_peer"] > 50 and turn.stats["relayed_to_client"] > 50
        assert turn.stats["channel_binds"] >= 2
        if transport != "udp":
            assert turn.stats["stream_connections"] >= 2
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


def test_turns_with_untrusted_certificate_fails_gathering_gracefully(mock_upstream, pki):
    """A TLS relay whose certificate does not verify gives no relayed
    candidate (the host path still connects) instead of an unauthenticated
    relay."""
    turn = _server("tls", pki)
    try:
        extra = ["--turn", turn.url, "--turn-user", "alice", "--turn-pass", "s3cret"]
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra, proxy_extra=extra) as t:
            assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"
            assert "TURN allocation: relayed" not in t.serve.text()
        assert turn.stats["allocations"] == 0
    finally:
        turn.stop()


@pytest.mark.parametrize("url,msg", [
    ("stun:relay.example.com", "unsupported TURN URL scheme 'stun:'"),
    ("turns:relay.example.com?transport=udp", "turns: over udp (DTLS) is not supported"),
    ("turn:relay.example.com?transport=sctp", "unsupported TURN transport 'sctp'"),
    ("relay.example.com:3478", "unsupported TURN URL scheme"),
])
def test_unsupported_turn_url_is_refused(url, msg):
    r = subprocess.run([binary("tunnel"), "proxy", "--room", "x", "--turn", url, "--signal", "ws://127.0.0.1:1",
                        "--max-retries", "0"], capture_output=True, text=True, timeout=10)
    assert r.returncode == 2 and msg in r.stderr, (r.returncode, r.stderr)


def _final_pair(proc):
    """The selected pair a tunnel process ended on: its "connection
    established via" line, or a later ICE pair switch."""
    pair = None
    for line in proc.text().splitlines():
        for key in ("WebRTC connection established", "ICE pair switched to "):
            if key in line:
                pair = (line.split(" via ", 1)[-1] if key.startswith("WebRTC") else line.split(key, 1)[1])
                pair = pair.split(" mtu=")[0].split(" (")[0]
    return pair


def test_relay_only_side_and_host_side_agree_on_the_pair(mock_upstream):
    # serve on its relayed candidate only, the proxy on its host candidates.
    # The relay (on loopback) reaches every host candidate, so serve checks and
    # nominates each; the proxy pairs loopback only with loopback and had no
    # pair for a nominated non-loopback one: it kept sending from its loopback
    # socket while serve sent to the other one (on the MI355X host the proxy's
    # socket reader then held a socket the data never came to; a 20 ms relay
    # row stalled). Both must end on the same pair.
    turn = _server("udp")
    env = {"RUST_LOG": "info"}
    try:
        extra = ["--turn", turn.url, "--turn-user", "alice", "--turn-pass", "s3cret", "--ice-relay-only"]
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=extra + ["--assoc", "1"],
                    proxy_extra=["--assoc", "1"], env=env) as t:
            c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=30)
            c.request("POST", "/echo", body=b"q" * 100000)
            assert c.getresponse().read() == b"q" * 100000
            s, p = _final_pair(t.serve), _final_pair(t.proxy)
            assert s and p and s.startswith("relay:"), (s, p)
            s_local, s_remote = s.split(":", 1)[1].split(" <-> ")
            p_local, p_remote = p.split(":", 1)[1].split(" <-> ")
            assert (s_local, s_remote) == (p_remote, p_local), (s, p)
    finally:
        turn.stop()
