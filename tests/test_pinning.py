"""Persistent DTLS identity + certificate pinning (`--identity`, `--pin-peer`,
`tunnel fingerprint`): the reference README lists "certificate pinning via
WebRTC DTLS fingerprints" as a future option (README.md:103-105). Without
these flags every process has a fresh ephemeral certificate, as in the
reference."""
import os
import stat
import subprocess
import time
import urllib.request

from p2p_llm_tunnel_amd import binary
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, start_proxy, start_serve, start_signal


def _fp(path):
    out = subprocess.run([binary("tunnel"), "fingerprint", "--identity", path], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    return out.stdout.strip()


def test_fingerprint_subcommand_creates_stable_identity(tmp_path):
    path = str(tmp_path / "id.pem")
    fp = _fp(path)
    assert fp.startswith("sha-256 ") and len(fp.split()[1].split(":")) == 32
    assert stat.S_IMODE(os.stat(path).st_mode) == 0o600
    assert _fp(path) == fp  # loaded, not regenerated
    text = open(path).read()
    assert "BEGIN PRIVATE KEY" in text and "BEGIN CERTIFICATE" in text


def test_mutual_pinning_connects(mock_upstream, tmp_path):
    a, b = str(tmp_path / "serve.pem"), str(tmp_path / "proxy.pem")
    fa, fb = _fp(a), _fp(b)
    # accepted spellings: "sha-256 AB:..", bare lower-case hex
    with Tunnel(mock_upstream, transport="webrtc",
                serve_extra=["--identity", a, "--pin-peer", fb],
                proxy_extra=["--identity", b, "--pin-peer", "ff" * 32 + "," + fa.split()[1].replace(":", "").lower()]) as t:
        assert urllib.request.urlopen(t.url + "/health", timeout=10).read() == b"ok"
        assert f"DTLS identity {a}: {fa}" in t.serve.text()
        assert "accepting only 2 pinned peer certificate(s)" in t.proxy.text()


def test_unpinned_peer_is_rejected(mock_upstream, tmp_path):
    a = str(tmp_path / "serve.pem")
    _fp(a)
    signal, sp = start_signal()
    room = f"pin-{time.time_ns()}"
    extra = ["--max-retries", "1"]
    serve = start_serve(room, mock_upstream, sp, extra + ["--identity", a])
    proxy = start_proxy(room, f"127.0.0.1:{free_port()}", sp, extra + ["--pin-peer", "AB" * 32])
    try:
        proxy.wait_for("is not pinned", 30)
        assert proxy.count("proxy listening") == 0
    finally:
        for p in (proxy, serve, signal):
            p.stop()


def test_bad_pin_and_bad_identity_exit_2(tmp_path):
    out = subprocess.run([binary("tunnel"), "proxy", "--room", "r", "--pin-peer", "sha-256 12:34"],
                         capture_output=True, text=True)
    assert out.returncode == 2 and "is not a SHA-256 fingerprint" in out.stderr
    bad = tmp_path / "bad.pem"
    bad.write_text("not a key\n")
    out = subprocess.run([binary("tunnel"), "proxy", "--room", "r", "--identity", str(bad)],
                         capture_output=True, text=True)
    assert out.returncode == 2 and "not a PEM private key" in out.stderr
