"""TLS paths: `wss://` signalling (the reference's default is
wss://signal-server.fly.dev, cli.rs:16; tokio-tungstenite + native-tls) and
`https://` upstreams (reqwest + native-tls, serve.rs:62), both through
OpenSSL with system-trust verification and hostname / IP-SAN checks.

Offline, a throwaway CA and server certificate are made with the `openssl`
CLI; a small Python TLS front terminates TLS in front of our plain signal
server / mock upstream; the tunnel binaries trust the CA through
SSL_CERT_FILE (honoured by OpenSSL's default verify paths).
"""
import http.client
import json
import os
import shutil
import socket
import ssl
import subprocess
import threading
import time

import pytest

from p2p_llm_tunnel_amd.utils.procs import free_port, start_proxy, start_serve, start_signal

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")


def _run(*args, cwd):
    subprocess.run(list(args), cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = tmp_path_factory.mktemp("pki")
    _run("openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes",
         "-keyout", "ca.key", "-out", "ca.pem", "-days", "2", "-subj", "/CN=p2pt test CA", cwd=d)
    (d / "ext.cnf").write_text("subjectAltName=DNS:localhost,IP:127.0.0.1\nbasicConstraints=CA:FALSE\n")
    _run("openssl", "req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes",
         "-keyout", "srv.key", "-out", "srv.csr", "-subj", "/CN=localhost", cwd=d)
    _run("openssl", "x509", "-req", "-in", "srv.csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial",
         "-out", "srv.pem", "-days", "2", "-extfile", "ext.cnf", cwd=d)
    return d


class TlsFront:
    """Accepts TLS on 127.0.0.1:port and pipes plaintext to 127.0.0.1:backend."""

    def __init__(self, pki, backend: int):
        self.ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        self.ctx.load_cert_chain(pki / "srv.pem", pki / "srv.key")
        self.backend = backend
        self.sock = socket.create_server(("127.0.0.1", 0))
        self.port = self.sock.getsockname()[1]
        self.handshakes = 0
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        self.sock.settimeout(0.2)
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except (socket.timeout, OSError):
                continue
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        try:
            t = self.ctx.wrap_socket(c, server_side=True)
        except (ssl.SSLError, OSError):
            c.close()
            return
        self.handshakes += 1
        b = socket.create_connection(("127.0.0.1", self.backend))

        def pipe(src, dst):
            try:
                while True:
                    data = src.recv(65536)
                    if not data:
                        break
                    dst.sendall(data)
            except OSError:
                pass
            for s in (src, dst):
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass

        threading.Thread(target=pipe, args=(b, t), daemon=True).start()
        pipe(t, b)

    def stop(self):
        self._stop = True
        self.sock.close()


def _sse(port):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=20)
    c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
    r = c.getresponse()
    return r.status, r.read()


def test_wss_signalling_and_https_upstream(pki, mock_upstream):
    signal, sp = start_signal()
    sig_front = TlsFront(pki, sp)
    up_front = TlsFront(pki, int(mock_upstream.rsplit(":", 1)[1]))
    env = {"SSL_CERT_FILE": str(pki / "ca.pem")}
    room = f"tls-{time.time_ns()}"
    listen = free_port()
    procs = [signal]
    try:
        serve = start_serve(room, f"https://localhost:{up_front.port}", None,
                            ["--signal", f"wss://localhost:{sig_front.port}"], env)
        proxy = start_proxy(room, f"127.0.0.1:{listen}", None, ["--signal", f"wss://127.0.0.1:{sig_front.port}"], env)
        procs += [serve, proxy]
        serve.wait_for("tunnel ready", 30)
        proxy.wait_for("proxy listening", 30)
        st, body = _sse(listen)
        assert st == 200 and body.count(b"data: ") == 7
        assert sig_front.handshakes >= 2 and up_front.handshakes >= 1
    finally:
        for p in reversed(procs):
            p.stop()
        sig_front.stop()
        up_front.stop()


def test_untrusted_certificates_are_rejected(pki, mock_upstream):
    """Without the test CA: the wss:// rendezvous fails verification (and is
    retried by the supervisor), and an https:// upstream answers 502."""
    signal, sp = start_signal()
    sig_front = TlsFront(pki, sp)
    up_front = TlsFront(pki, int(mock_upstream.rsplit(":", 1)[1]))
    room = f"tls-bad-{time.time_ns()}"
    procs = [signal]
    try:
        bad = start_serve(room, mock_upstream, None, ["--signal", f"wss://localhost:{sig_front.port}"],
                          {"SSL_CERT_FILE": os.devnull})
        procs.append(bad)
        line = bad.wait_for(r"serve failed \(attempt 1\)", 20)
        assert "certificate verify failed" in bad.text() or "verify" in line
        bad.stop()
        # https upstream with an untrusted certificate: the tunnel works, the request gets a 502.
        listen = free_port()
        serve = start_serve(room, f"https://localhost:{up_front.port}", sp, [], {"SSL_CERT_FILE": os.devnull})
        proxy = start_proxy(room, f"127.0.0.1:{listen}", sp, [], None)
        procs += [serve, proxy]
        serve.wait_for("tunnel ready", 30)
        proxy.wait_for("proxy listening", 30)
        c = http.client.HTTPConnection("127.0.0.1", listen, timeout=20)
        c.request("GET", "/v1/models")
        r = c.getresponse()
        body = r.read()
        assert r.status == 502 and b"Bad Gateway" in body
    finally:
        for p in reversed(procs):
            p.stop()
        sig_front.stop()
        up_front.stop()
