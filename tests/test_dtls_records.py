"""DTLS record-layer interop: our AES-GCM record layer (VAES/VPCLMULQDQ when
the CPU has it, OpenSSL EVP otherwise; native/core/aesgcm.h,
native/rtc/dtls.cc) against a peer that keeps OpenSSL's own DTLS record
layer (TUNNEL_DTLS_RECORDS=openssl, i.e. a standard DTLS 1.2 stack on the
wire) and against a peer on the EVP record path (TUNNEL_DTLS_RECORDS=evp).

Large echoed bodies cross every record size the SCTP packer produces, in
both directions; the SSE stream checks small records.
"""
import http.client
import json
import time

import pytest

from p2p_llm_tunnel_amd.utils.procs import free_port, start_proxy, start_serve, start_signal

CASES = {
    "openssl-records-vs-own": ({"TUNNEL_DTLS_RECORDS": "openssl"}, None),
    "own-vs-openssl-records": (None, {"TUNNEL_DTLS_RECORDS": "openssl"}),
    "evp-vs-vector": ({"TUNNEL_DTLS_RECORDS": "evp"}, None),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_record_layer_interop(mock_upstream, case):
    serve_env, proxy_env = CASES[case]
    env_dbg = {"TUNNEL_LOG": "debug"}
    signal, sp = start_signal()
    room = f"dtls-{time.time_ns()}"
    port = free_port()
    serve = start_serve(room, mock_upstream, sp, None, {**env_dbg, **(serve_env or {})})
    proxy = start_proxy(room, f"127.0.0.1:{port}", sp, None, {**env_dbg, **(proxy_env or {})})
    try:
        proxy.wait_for("proxy listening on", 30)
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        for n in (1, 1199, 70_000, 2_500_001):
            body = bytes((i * 7 + n) & 0xFF for i in range(n))
            c.request("POST", "/echo", body=body)
            r = c.getresponse()
            assert r.status == 200 and r.read() == body, n
        c.request("POST", "/v1/chat/completions", body=json.dumps({"stream": True}))
        r = c.getresponse()
        assert r.status == 200 and r.read().count(b"data: ") == 7
        c.close()
        armed = {p.name: [l for l in p.text().splitlines() if "own record layer armed" in l] for p in (serve, proxy)}
        for name, env in (("serve", serve_env), ("proxy", proxy_env)):
            if env and env.get("TUNNEL_DTLS_RECORDS") == "openssl":
                assert armed[name] == []
            else:
                # One per association (the first, and the "assoc" extension's
                # extra ones the 2.5 MB echo may have used), all on the same path.
                assert 1 <= len(armed[name]) <= 3, armed[name]
                if env and env.get("TUNNEL_DTLS_RECORDS") == "evp":
                    assert all("EVP AES-GCM" in a for a in armed[name])
    finally:
        for p in (proxy, serve, signal):
            p.stop()
