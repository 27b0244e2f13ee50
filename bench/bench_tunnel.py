#!/usr/bin/env python3
"""Benchmark matrix for BASELINE.md (SURVEY §4.2 "Bench", BASELINE.json configs).

  1. SSE streaming, 1/2/4/8 streams: tunneled vs direct req/s and TTFT, for the
     native mock, the threaded Python mock, and the reference's unthreaded
     (single-threaded, HTTP/1.0) Python mock; WebRTC and TCP transports.
  2. 64 concurrent streams x 1 MB POST bodies (REQ_BODY chunking + back-pressure).
  4. NAT traversal (config #4): both peers behind emulated port-restricted
     cone NATs (TUNNEL_NAT, native/rtc/ice.h), STUN-only ICE against a local
     STUN server, SSE at 1/8 streams through the hole-punched srflx path.
  3. Idle then burst: the tunnel sits idle (PING/PONG keepalive running), then
     16 concurrent streams (the 30-minute idle of config #5 is scaled down via
     --idle-s; keepalive behaviour is identical for any idle length).

Writes a JSON document (default: stdout) with every measured point.
``--std-mtu`` runs every WebRTC row on the standard 1200-byte SCTP packet
path (``--no-jumbo-loopback``) that cross-host deployments use; rows are then
labelled ``webrtc-1200``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT))

from bench import loadgen, start_mock  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel  # noqa: E402
from p2p_llm_tunnel_amd.utils.boxinfo import identity as _box  # noqa: E402


MTU_EXTRA: list[str] = []  # ["--no-jumbo-loopback"] with --std-mtu


def label(transport):
    return transport + ("-1200" if MTU_EXTRA and transport == "webrtc" else "")


def sse_matrix(transport, mock_kind, streams_list, steps, threaded=True, busy_poll_us=0, path=None, nat=None):
    mock, port = start_mock(mock_kind, 100, 5) if (mock_kind == "native" or threaded) else _unthreaded()
    rows = []
    extra = (["--busy-poll-us", str(busy_poll_us)] if busy_poll_us else []) + (MTU_EXTRA if transport == "webrtc" else [])
    env = None
    stun = None
    if nat:
        from p2p_llm_tunnel_amd.utils.turn_server import TurnServer
        stun = TurnServer().start()
        extra += ["--stun", f"stun:127.0.0.1:{stun.port}"]
        env = {"TUNNEL_NAT": nat}
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport, serve_extra=extra, proxy_extra=extra,
                    env=env) as t:
            for s in streams_list:
                loadgen(t.proxy_port, s, 1, path=path)
                tr = loadgen(t.proxy_port, s, steps, path=path)
                if not threaded:
                    time.sleep(1.3)  # let serve's spare upstream sockets expire (single-threaded upstream)
                dr = loadgen(port, s, steps, path=path)
                rows.append({"transport": label(transport) + (f"+nat:{nat}" if nat else ""),
                             "mock": mock_kind if threaded else "python-unthreaded",
                             "busy_poll_us": busy_poll_us, "path": path or "/v1/chat/completions",
                             "streams": s, "tunneled_req_s": tr["req_s"], "direct_req_s": dr["req_s"],
                             "tunneled_p50_ttft_ms": tr["p50_ttft_ms"], "direct_p50_ttft_ms": dr["p50_ttft_ms"],
                             "added_p50_ttft_ms": tr["p50_ttft_ms"] - dr["p50_ttft_ms"],
                             "tunneled_p99_ttft_ms": tr["p99_ttft_ms"], "errors": tr["errors"] + dr["errors"]})
                print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    finally:
        mock.stop()
        if stun:
            stun.stop()
    return rows


def _unthreaded():
    from p2p_llm_tunnel_amd.utils.procs import free_port, spawn
    port = free_port()
    p = spawn("mock", [sys.executable, "-m", "p2p_llm_tunnel_amd.utils.mock_llm", "--port", str(port)])
    p.wait_for("Mock LLM server running", 30)
    return p, port


def post_1mb(transport, streams=64, mb=1, steps=2):
    mock, port = start_mock("native", 100, 5)
    try:
        ex = MTU_EXTRA if transport == "webrtc" else []
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport, serve_extra=ex, proxy_extra=ex) as t:
            from p2p_llm_tunnel_amd import binary
            import subprocess
            def run(target):
                out = subprocess.run([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{target}", "--streams",
                                      str(streams), "--steps", str(steps), "--warmup", "1", "--post-bytes",
                                      str(mb << 20)], capture_output=True, text=True, timeout=600)
                return json.loads(out.stdout.strip().splitlines()[-1])
            tr, dr = run(t.proxy_port), run(port)
            # request + echoed response both cross the tunnel
            row = {"transport": label(transport), "streams": streams, "body_mb": mb,
                   "tunneled_req_s": tr["req_s"], "direct_req_s": dr["req_s"],
                   "tunneled_MBps_each_way": tr["req_s"] * mb * 1.048576,
                   "tunneled_p50_total_ms": tr["p50_total_ms"], "direct_p50_total_ms": dr["p50_total_ms"],
                   "errors": tr["errors"] + dr["errors"]}
            print(json.dumps(row), file=sys.stderr, flush=True)
            return row
    finally:
        mock.stop()


def idle_burst(transport, idle_s=30, burst=16):
    mock, port = start_mock("native", 100, 5)
    try:
        ex = MTU_EXTRA if transport == "webrtc" else []
        with Tunnel(f"http://127.0.0.1:{port}", transport=transport, serve_extra=ex, proxy_extra=ex,
                    env={"RUST_LOG": "info,tunnel::serve=debug"}) as t:
            loadgen(t.proxy_port, 1, 1)
            pings0 = t.serve.count("sent keepalive ping")
            t_end = time.time() + idle_s
            while time.time() < t_end:  # a progress line every 30 s (long idles must not look hung)
                time.sleep(min(30.0, max(0.0, t_end - time.time())))
                print(json.dumps({"idle_progress_s": round(idle_s - max(0.0, t_end - time.time()), 1),
                                  "pings": t.serve.count("sent keepalive ping") - pings0}), file=sys.stderr, flush=True)
            pings = t.serve.count("sent keepalive ping") - pings0
            r = loadgen(t.proxy_port, burst, 1)
            d = loadgen(port, burst, 1)
            row = {"transport": label(transport), "idle_s": idle_s, "burst_streams": burst, "pings_during_idle": pings,
                   "tunneled_req_s": r["req_s"], "tunneled_p50_ttft_ms": r["p50_ttft_ms"],
                   "direct_p50_ttft_ms": d["p50_ttft_ms"], "added_p50_ttft_ms": r["p50_ttft_ms"] - d["p50_ttft_ms"],
                   "errors": r["errors"]}
            print(json.dumps(row), file=sys.stderr, flush=True)
            return row
    finally:
        mock.stop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--idle-s", type=float, default=30)
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true", help="native mock + webrtc only")
    ap.add_argument("--busy-poll", default="", help="comma-separated busy-poll µs values to add as extra SSE rows")
    ap.add_argument("--std-mtu", action="store_true", help="WebRTC rows on the 1200-byte SCTP packet path")
    a = ap.parse_args()
    if a.std_mtu:
        MTU_EXTRA.append("--no-jumbo-loopback")
    ensure_native()
    res = {"host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "sse": []}
    streams = [1, 2, 4, 8]
    res["sse"] += sse_matrix("webrtc", "native", streams, a.steps)
    if not a.quick:
        res["sse"] += sse_matrix("tcp", "native", streams, a.steps)
        res["sse"] += sse_matrix("webrtc", "python", streams, a.steps)
        res["sse"] += sse_matrix("webrtc", "python", [1, 2, 4, 8], 3, threaded=False)
    # BASELINE config #2: Ollama /api/generate NDJSON stream, up to 8 concurrent streams.
    res["sse"] += sse_matrix("webrtc", "native", [1, 8], a.steps, path="/api/generate")
    # Beyond the 1-8 stream curve: 64 and 256 concurrent SSE streams on one tunnel.
    res["sse"] += sse_matrix("webrtc", "native", [64, 256], max(2, a.steps // 2))
    # BASELINE config #4: NAT traversal (emulated port-restricted NATs, STUN-only ICE).
    res["sse"] += sse_matrix("webrtc", "native", [1, 8], a.steps, nat="port-restricted")
    for bp in [int(x) for x in a.busy_poll.split(",") if x]:
        res["sse"] += sse_matrix("webrtc", "native", [1, 8], a.steps, busy_poll_us=bp)
    res["post_64x1MB"] = [post_1mb("webrtc")]
    if not a.quick:
        res["post_64x1MB"].append(post_1mb("tcp"))
    res["idle_burst"] = idle_burst("webrtc", a.idle_s)
    res["box"] = _box()
    doc = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(doc + "\n")
    print(doc)


if __name__ == "__main__":
    main()
