#!/usr/bin/env python3
"""Node-topology benchmark: ONE tunnel carrying a whole 8-GPU node.

One ``tunnel serve --upstream u0,...,u7`` fronts eight upstreams (one
inference endpoint per GPU; here eight native mocks), one ``tunnel proxy``
faces the clients, and ``tunnel-loadgen`` drives N concurrent SSE streams
through it. Tokens come every ``--interval-us`` (1 ms by default: a fast
decoder), ``--tokens`` per response. The direct baseline is the same load
generator spread over the eight mocks with no tunnel.

Per stream count it reports events/s (SSE token events delivered to clients),
TTFT p50/p99 and inter-token latency (ITL) p50/p99/p99.9, tunneled and direct,
plus the tunnel processes' CPU seconds. This is the workload the reference
would run on tokio's multi-threaded runtime (reference tunnel/src/main.rs:18,
serve.rs:131-137); here it measures the tunnel's worker threads
(``--workers``, native/tunnel/workers.h).

Each point alternates direct and tunneled runs of --seconds (10) each,
--reps (5) times, and reports median and min-max ("rows"; raw runs in "runs").

    python bench/bench_node.py --streams 256,512,1024 --workers auto [--seconds 10 --reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def start_mocks(n, interval_us, tokens, threads=1):
    mocks, ports = [], []
    for _ in range(n):
        port = free_port()
        p = spawn("mock", [binary("tunnel-mock"), "--port", str(port), "--interval-us", str(interval_us),
                           "--tokens", str(tokens), "--threads", str(threads)])
        p.wait_for("Mock LLM server running", 30)
        mocks.append(p)
        ports.append(port)
    return mocks, ports


def loadgen(targets, streams, steps, threads, warmup=1, extra=()):
    out = subprocess.run([binary("tunnel-loadgen"), "--target", ",".join(f"127.0.0.1:{p}" for p in targets),
                          "--streams", str(streams), "--steps", str(steps), "--warmup", str(warmup),
                          "--threads", str(threads), "--warm-conns", "1", *extra],
                         capture_output=True, text=True, timeout=900)
    try:
        return json.loads(out.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError):
        raise RuntimeError(f"loadgen failed (rc={out.returncode}): {out.stdout[-500:]} {out.stderr[-500:]}")


def cpu_s(pid):
    """utime + stime of a process, seconds."""
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


def row(kind, r):
    return {f"{kind}_{k}": r[k] for k in ("events_s", "req_s", "p50_ttft_ms", "p99_ttft_ms", "p50_itl_ms",
                                           "p99_itl_ms", "p999_itl_ms", "max_itl_ms", "errors")}


def summary(vals):
    v = sorted(x for x in vals if x is not None)
    if not v:
        return None
    return {"median": round(statistics.median(v), 4), "min": round(v[0], 4), "max": round(v[-1], 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="256,512,1024")
    ap.add_argument("--upstreams", type=int, default=8)
    ap.add_argument("--interval-us", type=int, default=1000)
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=10.0, help="length of each run (repeated steps)")
    ap.add_argument("--reps", type=int, default=5, help="alternating direct / tunneled repetitions per point")
    ap.add_argument("--workers", default="auto", help="comma list of tunnel --workers values to compare")
    ap.add_argument("--lg-threads", type=int, default=4)
    ap.add_argument("--transport", default="webrtc")
    ap.add_argument("--extra", default="", help="extra flags for both tunnel processes")
    ap.add_argument("--profile-dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ensure_native()
    counts = [int(x) for x in a.streams.split(",") if x]
    mocks, ports = start_mocks(a.upstreams, a.interval_us, a.tokens)
    res = {"host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "upstreams": a.upstreams, "interval_us": a.interval_us, "tokens": a.tokens, "seconds_per_run": a.seconds,
           "reps": a.reps, "transport": a.transport, "cpus": os.cpu_count(), "runs": [], "rows": []}
    dur = ["--duration-s", str(a.seconds)]
    try:
        for w in [x for x in a.workers.split(",") if x]:
            extra = ["--workers", w] + [x for x in a.extra.split() if x]
            env = {"RUST_LOG": "warn,tunnel::serve=info,tunnel::proxy=info"}
            if a.profile_dir:
                os.makedirs(a.profile_dir, exist_ok=True)
                env["TUNNEL_PROFILE"] = os.path.join(os.path.abspath(a.profile_dir), f"tunnel.w{w}.%p.prof")
                env["TUNNEL_PROFILE_HZ"] = "1000"
            up = ",".join(f"http://127.0.0.1:{p}" for p in ports)
            with Tunnel(up, transport=a.transport, serve_extra=extra, proxy_extra=extra, env=env) as t:
                for s in counts:
                    loadgen([t.proxy_port], s, 1, a.lg_threads, warmup=0)
                    for rep in range(a.reps):
                        d = loadgen(ports, s, 1 << 20, a.lg_threads, extra=dur)
                        c0 = (cpu_s(t.serve.popen.pid), cpu_s(t.proxy.popen.pid))
                        tr = loadgen([t.proxy_port], s, 1 << 20, a.lg_threads, extra=dur)
                        c1 = (cpu_s(t.serve.popen.pid), cpu_s(t.proxy.popen.pid))
                        r = {"workers": w, "streams": s, "rep": rep, **row("tunneled", tr), **row("direct", d),
                             "events_ratio": tr["events_s"] / d["events_s"] if d["events_s"] else None,
                             "added_p50_ttft_ms": tr["p50_ttft_ms"] - d["p50_ttft_ms"],
                             "added_p99_ttft_ms": tr["p99_ttft_ms"] - d["p99_ttft_ms"],
                             "added_p99_itl_ms": tr["p99_itl_ms"] - d["p99_itl_ms"],
                             "serve_cpu_s": round(c1[0] - c0[0], 3), "proxy_cpu_s": round(c1[1] - c0[1], 3),
                             "seconds": tr["seconds"], "direct_seconds": d["seconds"]}
                        res["runs"].append(r)
                        print(json.dumps(r), file=sys.stderr, flush=True)
        keys = ["events_ratio", "tunneled_events_s", "direct_events_s", "added_p50_ttft_ms", "added_p99_ttft_ms",
                "tunneled_p99_ttft_ms", "direct_p99_ttft_ms", "tunneled_p99_itl_ms", "direct_p99_itl_ms",
                "added_p99_itl_ms", "serve_cpu_s", "proxy_cpu_s"]
        for w in [x for x in a.workers.split(",") if x]:
            for s in counts:
                runs = [r for r in res["runs"] if r["workers"] == w and r["streams"] == s]
                row_ = {"workers": w, "streams": s, "reps": len(runs),
                        "errors": sum(r["tunneled_errors"] + r["direct_errors"] for r in runs),
                        "seconds_per_run": summary([r["seconds"] for r in runs])}
                for k in keys:
                    row_[k] = summary([r[k] for r in runs])
                res["rows"].append(row_)
                print(json.dumps({"summary": row_}), file=sys.stderr, flush=True)
    finally:
        for m in mocks:
            m.stop()
    doc = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(doc + "\n")
    print(doc)


if __name__ == "__main__":
    main()
