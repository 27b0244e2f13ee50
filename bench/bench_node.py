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
from p2p_llm_tunnel_amd.utils.boxinfo import identity as _box  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.pinning import cgroup_cpu_stat, cpu_stat_delta  # noqa: E402
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


SCRAPE = ("tunnel_sctp_packets_sent", "tunnel_frames_sent_total", "tunnel_frames_received_total",
          "tunnel_dtls_inline_tx_batches", "tunnel_dtls_lane_tx_batches", "tunnel_dtls_lane_datagrams",
          "tunnel_udp_gso_sends", "tunnel_udp_reader_bursts", "tunnel_udp_reader_datagrams", "tunnel_udp_reader_raw",
          "tunnel_sctp_retransmits", "tunnel_sctp_tlp_probes")


def scrape(port):
    """The SCRAPE counters of one tunnel process's /metrics."""
    import urllib.request
    txt = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    out = {}
    for line in txt.splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[0] in SCRAPE:
            out[parts[0]] = float(parts[1])
    return out


def row(kind, r):
    return {f"{kind}_{k}": r[k] for k in ("events_s", "req_s", "p50_ttft_ms", "p99_ttft_ms", "p50_itl_ms",
                                           "p99_itl_ms", "p999_itl_ms", "max_itl_ms", "errors")}


def summary(vals):
    v = sorted(x for x in vals if x is not None)
    if not v:
        return None
    return {"median": round(statistics.median(v), 4), "min": round(v[0], 4), "max": round(v[-1], 4)}


HOPS = [("proxy", "accept", "proxy", "req_end"), ("proxy", "req_end", "serve", "req_headers"),
        ("serve", "req_headers", "serve", "req_end"), ("serve", "req_end", "serve", "upstream_sent"),
        ("serve", "upstream_sent", "serve", "first_body"), ("serve", "first_body", "serve", "sched_in"),
        ("serve", "sched_in", "serve", "chan_tx"), ("serve", "chan_tx", "proxy", "chan_rx"),
        ("proxy", "chan_rx", "proxy", "first_body"), ("proxy", "accept", "proxy", "first_body"),
        # the two crossings split at the transport stamps (scripts/ttft_breakdown.py)
        ("proxy", "req_end", "proxy", "udp_tx"), ("proxy", "udp_tx", "serve", "udp_kernel"),
        ("serve", "udp_kernel", "serve", "udp_read"), ("serve", "udp_read", "serve", "rx_assoc"),
        ("serve", "rx_assoc", "serve", "req_headers"),
        ("serve", "chan_tx", "serve", "udp_tx"), ("serve", "udp_tx", "proxy", "udp_kernel"),
        ("proxy", "udp_kernel", "proxy", "udp_read"), ("proxy", "udp_read", "proxy", "rx_assoc"),
        ("proxy", "rx_assoc", "proxy", "chan_rx")]


def node_hops(traces, windows):
    """Per (workers, streams): hop p50 over all requests of the tunneled runs,
    and the hops of the slowest 1 % by time inside the tunnel (proxy accept ->
    proxy first_body), median over those requests."""
    ev = {}
    for i, tf in enumerate(traces):  # stream ids restart with every tunnel
        with open(tf) as f:
            for line in f:
                try:
                    e = json.loads(line)
                except ValueError:
                    continue
                ev.setdefault((i, e["sid"]), {})[(e["role"], e["ev"])] = e["t_us"]
    out = []
    for w, s, t0, t1 in windows:
        reqs = [e for e in ev.values() if ("proxy", "accept") in e and ("proxy", "first_body") in e
                and t0 <= e[("proxy", "accept")] <= t1]
        if not reqs:
            continue
        reqs.sort(key=lambda e: e[("proxy", "first_body")] - e[("proxy", "accept")])
        tail = reqs[int(len(reqs) * 0.99):] or reqs[-1:]
        row = {"workers": w, "streams": s, "requests": len(reqs), "tail_requests": len(tail)}
        for a_, b_, c_, d_ in HOPS:
            k = f"{a_}.{b_} -> {c_}.{d_}"
            allv = sorted(e[(c_, d_)] - e[(a_, b_)] for e in reqs if (a_, b_) in e and (c_, d_) in e)
            tv = sorted(e[(c_, d_)] - e[(a_, b_)] for e in tail if (a_, b_) in e and (c_, d_) in e)
            if allv:
                row[k] = {"p50_us": allv[len(allv) // 2], "p99_us": allv[int(0.99 * (len(allv) - 1))],
                          "tail_p50_us": tv[len(tv) // 2] if tv else None}
        out.append(row)
    return out


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
    ap.add_argument("--trace", action="store_true",
                    help="stamp every request's hops (TUNNEL_TRACE, buffered) and report where the slowest 1 %% "
                         "of first tokens spent their time inside the tunnel (\"hops\" per stream count)")
    ap.add_argument("--metrics", action="store_true",
                    help="per tunneled run, the packet / batch / syscall counters of both tunnel processes (deltas)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ensure_native()
    counts = [int(x) for x in a.streams.split(",") if x]
    mocks, ports = start_mocks(a.upstreams, a.interval_us, a.tokens)
    res = {"host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "upstreams": a.upstreams, "interval_us": a.interval_us, "tokens": a.tokens, "seconds_per_run": a.seconds,
           "reps": a.reps, "transport": a.transport, "cpus": os.cpu_count(), "runs": [], "rows": []}
    dur = ["--duration-s", str(a.seconds)]
    windows = []  # (workers, streams, t0_us, t1_us): the tunneled runs, CLOCK_MONOTONIC like the trace
    traces = []
    try:
        for w in [x for x in a.workers.split(",") if x]:
            extra = ["--workers", w] + [x for x in a.extra.split() if x]
            env = {"RUST_LOG": "warn,tunnel::serve=info,tunnel::proxy=info"}
            trace = None
            if a.trace:
                import tempfile
                trace = tempfile.NamedTemporaryFile(suffix=".jsonl", prefix="p2pt-node-trace-", delete=False).name
                env.update({"TUNNEL_TRACE": trace})
            if a.profile_dir:
                os.makedirs(a.profile_dir, exist_ok=True)
                env["TUNNEL_PROFILE"] = os.path.join(os.path.abspath(a.profile_dir), f"tunnel.w{w}.%p.prof@1000")
            up = ",".join(f"http://127.0.0.1:{p}" for p in ports)
            if trace:
                traces.append(trace)
            mports = (free_port(), free_port()) if a.metrics else None
            mx = (["--metrics-listen", f"127.0.0.1:{mports[0]}"], ["--metrics-listen", f"127.0.0.1:{mports[1]}"]) \
                if mports else ([], [])
            with Tunnel(up, transport=a.transport, serve_extra=extra + mx[0], proxy_extra=extra + mx[1], env=env) as t:
                for s in counts:
                    loadgen([t.proxy_port], s, 1, a.lg_threads, warmup=0)
                    sid_lo = None
                    for rep in range(a.reps):
                        g0 = cgroup_cpu_stat()
                        d = loadgen(ports, s, 1 << 20, a.lg_threads, extra=dur)
                        g1 = cgroup_cpu_stat()
                        c0 = (cpu_s(t.serve.popen.pid), cpu_s(t.proxy.popen.pid))
                        m0 = (scrape(mports[0]), scrape(mports[1])) if mports else None
                        t_tr0 = time.monotonic_ns() // 1000
                        tr = loadgen([t.proxy_port], s, 1 << 20, a.lg_threads, extra=dur)
                        t_tr1 = time.monotonic_ns() // 1000
                        c1 = (cpu_s(t.serve.popen.pid), cpu_s(t.proxy.popen.pid))
                        g2 = cgroup_cpu_stat()
                        m1 = (scrape(mports[0]), scrape(mports[1])) if mports else None
                        if trace:
                            windows.append((w, s, t_tr0, t_tr1))
                        r = {"workers": w, "streams": s, "rep": rep, **row("tunneled", tr), **row("direct", d),
                             "events_ratio": tr["events_s"] / d["events_s"] if d["events_s"] else None,
                             "added_p50_ttft_ms": tr["p50_ttft_ms"] - d["p50_ttft_ms"],
                             "added_p99_ttft_ms": tr["p99_ttft_ms"] - d["p99_ttft_ms"],
                             "added_p99_itl_ms": tr["p99_itl_ms"] - d["p99_itl_ms"],
                             "serve_cpu_s": round(c1[0] - c0[0], 3), "proxy_cpu_s": round(c1[1] - c0[1], 3),
                             "seconds": tr["seconds"], "direct_seconds": d["seconds"],
                             # job-wide CPU use and quota throttling during each leg
                             "direct_cgroup": cpu_stat_delta(g0, g1), "tunneled_cgroup": cpu_stat_delta(g1, g2)}
                        if m0:
                            for side, x0, x1 in (("serve", m0[0], m1[0]), ("proxy", m0[1], m1[1])):
                                r[f"{side}_counters"] = {k[len("tunnel_"):]: x1[k] - x0.get(k, 0.0) for k in x1}
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
        if traces:
            res["hops"] = node_hops(traces, windows)
    finally:
        for m in mocks:
            m.stop()
        for tf in traces:
            if os.path.exists(tf):
                os.unlink(tf)
    res["box"] = _box()
    doc = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(doc + "\n")
    print(doc)


if __name__ == "__main__":
    main()
