#!/usr/bin/env python3
"""Head-of-line benchmark: SSE token streams sharing one tunnel with bulk
downloads and a slow client.

    8 SSE streams (a token every --interval-ms, --tokens per response)
  + 8 concurrent 64 MB downloads (GET /bulk), repeated while the SSE runs
  + 1 client reading a 64 MB download at 100 KB/s

The reference sends every frame straight into its one ordered data channel
with no scheduling or back-pressure (reference serve.rs:274, proxy.rs:391-419),
so a token waits behind whatever body bytes were queued before it. Reported
per transport (jumbo same-host packets and the standard 1200-byte path):
inter-token latency (ITL) p50/p99/max of the SSE streams, tunneled vs direct
(the same load straight to the upstream), the added ITL p99, bulk MB/s, and
the proxy's peak RSS (the slow client must not make it grow), and the SSE
time to first token (TTFT) p99 next to the bulk, tunneled vs direct.

Each run lasts --seconds (10 by default) with the downloads repeating for its
whole length; --reps alternating direct / tunneled repetitions (5) are
summarised as median and min-max per transport ("rows"), raw runs in "runs".

    python bench/bench_mixed.py [--transports jumbo,std] [--seconds 10] [--reps 5] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.boxinfo import identity as _box  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def rss_kb(pid):
    try:
        for line in open(f"/proc/{pid}/status"):
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    except OSError:
        pass
    return 0


def cpu_stat():
    """The job cgroup's CPU-quota counters (cgroup v2 cpu.stat): usage and how
    often / how long the quota throttled every thread of the job. {} when not
    readable."""
    out = {}
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def stat_delta(a, b):
    """Usage, periods and throttling over one run (cpu_stat() before / after)."""
    if not a or not b:
        return None
    d = {k: b[k] - a.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec") if k in b}
    return d


def lg(port, *args, timeout=600):
    return subprocess.Popen([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{port}", *map(str, args)],
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)


def result(p, timeout=600):
    out, _ = p.communicate(timeout=timeout)
    return json.loads(out.strip().splitlines()[-1])


def slow_reader(port, rate, stop, stats):
    """Reads a 64 MB download at `rate` bytes/s until stopped."""
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"GET /bulk?bytes=67108864 HTTP/1.1\r\nHost: x\r\n\r\n")
    s.settimeout(1)
    t0, got = time.time(), 0
    while not stop.is_set():
        due = t0 + got / rate
        if time.time() < due:
            time.sleep(min(0.01, due - time.time()))
            continue
        try:
            d = s.recv(8192)
        except socket.timeout:
            continue
        if not d:
            break
        got += len(d)
    stats["slow_bytes"] = got
    s.close()


def scenario(port, a, watch_pid=None):
    """Bulk + slow reader + SSE against `port` for a.seconds; returns the SSE
    loadgen result etc. The bulk downloads start first and run until after
    the SSE load ends, so every token competes with them."""
    stop = threading.Event()
    stats = {}
    peak = [0]

    def watch():
        while not stop.is_set():
            if watch_pid:
                peak[0] = max(peak[0], rss_kb(watch_pid))
            time.sleep(0.05)

    w = threading.Thread(target=watch)
    w.start()
    sr = threading.Thread(target=slow_reader, args=(port, a.slow_rate, stop, stats))
    sr.start()
    bulk = lg(port, "--streams", a.bulk_streams, "--steps", 1 << 20, "--warmup", 0, "--method", "GET",
              "--path", f"/bulk?bytes={a.bulk_mb << 20}", "--events", "none", "--duration-s", a.seconds + 0.5)
    time.sleep(0.3)
    sse = lg(port, "--streams", a.sse_streams, "--steps", 1 << 20, "--warmup", 1, "--warm-conns", 1,
             "--duration-s", a.seconds)
    sse_r = result(sse)
    bulk_r = result(bulk)
    stop.set()
    sr.join()
    w.join()
    return sse_r, bulk_r, stats, peak[0]


def summary(vals):
    v = sorted(x for x in vals if x is not None)
    if not v:
        return None
    return {"median": round(statistics.median(v), 3), "min": round(v[0], 3), "max": round(v[-1], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transports", default="jumbo,std")
    ap.add_argument("--interval-ms", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=100)
    ap.add_argument("--sse-streams", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=10.0, help="length of each run (SSE load; bulk overlaps it)")
    ap.add_argument("--reps", type=int, default=5, help="alternating direct / tunneled repetitions")
    ap.add_argument("--bulk-streams", type=int, default=8)
    ap.add_argument("--bulk-mb", type=int, default=64)
    ap.add_argument("--slow-rate", type=int, default=100 * 1024)
    ap.add_argument("--extra", default="", help="extra flags for both tunnel processes")
    ap.add_argument("--mock-threads", type=int, default=4,
                    help="reactor threads of the native mock (it serves the SSE and the downloads, tunneled and direct)")
    ap.add_argument("--profile-dir", default=None,
                    help="sampling CPU profile of every tunnel process (TUNNEL_PROFILE), reports next to it")
    ap.add_argument("--timeline", action="store_true",
                    help="per-thread CPU utilisation of both tunnels in 2 ms intervals (which stage saturates)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ensure_native()
    mport = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(mport), "--interval-ms", str(a.interval_ms),
                          "--tokens", str(a.tokens), "--threads", str(a.mock_threads)])
    tl_dir, tl_env = None, None
    if a.timeline:
        from p2p_llm_tunnel_amd.utils import timeline
        tl_dir, tl_env = timeline.new_dir()
    if a.profile_dir:
        os.makedirs(a.profile_dir, exist_ok=True)
        tl_env = dict(tl_env or {}, TUNNEL_PROFILE=os.path.join(os.path.abspath(a.profile_dir), "tunnel.%p.prof@1000"))
    mock.wait_for("Mock LLM server running", 10)
    trs = [x for x in a.transports.split(",") if x]
    res = {"host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "sse": f"{a.sse_streams} streams x {a.tokens} tokens @ {a.interval_ms} ms",
           "bulk": f"{a.bulk_streams} x {a.bulk_mb} MB GET, repeated for the whole run",
           "slow_client_Bps": a.slow_rate, "seconds_per_run": a.seconds, "reps": a.reps, "extra": a.extra,
           "mock_threads": a.mock_threads,
           "runs": [], "rows": []}
    tunnels = {}
    try:
        for tr in trs:
            extra = [x for x in a.extra.split() if x] + (["--no-jumbo-loopback"] if tr == "std" else [])
            t = Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc", serve_extra=extra, proxy_extra=extra, env=tl_env)
            t.__enter__()
            tunnels[tr] = t
        for rep in range(a.reps):
            c0 = cpu_stat()
            d_sse, d_bulk, _, _ = scenario(mport, a)
            d_cg = stat_delta(c0, cpu_stat())
            print(json.dumps({"rep": rep, "direct_itl_p99_ms": d_sse["p99_itl_ms"],
                              "direct_ttft_p99_ms": d_sse["p99_ttft_ms"], "direct_bulk_MBps": d_bulk["MBps"]}),
                  file=sys.stderr, flush=True)
            for tr in trs:
                t = tunnels[tr]
                path = t.serve.wait_for("WebRTC connection established", 5).split(" via ", 1)[-1]
                base = rss_kb(t.proxy.popen.pid)
                c0 = cpu_stat()
                sse_r, bulk_r, stats, peak = scenario(t.proxy_port, a, t.proxy.popen.pid)
                t_cg = stat_delta(c0, cpu_stat())
                run = {"rep": rep, "transport": tr, "path": path,
                       "tunneled_itl_p50_ms": sse_r["p50_itl_ms"], "tunneled_itl_p99_ms": sse_r["p99_itl_ms"],
                       "tunneled_itl_max_ms": sse_r["max_itl_ms"], "direct_itl_p50_ms": d_sse["p50_itl_ms"],
                       "direct_itl_p99_ms": d_sse["p99_itl_ms"], "direct_itl_max_ms": d_sse["max_itl_ms"],
                       "added_itl_p99_ms": sse_r["p99_itl_ms"] - d_sse["p99_itl_ms"],
                       "tunneled_ttft_p50_ms": sse_r["p50_ttft_ms"], "direct_ttft_p50_ms": d_sse["p50_ttft_ms"],
                       "tunneled_ttft_p99_ms": sse_r["p99_ttft_ms"], "direct_ttft_p99_ms": d_sse["p99_ttft_ms"],
                       "added_ttft_p99_ms": sse_r["p99_ttft_ms"] - d_sse["p99_ttft_ms"],
                       "sse_requests": sse_r["requests"], "sse_events": sse_r["events"], "sse_errors": sse_r["errors"],
                       "bulk_MBps": bulk_r["MBps"], "direct_bulk_MBps": d_bulk["MBps"],
                       "bulk_ratio": bulk_r["MBps"] / d_bulk["MBps"] if d_bulk["MBps"] else None,
                       "bulk_errors": bulk_r["errors"], "slow_client_bytes": stats.get("slow_bytes"),
                       "proxy_rss_base_mib": round(base / 1024, 1), "proxy_rss_peak_mib": round(peak / 1024, 1),
                       # the job's CPU quota over the run (cgroup v2): a throttled period stops every thread
                       "cgroup_tunneled": t_cg, "cgroup_direct": d_cg}
                res["runs"].append(run)
                print(json.dumps(run), file=sys.stderr, flush=True)
        keys = ["added_itl_p99_ms", "tunneled_itl_p99_ms", "direct_itl_p99_ms", "added_ttft_p99_ms",
                "tunneled_ttft_p99_ms", "direct_ttft_p99_ms", "tunneled_ttft_p50_ms", "bulk_MBps", "direct_bulk_MBps",
                "bulk_ratio", "proxy_rss_peak_mib"]
        for tr in trs:
            runs = [r for r in res["runs"] if r["transport"] == tr]
            row = {"transport": tr, "path": runs[0]["path"] if runs else "", "reps": len(runs),
                   "sse_errors": sum(r["sse_errors"] for r in runs), "bulk_errors": sum(r["bulk_errors"] for r in runs)}
            for k in keys:
                row[k] = summary([r[k] for r in runs])
            res["rows"].append(row)
    finally:
        pids = {f"{tr}.{role}": getattr(t, role).popen.pid for tr, t in tunnels.items() for role in ("serve", "proxy")}
        for t in tunnels.values():
            t.__exit__(None, None, None)
        mock.stop()
    if tl_dir:  # over each process's life; the direct runs add idle intervals only
        res["timeline"] = timeline.summarise(tl_dir, pids)
    if a.profile_dir:
        res["profiles"] = {k: f"tunnel.{v}.prof" for k, v in pids.items()}
        for k, v in pids.items():
            f = os.path.join(a.profile_dir, f"tunnel.{v}.prof")
            if os.path.exists(f):
                for thread, suffix in ((None, ""), ("0", ".main")):
                    rep = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "profile_report.py"), f, "--top", "30"] +
                                         (["--thread", thread] if thread else []), capture_output=True, text=True).stdout
                    with open(os.path.join(a.profile_dir, f"{k}{suffix}.txt"), "w") as fh:
                        fh.write(rep)
    res["box"] = _box()
    doc = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(doc + "\n")
    print(doc)


if __name__ == "__main__":
    main()
