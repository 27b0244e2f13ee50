"""Where the tunnel's added time-to-first-token goes, hop by hop.

    python scripts/ttft_breakdown.py [--requests 40] [--transport webrtc|tcp]

Runs the native mock behind a tunnel with TUNNEL_TRACE (serve + proxy) and
MOCK_TRACE on, sends sequential streamed requests with the native load
generator, joins the per-stream events (all processes stamp CLOCK_MONOTONIC
µs on one host) and prints the median and p90 of each hop:

  proxy accept -> proxy req_end           proxy parses the request, queues the frames
  proxy req_end -> serve req_headers      the request crosses the tunnel
  serve req_headers -> req_end            serve receives the rest of the request
  serve req_end -> upstream_sent          serve picks an upstream socket and writes
  upstream_sent -> mock_req               upstream wakes up and parses
  mock_req -> serve first_body            first event back at serve
  serve first_body -> proxy first_body    response crosses the tunnel, split into
    serve first_body -> serve sched_in      upstream reader -> serve association thread
    serve sched_in -> serve chan_tx         frame scheduler (queued behind the channel window?)
    serve chan_tx -> proxy chan_rx          SCTP, DTLS, UDP, socket reader, proxy association thread:
      serve chan_tx -> serve udp_tx           SCTP + DTLS seal + sendmmsg returned
      serve udp_tx -> proxy udp_kernel        loopback delivery (kernel receive timestamp; may be < 0:
                                              the kernel stamps before the sender's syscall returns)
      proxy udp_kernel -> proxy udp_read      the receiving thread's wake-up and recvmmsg
      proxy udp_read -> proxy rx_assoc        socket reader -> association thread (0 when it reads itself)
      proxy rx_assoc -> proxy chan_rx         DTLS open + SCTP + frame dispatch
    proxy chan_rx -> proxy first_body       hand-off to the client connection, its write
  the request crossing, split the same way: proxy req_end -> udp_tx -> serve
    udp_kernel -> udp_read -> rx_assoc -> req_headers
  client TTFT (the load generator's p50) minus proxy accept -> first_body: the
    client's own hops (its write to the proxy's wake-up, the proxy's write to
    its wake-up)

Tracing is buffered in memory and written at exit,
so stamping costs no syscall on the measured path.

--bulk-echo: BASELINE config #3 (N streams x 1 MB POST echoed) as a waterfall.
Every request is stamped at each hop (TUNNEL_TRACE, buffered), and the steps
of the load generator (all N requests in flight, the step ends with its
slowest) are laid out against the direct run of the same load:

  per request   proxy accept -> body_first -> req_end (client upload into the proxy)
                proxy req_end -> chan_end (REQ_END waits in the proxy's scheduler)
                proxy chan_end -> serve req_end (the upload's tail crosses)
                serve req_end -> upstream_sent (buffered body written to the upstream)
                serve upstream_sent -> res_headers -> res_end (upstream echo)
                serve res_end -> chan_end -> proxy res_end (the download's tail crosses)
  per step      when the last upload reached serve, the last upstream send,
                the first / last echo finished at serve, the last response at
                the proxy (ms from the step's first accept)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=40)
    ap.add_argument("--transport", default="webrtc")
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--bulk", type=int, default=0, help="concurrent 64 MB GET /bulk downloads running through the "
                    "same tunnel for the whole measurement (the mixed row's head-of-line load)")
    ap.add_argument("--extra", default="", help="extra flags for both tunnel processes, e.g. --no-jumbo-loopback")
    ap.add_argument("--bulk-echo", action="store_true", help="N x 1 MB POST echo waterfall (BASELINE config #3)")
    ap.add_argument("--mb", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40, help="--bulk-echo: timed steps")
    ap.add_argument("--pin", action="store_true", help="pin loadgen / mock / serve / proxy to disjoint CPUs")
    ap.add_argument("--mock-threads", type=int, default=1, help="--bulk-echo: reactor threads of the echo upstream")
    a = ap.parse_args()
    ensure_native()
    if a.bulk_echo:
        return bulk_echo(a)
    with tempfile.NamedTemporaryFile(suffix=".jsonl", prefix="p2pt-trace-", delete=False) as tf:
        trace = tf.name
    port = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(port), "--interval-ms", "20"], env={"MOCK_TRACE": "1"})
    mock.wait_for("Mock LLM server running", 10)
    try:
        extra = [x for x in a.extra.split() if x]
        with Tunnel(f"http://127.0.0.1:{port}", transport=a.transport,
                    env={"TUNNEL_TRACE": trace},
                    serve_extra=extra, proxy_extra=extra) as t:
            bulk = None
            if a.bulk:
                bulk = subprocess.Popen([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{t.proxy_port}", "--streams",
                                         str(a.bulk), "--steps", str(1 << 20), "--warmup", "0", "--method", "GET",
                                         "--path", f"/bulk?bytes={64 << 20}", "--events", "none", "--duration-s", "600"],
                                        stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                time.sleep(0.5)
            lg = subprocess.run([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{t.proxy_port}", "--streams",
                                 str(a.streams), "--steps", str(a.requests // a.streams), "--warmup", "1"],
                                check=True, capture_output=True, text=True)
            client = json.loads(lg.stdout.strip().splitlines()[-1])
            if bulk:
                bulk.kill()
                bulk.wait()
        ev = {}
        with open(trace) as f:
            for line in f:
                e = json.loads(line)
                ev.setdefault(e["sid"], {})[(e["role"], e["ev"])] = e["t_us"]
        # SSE requests are POSTs; the --bulk downloads are GETs (left out on both sides).
        mock_t = sorted(int(l.split()[1]) for l in mock.lines if l.startswith("mock_req ") and "GET" not in l.split()[2:])
    finally:
        mock.stop()
        if os.path.exists(trace):
            os.unlink(trace)
    hops = [("proxy", "tcp_accept", "proxy", "conn_adopt"), ("proxy", "conn_adopt", "proxy", "accept"),
            ("proxy", "accept", "proxy", "req_end"), ("proxy", "req_end", "serve", "req_headers"),
            ("serve", "req_headers", "serve", "req_end"), ("serve", "req_end", "serve", "upstream_sent"),
            ("serve", "upstream_sent", "mock", "req"), ("mock", "req", "serve", "first_body"),
            ("serve", "first_body", "proxy", "first_body"),
            # the token crossing split: upstream reader -> serve association thread,
            # scheduler + SCTP + DTLS + UDP + socket reader -> proxy association
            # thread, then the hand-off to the client connection and its write
            ("serve", "first_body", "serve", "sched_in"), ("serve", "sched_in", "serve", "chan_tx"),
            ("serve", "chan_tx", "proxy", "chan_rx"),
            ("serve", "chan_tx", "serve", "udp_tx"), ("serve", "udp_tx", "proxy", "udp_kernel"),
            ("serve", "chan_tx", "proxy", "udp_kernel"),
            ("proxy", "udp_kernel", "proxy", "udp_read"), ("proxy", "udp_read", "proxy", "rx_assoc"),
            ("proxy", "rx_assoc", "proxy", "chan_rx"),
            ("proxy", "chan_rx", "proxy", "first_body"),
            # the request crossing split the same way
            ("proxy", "req_end", "proxy", "udp_tx"), ("proxy", "udp_tx", "serve", "udp_kernel"),
            ("proxy", "req_end", "serve", "udp_kernel"),
            ("serve", "udp_kernel", "serve", "udp_read"), ("serve", "udp_read", "serve", "rx_assoc"),
            ("serve", "rx_assoc", "serve", "req_headers"),
            # the upstream's own turnaround (joinable per stream at serve) and
            # the whole time inside the tunnel processes
            ("serve", "upstream_sent", "serve", "first_body"),
            ("proxy", "accept", "proxy", "first_body")]
    rows = {f"{a_}.{b_} -> {c_}.{d_}": [] for a_, b_, c_, d_ in hops}
    # The mock's trace line carries no stream id, so a mock request can only be
    # paired with the upstream send that preceded it when one stream runs at a
    # time; with concurrent streams the two mock hops are left out.
    join_mock = a.streams == 1
    if not join_mock:
        hops = [h for h in hops if "mock" not in (h[0], h[2])]
        rows = {f"{a_}.{b_} -> {c_}.{d_}": [] for a_, b_, c_, d_ in hops}
    for sid, e in sorted(ev.items()):
        if ("serve", "upstream_sent") not in e or ("proxy", "first_body") not in e or ("proxy", "get") in e:
            continue
        if sid <= a.streams:  # the load generator's warm-up step (cold pools, first connections)
            continue
        if join_mock:
            up = e[("serve", "upstream_sent")]
            m = next((x for x in mock_t if x >= up), None)  # the mock request that followed this send
            if m is None:
                continue
            e[("mock", "req")] = m
        for a_, b_, c_, d_ in hops:
            if (a_, b_) in e and (c_, d_) in e:
                rows[f"{a_}.{b_} -> {c_}.{d_}"].append(e[(c_, d_)] - e[(a_, b_)])
    out = {}
    for k, v in rows.items():
        if v:
            v.sort()
            out[k] = {"n": len(v), "p50_us": statistics.median(v), "p90_us": v[int(0.9 * (len(v) - 1))],
                      "p99_us": v[int(0.99 * (len(v) - 1))], "max_us": v[-1]}
    # The slowest requests inside the tunnel (proxy accept -> proxy first_body):
    # every hop of each, so a tail is pinned on the hop that made it.
    tot = ("proxy", "accept"), ("proxy", "first_body")
    done = [(sid, e) for sid, e in ev.items() if tot[0] in e and tot[1] in e and ("proxy", "get") not in e
            and sid > a.streams]
    done.sort(key=lambda x: x[1][tot[1]] - x[1][tot[0]])
    worst = []
    for sid, e in done[-max(3, len(done) // 50):]:
        w = {"sid": sid, "total_us": e[tot[1]] - e[tot[0]]}
        for a_, b_, c_, d_ in hops:
            if (a_, b_) in e and (c_, d_) in e:
                w[f"{a_}.{b_} -> {c_}.{d_}"] = e[(c_, d_)] - e[(a_, b_)]
        worst.append(w)
    res = {"transport": a.transport, "streams": a.streams, "bulk": a.bulk, "extra": a.extra,
           "env": {k: v for k, v in os.environ.items() if k.startswith("TUNNEL_")}, "hops": out,
           "client_p50_ttft_us": client.get("p50_ttft_ms", 0) * 1000, "client_p99_ttft_us": client.get("p99_ttft_ms", 0) * 1000,
           "worst": worst}
    inside = out.get("proxy.accept -> proxy.first_body")
    if inside:
        res["client_hops_p50_us"] = res["client_p50_ttft_us"] - inside["p50_us"]
    if not join_mock:
        res["note"] = "mock hops omitted: mock trace lines cannot be joined to streams when streams > 1"
    print(json.dumps(res, indent=1))


def _pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))] if v else None


def bulk_echo(a):
    from p2p_llm_tunnel_amd.utils import netstat
    from p2p_llm_tunnel_amd.utils.pinning import cpu_plan
    streams = a.streams if a.streams > 1 else 64
    plan = cpu_plan() if a.pin else {}
    with tempfile.NamedTemporaryFile(suffix=".jsonl", prefix="p2pt-trace-", delete=False) as tf:
        trace = tf.name
    port = free_port()
    mock = spawn("mock", (["taskset", "-c", plan["mock"]] if plan else []) + [binary("tunnel-mock"), "--port", str(port),
                                                                               "--threads", str(a.mock_threads)])
    mock.wait_for("Mock LLM server running", 10)

    def run(target, trace_file=None):
        cmd = [binary("tunnel-loadgen"), "--target", f"127.0.0.1:{target}", "--streams", str(streams), "--steps",
               str(a.steps), "--warmup", "2", "--post-bytes", str(a.mb << 20)]
        if plan:
            cmd = ["taskset", "-c", plan["loadgen"]] + cmd
        env = dict(os.environ, LOADGEN_TRACE=trace_file) if trace_file else None
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        return json.loads(r.stdout.strip().splitlines()[-1])
    try:
        extra = [x for x in a.extra.split() if x]
        pin_s = ["--cpu-affinity", plan["serve"]] if plan else []
        pin_p = ["--cpu-affinity", plan["proxy"]] if plan else []
        ms, mp = free_port(), free_port()
        with Tunnel(f"http://127.0.0.1:{port}", transport=a.transport,
                    env={"TUNNEL_TRACE": trace},
                    serve_extra=extra + pin_s + ["--metrics-listen", f"127.0.0.1:{ms}"],
                    proxy_extra=extra + pin_p + ["--metrics-listen", f"127.0.0.1:{mp}"]) as t:
            path = t.serve.wait_for("WebRTC connection established", 1).split(" via ", 1)[-1] if a.transport == "webrtc" else ""
            n0 = netstat.snapshot()
            tr = run(t.proxy_port, trace)
            n1 = netstat.snapshot()
            # Recovery events during the run (a timer-driven retransmission
            # stalls a step by its timeout): both sides summed.
            import urllib.request
            counters = {}
            for p_ in (ms, mp):
                txt = urllib.request.urlopen(f"http://127.0.0.1:{p_}/metrics", timeout=5).read().decode()
                for l in txt.splitlines():
                    if l.startswith(("tunnel_sctp_", "tunnel_udp_rx_overflow", "tunnel_udp_send_drops", "tunnel_dtls_lane_send",
                                     "tunnel_dtls_rx_dropped")):
                        k, v = l.split()[0], float(l.split()[1])
                        if any(x in k for x in ("retransmits", "t3_", "tlp_", "rack_marks", "overflow", "drops", "undos", "late_tsns",
                                                    "dup_tsns", "rx_dropped")):
                            counters[k] = counters.get(k, 0.0) + v
        n2 = netstat.snapshot()
        dr = run(port)
        n3 = netstat.snapshot()
        ev, lg = {}, {}
        with open(trace) as f:
            for line in f:
                try:
                    e = json.loads(line)
                except ValueError:  # a torn line (should not happen: whole-line appends)
                    continue
                if e["role"] == "loadgen":  # the client's step boundaries
                    lg.setdefault(e["sid"], {})[e["ev"]] = e["t_us"]
                    continue
                ev.setdefault(e["sid"], {})[(e["role"], e["ev"])] = e["t_us"]
    finally:
        mock.stop()
        if os.path.exists(trace):
            os.unlink(trace)
    hops = [("proxy", "accept", "proxy", "body_first"), ("proxy", "body_first", "proxy", "req_end"),
            ("proxy", "body_first", "proxy", "chan_tx"), ("proxy", "req_end", "proxy", "chan_end"),
            ("proxy", "chan_end", "serve", "req_end"), ("serve", "req_headers", "serve", "req_end"),
            ("serve", "req_end", "serve", "upstream_sent"), ("serve", "upstream_sent", "serve", "res_headers"),
            ("serve", "res_headers", "serve", "res_end"), ("serve", "res_end", "serve", "chan_end"),
            ("serve", "chan_end", "proxy", "res_end"), ("proxy", "accept", "proxy", "res_end")]
    reqs = [e for sid, e in sorted(ev.items()) if ("proxy", "accept") in e and ("proxy", "res_end") in e]
    per_hop = {}
    for a_, b_, c_, d_ in hops:
        v = [e[(c_, d_)] - e[(a_, b_)] for e in reqs if (a_, b_) in e and (c_, d_) in e]
        if v:
            per_hop[f"{a_}.{b_} -> {c_}.{d_}"] = {"n": len(v), "p10_ms": _pct(v, .1) / 1e3,
                                                  "p50_ms": _pct(v, .5) / 1e3, "p90_ms": _pct(v, .9) / 1e3}
    # Steps: the load generator releases `streams` requests at once; consecutive
    # groups of that many accepts (the 2 warm-up steps included, then dropped).
    reqs.sort(key=lambda e: e[("proxy", "accept")])
    marks = {"last upload at proxy (req_end)": ("proxy", "req_end", max),
             "last REQ_END into the channel": ("proxy", "chan_end", max),
             "first upload complete at serve": ("serve", "req_end", min),
             "last upload complete at serve": ("serve", "req_end", max),
             "last request written upstream": ("serve", "upstream_sent", max),
             "first echo complete at serve": ("serve", "res_end", min),
             "last echo complete at serve": ("serve", "res_end", max),
             "last response complete at proxy": ("proxy", "res_end", max)}
    steps = []
    if lg:  # the client's own steps: marks from its step start
        bounds = sorted((v["step_start"], v["step_end"], v.get("connected")) for v in lg.values()
                        if "step_start" in v and "step_end" in v)
        for t0, t1, conn in bounds:
            g = [e for e in reqs if t0 <= e[("proxy", "accept")] <= t1]
            if not g:
                continue
            acc = [e[("proxy", "accept")] for e in g]
            row = {"first request parsed at proxy": (min(acc) - t0) / 1e3, "last request parsed at proxy": (max(acc) - t0) / 1e3}
            for name, (role, evn, agg) in marks.items():
                vals = [e[(role, evn)] for e in g if (role, evn) in e]
                row[name] = (agg(vals) - t0) / 1e3 if vals else None
            row["step end at the client"] = (t1 - t0) / 1e3
            row["new connections"] = sum(1 for e in g if ("proxy", "tcp_accept") in e)
            # the client's last connect() of this step completing (new connections only)
            row["last client connect done"] = (conn - t0) / 1e3 if conn and conn >= t0 else None
            # The straggler: the request whose upload ended last, every stamp
            # it has relative to the step start (ms).
            late = max(g, key=lambda e: e.get(("proxy", "req_end"), 0))
            row["straggler"] = {f"{r_}.{n_}": round((v - t0) / 1e3, 3) for (r_, n_), v in sorted(late.items(), key=lambda x: x[1])}
            steps.append(row)
    else:
        for i in range(0, len(reqs) - streams + 1, streams):
            g = reqs[i:i + streams]
            t0 = min(e[("proxy", "accept")] for e in g)
            row = {"accept_spread_ms": (max(e[("proxy", "accept")] for e in g) - t0) / 1e3}
            for name, (role, evn, agg) in marks.items():
                vals = [e[(role, evn)] for e in g if (role, evn) in e]
                row[name] = (agg(vals) - t0) / 1e3 if vals else None
            steps.append(row)
    steps = steps[2:] if len(steps) > 4 else steps
    waterfall = {k: statistics.median([s[k] for s in steps if s.get(k) is not None]) for k in steps[0]
                 if k != "straggler"} if steps else {}
    slowest = sorted(steps, key=lambda s: s.get("step end at the client") or 0)[-3:]

    def step_stats(r):
        v = r["step_ms"]
        return {"req_s": r["req_s"], "step_ms_p50": statistics.median(v), "step_ms_mean": statistics.fmean(v),
                "step_ms_p90": _pct(v, .9), "step_ms_max": max(v), "errors": r["errors"]}
    res = {"mode": "bulk-echo", "transport": a.transport, "extra": a.extra, "path": path, "pinned": plan,
           "streams": streams, "mb": a.mb, "steps": a.steps,
           "tunneled": step_stats(tr), "direct": step_stats(dr),
           "ratio": tr["req_s"] / dr["req_s"] if dr["req_s"] else None,
           "step_waterfall_ms_median": waterfall, "slowest_steps": slowest, "recovery": counters,
           "kernel_tunneled": netstat.delta(n0, n1, True), "kernel_direct": netstat.delta(n2, n3, True),
           "tunneled_step_ms": tr["step_ms"], "direct_step_ms": dr["step_ms"], "per_request": per_hop}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
