#!/usr/bin/env python3
"""Headline benchmark: tunneled req/s + added p50 TTFT vs direct, mock-LLM SSE
at 1/2/4/8 multiplexed streams (BASELINE.json "metric").

Per rank (one rank per GPU of the node, launched by torch.distributed.run for
N > 1): a mock OpenAI upstream (reference tmp/mock_llm.py workload: 5 SSE
tokens 100 ms apart; threaded so concurrency is not capped by the mock),
the local signal server, ``tunnel serve`` and ``tunnel proxy`` (native C++,
WebRTC data channel over loopback by default). A *step* is one streamed
completion on each of S concurrent keep-alive client connections (S = 8 for
the headline; the 1/2/4 points are measured too and reported in "curve").
``value`` is the whole-job aggregate tunneled requests/s over all ranks
(weak scaling: every rank runs its own tunnel with S streams).

The tunnel has no GPU compute: the measured path is
host-side networking on the MI355X node, so "dtype" is reported as n/a.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "tunneled req/s + added p50 TTFT vs direct, mock-LLM SSE at 1/2/4/8 streams"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=8, help="concurrent streams per rank for the headline")
    ap.add_argument("--curve", default="1,2,4", help="extra stream counts measured for the scaling curve")
    ap.add_argument("--curve-steps", type=int, default=3)
    ap.add_argument("--transport", default=os.environ.get("BENCH_TRANSPORT", "webrtc"))
    ap.add_argument("--interval-ms", type=float, default=100.0)
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--unthreaded-mock", action="store_true")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    return ap.parse_args()


def dist_init():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return None, 0, 1
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # Host-side workload: gloo carries the barrier / max-reduce; no GPU collectives involved.
    dist.init_process_group("gloo")
    return dist, dist.get_rank(), dist.get_world_size()


def sync_device():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def main():
    a = parse()
    dist, rank, world = dist_init()
    from p2p_llm_tunnel_amd.parallel.loadgen import run_steps, summarize
    from p2p_llm_tunnel_amd.utils import mock_llm
    from p2p_llm_tunnel_amd.utils.build import ensure_native
    from p2p_llm_tunnel_amd.utils.procs import Tunnel

    if rank == 0:
        ensure_native()
    if dist:
        dist.barrier()

    srv, up_port = mock_llm.start_in_thread(threaded=not a.unthreaded_mock, tokens=a.tokens,
                                            interval_ms=a.interval_ms)
    tun = Tunnel(f"http://127.0.0.1:{up_port}", transport=a.transport,
                 env={"RUST_LOG": "warn,tunnel::serve=info,tunnel::proxy=info,tunnel::transport=info"})
    tun.start(timeout=60)
    loop = asyncio.new_event_loop()

    def run(port, streams, steps):
        return loop.run_until_complete(run_steps("127.0.0.1", port, streams, steps))

    def barrier():
        if dist:
            dist.barrier()

    # Warmup (untimed): connections, SCTP cwnd, pools.
    if a.warmup:
        run(tun.proxy_port, a.streams, a.warmup)

    # ---- headline: timed K steps at S streams
    barrier()
    sync_device()
    t0 = time.perf_counter()
    dt_local, stats = run(tun.proxy_port, a.streams, a.steps)
    barrier()
    sync_device()
    dt_wall = time.perf_counter() - t0
    head = summarize(stats)

    # ---- untimed extras: curve points and the direct (untunneled) baseline
    curve = {}
    for s in sorted({int(x) for x in a.curve.split(",") if x} | {a.streams}):
        if s == a.streams:
            tun_sum, tun_dt = head, dt_local
        else:
            tun_dt, st_ = run(tun.proxy_port, s, a.curve_steps)
            tun_sum = summarize(st_)
        d_dt, d_st = run(up_port, s, a.curve_steps)
        d_sum = summarize(d_st)
        curve[str(s)] = {
            "tunneled_req_s": tun_sum["requests"] / tun_dt if s != a.streams else head["requests"] / dt_local,
            "direct_req_s": d_sum["requests"] / d_dt,
            "tunneled_p50_ttft_ms": tun_sum["p50_ttft_ms"],
            "direct_p50_ttft_ms": d_sum["p50_ttft_ms"],
            "added_p50_ttft_ms": tun_sum["p50_ttft_ms"] - d_sum["p50_ttft_ms"],
            "tunneled_p99_ttft_ms": tun_sum["p99_ttft_ms"],
            "errors": tun_sum["errors"],
        }

    tun.stop()
    srv.shutdown()

    requests = head["requests"]
    errors = head["errors"]
    dt = dt_wall
    if dist:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        r = torch.tensor([requests, errors], dtype=torch.float64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        requests, errors = int(r[0].item()), int(r[1].item())
        added = torch.tensor([curve[str(a.streams)]["added_p50_ttft_ms"]], dtype=torch.float64)
        dist.all_reduce(added, op=dist.ReduceOp.MAX)
        added_max = float(added.item())
    else:
        added_max = curve[str(a.streams)]["added_p50_ttft_ms"]

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": requests / dt,
            "unit": "req/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "n/a",
            "data": "synthetic: mock-LLM SSE upstream (5 tokens, %g ms apart, %s), no network/datasets" % (
                a.interval_ms, "unthreaded" if a.unthreaded_mock else "threaded"),
            "config": {
                "model": "mock-llm-sse (reference tmp/mock_llm.py workload)",
                "global_batch": a.streams * world,
                "seq_len": len(mock_llm.TOKENS) if a.tokens is None else a.tokens,
                "parallelism": f"{world} tunnel(s) x {a.streams} multiplexed streams",
                "transport": a.transport,
            },
            "added_p50_ttft_ms": added_max,
            "p50_ttft_ms": head["p50_ttft_ms"],
            "p99_ttft_ms": head["p99_ttft_ms"],
            "errors": errors,
            "curve_rank0": curve,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
