#!/usr/bin/env python3
"""Headline benchmark: tunneled req/s + added p50 TTFT vs direct, mock-LLM SSE
at 1/2/4/8 multiplexed streams (BASELINE.json "metric").

Per rank (one rank per GPU of the node; torch.distributed.run launches N > 1):
a mock OpenAI upstream serving the reference workload (tmp/mock_llm.py: 5 SSE
tokens 100 ms apart, then a stop event and [DONE]; HTTP/1.0, no
Content-Length), the local signal server, ``tunnel serve`` and ``tunnel proxy``
(native C++; WebRTC data channel over the host's interfaces by default, on the
1200-byte SCTP path a reference webrtc-rs peer negotiates — ``--mtu jumbo``
takes this repo's same-host 16 KiB extension instead, and an untimed jumbo
point is reported beside the headline as ``jumbo_rank0``).
A *step* = one streamed completion on each of S concurrent keep-alive client
connections (S = 8 for the headline). ``value`` = whole-job tunneled
requests/s (weak scaling: S streams per GPU).

Topology for N > 1 (``--topology node``, the default): the deployment shape
of one MI355X node — every rank starts the upstream of its GPU, rank 0 runs
ONE ``tunnel serve --upstream <all N upstreams>`` and ONE proxy, and a single
load generator drives S x N streams through that tunnel; serve spreads them
over the upstreams by fewest in flight (``--workers`` auto: one reactor per 4
CPUs beside the association thread). ``--topology independent`` instead
gives every rank its own tunnel (round 1's layout).

The upstream and the client are native by default (``tunnel-mock``,
``tunnel-loadgen``) so the TTFT numbers measure the tunnel rather than
CPython; ``--mock python`` uses the Python mock instead. The untimed tail
measures the 1/2/4-stream points and the direct (untunneled) baseline that
"added TTFT" is computed against.

The tunnel has no GPU compute: the measured path is
host-side networking on the MI355X node, so "dtype" is n/a.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
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
    ap.add_argument("--curve", default="1,2,4", help="extra stream counts measured (untimed) for the curve")
    ap.add_argument("--curve-steps", type=int, default=None,
                    help="timed steps (and warm-up) of each extra curve point; default: the headline's --steps / --warmup, "
                         "so every point and its direct leg compare samples of the headline's size")
    ap.add_argument("--transport", default=os.environ.get("BENCH_TRANSPORT", "webrtc"))
    ap.add_argument("--mock", choices=["native", "python", "reference"], default="native",
                    help="native: tunnel-mock; python: utils/mock_llm.py threaded; reference: utils/mock_llm.py "
                         "single-threaded, as the reference's tmp/mock_llm.py:97 (one response at a time, ~2 req/s "
                         "at 5 x 100 ms tokens, whatever the tunnel)")
    ap.add_argument("--interval-ms", type=float, default=100.0)
    ap.add_argument("--tokens", type=int, default=5)
    ap.add_argument("--topology", choices=["node", "independent"], default="node",
                    help="N > 1: one tunnel fronting every rank's upstream (node) or one tunnel per rank")
    ap.add_argument("--mtu", choices=["std", "jumbo"], default="std",
                    help="std: the 1200-byte SCTP path a reference (webrtc-rs) peer negotiates (headline); jumbo: "
                         "this repo's same-host 16 KiB extension (a=x-p2pt-jumbo)")
    ap.add_argument("--no-jumbo-extra", action="store_true",
                    help="skip the untimed jumbo-path point reported beside a std headline")
    ap.add_argument("--pin", choices=["ccd", "l3", "numa", "none"], default=os.environ.get("P2PT_BENCH_PIN", "none"),
                    help="none (default): wherever the scheduler puts them; ccd (one GPU): load generator, mock, "
                         "serve and proxy on the cores of the idlest L3 domain (utils/pinning.py ccd_plan), the "
                         "direct leg on the same cores. On the shared pool hosts pinned runs stalled ~10 ms behind "
                         "other jobs' work on those cores in both legs (profiles/r05/b03, b04); l3: every process "
                         "on one CPU set, a hardware thread per core of the idlest L3 domain, threads placed by the "
                         "scheduler within it (pinning.l3_set_plan); numa: every process on the CPUs of the idlest "
                         "NUMA node (pinning.numa_plan)")
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


_DEVICE_SET = False


def sync_device():
    """Synchronise this rank's GPU (one rank per GPU: LOCAL_RANK's device)."""
    global _DEVICE_SET
    try:
        import torch
        if torch.cuda.is_available():
            if not _DEVICE_SET:
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
                _DEVICE_SET = True
            torch.cuda.synchronize()
    except Exception:
        pass


def start_mock(kind, interval_ms, tokens, cpus=None, threads=1):
    from p2p_llm_tunnel_amd import binary
    from p2p_llm_tunnel_amd.utils.procs import free_port, spawn
    port = free_port()
    pin = ["taskset", "-c", cpus] if cpus else []
    if kind == "native":
        p = spawn("mock", pin + [binary("tunnel-mock"), "--port", str(port), "--interval-ms", str(int(interval_ms)),
                                 "--tokens", str(tokens), "--threads", str(threads)])
    else:
        threaded = ["--threaded"] if kind == "python" else []  # "reference": single-threaded TCPServer
        p = spawn("mock", [sys.executable, "-m", "p2p_llm_tunnel_amd.utils.mock_llm", "--port", str(port)] + threaded +
                  ["--interval-ms", str(interval_ms), "--tokens", str(tokens)])
    p.wait_for("Mock LLM server running", 30)
    return p, port


PLAN: dict = {}  # role -> CPU list (--pin ccd), {} unpinned


def taskset(role):
    return ["taskset", "-c", PLAN[role]] if PLAN.get(role) else []


def loadgen(port, streams, steps, warmup=0, path=None):
    from p2p_llm_tunnel_amd import binary
    extra = ["--path", path] if path else []
    out = subprocess.run(taskset("loadgen") + [binary("tunnel-loadgen"), "--target", f"127.0.0.1:{port}", "--streams", str(streams),
                          "--steps", str(steps), "--warmup", str(warmup)] + extra, capture_output=True, text=True,
                         timeout=600)
    try:
        return json.loads(out.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError):
        raise RuntimeError(f"loadgen failed (rc={out.returncode}): {out.stdout[-500:]} {out.stderr[-500:]}")


def direct(ups, streams, steps, warmup=1):
    """The same load straight to the upstreams (no tunnel): streams split
    evenly over them, one load generator each, run concurrently; merged
    req/s and the p50/p99 TTFT of the most loaded one."""
    from p2p_llm_tunnel_amd import binary
    n = len(ups)
    share = [streams // n + (1 if i < streams % n else 0) for i in range(n)]
    procs = [subprocess.Popen(taskset("loadgen") + [binary("tunnel-loadgen"), "--target", f"127.0.0.1:{p}", "--streams", str(k),
                               "--steps", str(steps), "--warmup", str(max(1, warmup))], stdout=subprocess.PIPE,
                              text=True)
             for p, k in zip(ups, share) if k]
    res = []
    for pr in procs:
        out, _ = pr.communicate(timeout=600)
        res.append(json.loads(out.strip().splitlines()[-1]))
    return {"req_s": sum(r["req_s"] for r in res), "p50_ttft_ms": max(r["p50_ttft_ms"] for r in res),
            "p99_ttft_ms": max(r["p99_ttft_ms"] for r in res), "errors": sum(r["errors"] for r in res)}


def main():
    a = parse()
    dist, rank, world = dist_init()
    # Bring the GPU runtime up now: its first synchronise (import torch, HIP
    # init and its threads) used to land between the warm-up and the first
    # timed step, and that step's TTFT (0.82-0.91 ms against 0.26-0.39 ms for
    # the other nine on the MI355X host, profiles/r04/head_hold) set the p99.
    sync_device()
    if world > 1:  # disjoint port blocks: ranks start their tunnels concurrently
        os.environ.setdefault("P2PT_PORT_BASE", str(20000 + 500 * int(os.environ.get("LOCAL_RANK", rank))))
    from p2p_llm_tunnel_amd.utils.build import ensure_native
    from p2p_llm_tunnel_amd.utils.procs import Tunnel

    if rank == 0:
        ensure_native()
    if dist:
        dist.barrier()

    global PLAN
    if a.pin != "none" and world == 1:  # one GPU's share of the host; N > 1 ranks leave placement to the scheduler
        from p2p_llm_tunnel_amd.utils import pinning
        PLAN = {"ccd": pinning.ccd_plan, "l3": pinning.l3_set_plan, "numa": pinning.numa_plan}[a.pin]()
    mock, up_port = start_mock(a.mock, a.interval_ms, a.tokens, cpus=PLAN.get("mock"))
    node = dist is not None and a.topology == "node"
    ups = [up_port]
    if node:
        ups = [None] * world
        dist.all_gather_object(ups, up_port)
    drive = rank == 0 or not node  # ranks that run a tunnel and a load generator
    streams = a.streams * (world if node else 1)
    tun = None
    log_env = {"RUST_LOG": "warn,tunnel::serve=info,tunnel::proxy=info,tunnel::transport=info,tunnel::rtc=info"}
    if PLAN.get("set"):
        log_env["TUNNEL_PIN_THREADS"] = "0"  # the process on the set, its threads placed by the scheduler
    mtu_flags = ["--no-jumbo-loopback"] if a.mtu == "std" and a.transport == "webrtc" else []
    pin_s = ["--cpu-affinity", PLAN["serve"]] if PLAN else []
    pin_p = ["--cpu-affinity", PLAN["proxy"]] if PLAN else []
    upstreams = ",".join(f"http://127.0.0.1:{p}" for p in ups)
    if drive:
        tun = Tunnel(upstreams, transport=a.transport, env=log_env, serve_extra=mtu_flags + pin_s,
                     proxy_extra=mtu_flags + pin_p)
        tun.start(timeout=60)

    def barrier():
        if dist:
            dist.barrier()

    # Warmup (untimed) on the very keep-alive connections the timed steps then
    # use: the load generator runs its W warm-up steps, reports READY and
    # waits; the timed region brackets only its K timed steps. (Run as a
    # separate process, the warm-up left the timed steps on fresh client
    # connections, and the first timed step's TTFT — 0.76-0.82 ms against
    # 0.2-0.34 ms for the others on the MI355X host — set the p99.)
    from p2p_llm_tunnel_amd import binary
    lg = None
    if drive:
        lg = subprocess.Popen(taskset("loadgen") + [binary("tunnel-loadgen"), "--target", f"127.0.0.1:{tun.proxy_port}", "--streams",
                               str(streams), "--steps", str(a.steps), "--warmup", str(max(1, a.warmup)), "--hold", "1"],
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        ready = lg.stdout.readline()
        if ready.strip() != "READY":
            raise RuntimeError(f"loadgen did not get ready: {ready!r} {lg.stderr.read()[-500:]}")

    # ---- headline: exactly K timed steps at S streams per GPU
    barrier()
    sync_device()
    cpu0 = tun.serve.cpu_s() + tun.proxy.cpu_s() if tun else 0.0
    t0 = time.perf_counter()
    head = {"requests": 0, "errors": 0}
    if lg:
        lg.stdin.write("go\n")
        lg.stdin.flush()
        out, err = lg.communicate(timeout=600)
        try:
            head = json.loads(out.strip().splitlines()[-1])
        except (IndexError, ValueError):
            raise RuntimeError(f"loadgen failed (rc={lg.returncode}): {out[-500:]} {err[-500:]}")
    barrier()
    sync_device()
    dt_wall = time.perf_counter() - t0
    # CPU the two tunnel processes used in the timed region (every thread,
    # busy polling included): the price of the latency, reported beside it.
    tunnel_cpu_s = (tun.serve.cpu_s() + tun.proxy.cpu_s() - cpu0) if tun else 0.0
    from p2p_llm_tunnel_amd.utils.pinning import where
    placement = {"serve": where(tun.serve.popen.pid), "proxy": where(tun.proxy.popen.pid),
                 "mock": where(mock.popen.pid)} if tun else None

    # ---- untimed: curve points + direct baseline (the same load straight to
    # the upstream; node topology: S x N streams split evenly over the N upstreams)
    curve = {}
    for s in sorted({int(x) for x in a.curve.split(",") if x} | {a.streams}) if drive else []:
        n = s * (world if node else 1)
        c_steps = a.curve_steps or a.steps
        c_warm = max(1, a.warmup if a.curve_steps is None else 1)
        tun_r = head if s == a.streams else loadgen(tun.proxy_port, n, c_steps, warmup=c_warm)
        # Every direct leg runs its tunneled leg's steps and warm-up: added
        # p50 / p99 then compare samples of equal size.
        dir_r = direct(ups, n, a.steps, a.warmup) if s == a.streams else direct(ups, n, c_steps, c_warm)
        curve[str(s)] = {
            "tunneled_req_s": tun_r["req_s"],
            "direct_req_s": dir_r["req_s"],
            "tunneled_p50_ttft_ms": tun_r["p50_ttft_ms"],
            "direct_p50_ttft_ms": dir_r["p50_ttft_ms"],
            "added_p50_ttft_ms": tun_r["p50_ttft_ms"] - dir_r["p50_ttft_ms"],
            "tunneled_p99_ttft_ms": tun_r["p99_ttft_ms"],
            "direct_p99_ttft_ms": dir_r["p99_ttft_ms"],
            "errors": tun_r["errors"],
        }

    path = ""
    if drive:
        for line in tun.serve.lines:
            if "WebRTC connection established" in line:
                path = line.split(" via ", 1)[-1]
        tun.stop()
    # Untimed extra: the same headline load on the same-host jumbo path.
    jumbo = None
    if drive and a.mtu == "std" and a.transport == "webrtc" and not a.no_jumbo_extra:
        with Tunnel(upstreams, transport=a.transport, env=log_env, serve_extra=pin_s, proxy_extra=pin_p) as tj:
            loadgen(tj.proxy_port, streams, max(1, a.warmup))
            r = loadgen(tj.proxy_port, streams, a.steps)
            jp = ""
            for line in tj.serve.lines:
                if "WebRTC connection established" in line:
                    jp = line.split(" via ", 1)[-1]
        d = curve[str(a.streams)]
        jumbo = {"path": jp, "tunneled_req_s": r["req_s"], "p50_ttft_ms": r["p50_ttft_ms"],
                 "p99_ttft_ms": r["p99_ttft_ms"], "added_p50_ttft_ms": r["p50_ttft_ms"] - d["direct_p50_ttft_ms"],
                 "errors": r["errors"]}
    barrier()  # every upstream stays up until the driving rank is done
    mock.stop()

    requests = head["requests"]
    errors = head["errors"]
    dt = dt_wall
    added = curve[str(a.streams)]["added_p50_ttft_ms"] if drive else 0.0
    added_p99 = (curve[str(a.streams)]["tunneled_p99_ttft_ms"] - curve[str(a.streams)]["direct_p99_ttft_ms"]
                 if drive else 0.0)
    if dist:
        import torch
        t = torch.tensor([dt, added, added_p99], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, added, added_p99 = float(t[0].item()), float(t[1].item()), float(t[2].item())
        r = torch.tensor([requests, errors], dtype=torch.float64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        requests, errors = int(r[0].item()), int(r[1].item())

    if rank == 0:
        from p2p_llm_tunnel_amd.utils.boxinfo import identity
        box = identity()
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
            "data": f"synthetic: mock-LLM SSE upstream ({a.mock}; {a.tokens} tokens, {a.interval_ms:g} ms apart), "
                    "no network/datasets",
            "config": {
                "model": "mock-llm-sse (reference tmp/mock_llm.py workload)",
                "global_batch": a.streams * world,
                "seq_len": a.tokens,
                "parallelism": (f"1 tunnel x {world} upstreams (one per GPU) x {a.streams} streams each"
                                if node else f"{world} tunnel(s) x {a.streams} multiplexed streams"),
                "topology": "node" if node else ("independent" if world > 1 else "single"),
                "transport": a.transport,
                "mtu": a.mtu if a.transport == "webrtc" else "n/a",
                # parallel associations offered by both tunnel processes (--assoc; used on short paths)
                "assoc": int(os.environ.get("TUNNEL_ASSOC", "3")) if a.transport == "webrtc" else 1,
                "path_rank0": path,
                "pinned_rank0": {k: v for k, v in PLAN.items() if k != "set"} or None,
            },
            "added_p50_ttft_ms": added,
            "added_p99_ttft_ms": added_p99,
            "tunnel_cpu_s_rank0": round(tunnel_cpu_s, 3),
            "cpus_rank0": placement,
            "tunnel_cpu_cores_rank0": round(tunnel_cpu_s / dt_wall, 4) if dt_wall > 0 else None,
            "p50_ttft_ms": head["p50_ttft_ms"],
            "p99_ttft_ms": head["p99_ttft_ms"],
            "step_max_ttft_ms_rank0": head.get("step_max_ttft_ms"),
            "errors": errors,
            "curve_rank0": curve,
            "curve_steps": a.curve_steps or a.steps,
            "box": box,
            "jumbo_rank0": jumbo,
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
