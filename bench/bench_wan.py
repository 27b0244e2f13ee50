#!/usr/bin/env python3
"""The tunnel over an emulated WAN path at the standard 1200-byte SCTP MTU.

Both peers' datagrams go through the ICE agent's WAN shim (native/rtc/ice.cc):
a bottleneck link of --rate-mbps with a drop-tail queue, a fixed round-trip
time and Bernoulli loss (TUNNEL_FAULT rtt_ms / rate_mbps / loss). For each
(RTT, loss) it measures

  * SSE alone: 8 streams, a token every 10 ms — inter-token latency (ITL);
  * SSE + bulk: the same 8 SSE streams while 4 downloads (--bulk-mb) share the
    path — a lost bulk packet holds back every later message on the single
    ordered SCTP stream (the reference's layout, rtc.rs:133), so the SSE ITL
    tail measures that cross-stream head-of-line stall;
  * bulk alone: 8 concurrent 1 MB echoes (req/s, MB/s each way).

    python bench/bench_wan.py [--rtts 20,50] [--losses 0,0.005,0.02]

--relay puts the path in the native TURN relay instead (bin/relay_main.cc:
serve relays through it, --ice-relay-only; the relay's forward link has the
rate, a one-BDP drop-tail queue, RTT/2 of delay each way and the loss), the
shared-bottleneck emulator of bench/bench_fairness.py. --policy keep runs the
serve side with TUNNEL_SCTP_CC=beta=100 (random losses keep cwnd).

--steady-mb N adds steady-state rows (run alone with --rtts ''): 4 downloads of
N MB each at every (rate, RTT, loss, queue) of --steady-*, reporting goodput
as a share of the bottleneck and the sending process's per-thread CPU.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402


def lg(port, *args):
    return subprocess.Popen([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{port}", *map(str, args)],
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)


PHASE = ["start"]  # what the run is doing (the heartbeat prints it)


def heartbeat(period_s=30.0):
    """A line on stderr every period_s: a slow lossy row is never silent, and a
    stuck one says where it is."""
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(period_s)
            print(json.dumps({"heartbeat_s": round(time.time() - t0), "phase": PHASE[0]}), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


TUNNEL = [None]  # the tunnel of the current row (its logs are printed if a load stalls)
LOGDIR = [None]  # --logs: where a stalled row's full logs go


def result(p, timeout=180):
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        t = TUNNEL[0]
        if t is not None:
            for proc in (t.serve, t.proxy):
                lines = proc.text().splitlines()
                print(f"---- {proc.name} log tail ({len(lines)} lines)", file=sys.stderr)
                print("\n".join(lines[-80:]), file=sys.stderr, flush=True)
                if LOGDIR[0]:
                    os.makedirs(LOGDIR[0], exist_ok=True)
                    with open(os.path.join(LOGDIR[0], f"stalled_{proc.name}.log"), "w") as f:
                        f.write(proc.text() + "\n")
        p.kill()
        raise
    return json.loads(out.strip().splitlines()[-1])


SCTP_GAUGES = ("tunnel_sctp_fast_retransmits", "tunnel_sctp_t3_expirations", "tunnel_sctp_tlp_probes",
               "tunnel_sctp_rack_marks", "tunnel_sctp_random_loss_events", "tunnel_sctp_cwnd_bytes",
               "tunnel_sctp_rto_us", "tunnel_sctp_packets_sent", "tunnel_sctp_dup_copies",
               "tunnel_sctp_hystart_exits", "tunnel_sctp_random_loss_cuts", "tunnel_sctp_congestion_cuts",
               "tunnel_sctp_over_bdp_losses")


def scrape(port):
    """The SCTP loss-recovery gauges of one tunnel process (--metrics-listen)."""
    try:
        text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    except OSError:
        return {}
    out = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[0] in SCTP_GAUGES:
            out[parts[0].replace("tunnel_sctp_", "")] = float(parts[1])
    return out


def scrape_all(port):
    """Every SCTP / UDP / DTLS gauge of one tunnel process (for --timeline)."""
    try:
        text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2).read().decode()
    except OSError:
        return {}
    out = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[0].startswith(("tunnel_sctp_", "tunnel_udp_", "tunnel_dtls_")):
            out[parts[0][len("tunnel_"):]] = float(parts[1])
    return out


class Timeline:
    """Samples both tunnel processes' gauges every period_s while a phase
    runs: a stalled transfer shows which counter stopped moving."""

    def __init__(self, ports, period_s=0.5):
        import threading
        self.ports, self.period, self.rows, self.stop_ev = ports, period_s, [], threading.Event()
        self.t0 = time.time()
        self.th = threading.Thread(target=self.run, daemon=True)
        self.th.start()

    def run(self):
        prev = {}
        while not self.stop_ev.wait(self.period):
            row = {"t": round(time.time() - self.t0, 2)}
            for side, port in self.ports.items():
                cur = scrape_all(port)
                # counters as deltas since the last sample, gauges as is
                row[side] = {k: (v - prev.get((side, k), 0.0)) if not k.endswith(("_bytes", "_us")) else v
                             for k, v in cur.items() if v != prev.get((side, k))}
                for k, v in cur.items():
                    prev[(side, k)] = v
            self.rows.append(row)
            print(json.dumps({"timeline": row}), file=sys.stderr, flush=True)

    def stop(self):
        self.stop_ev.set()
        self.th.join(5)
        return self.rows


def thread_cpu(pid):
    """CPU seconds per thread of a process, keyed "name/tid"."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    try:
        for tid in os.listdir(f"/proc/{pid}/task"):
            try:
                st = open(f"/proc/{pid}/task/{tid}/stat").read()
            except OSError:
                continue
            name = st[st.index("(") + 1:st.rindex(")")]
            f = st.rsplit(")", 1)[1].split()
            out[f"{name}/{tid}"] = (int(f[11]) + int(f[12])) / tck
    except OSError:
        pass
    return out


def steady_row(mport, rtt, loss, rate, qkb, mb, streams, extra):
    """Steady-state goodput: `streams` downloads of `mb` MB each over the
    emulated path, alone; MB/s against the bottleneck rate, and the CPU share
    of every thread of the sending side (serve) over the transfer."""
    env = {"TUNNEL_FAULT": f"rtt_ms={rtt},rate_mbps={rate},queue_kb={qkb},loss={loss}",
           "RUST_LOG": "warn,tunnel::rtc=info,tunnel::serve=info,tunnel::proxy=info"}
    sm, pm = free_port(), free_port()
    with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc",
                serve_extra=extra + ["--metrics-listen", f"127.0.0.1:{sm}"],
                proxy_extra=extra + ["--metrics-listen", f"127.0.0.1:{pm}"], env=env) as t:
        result(sse(t.proxy_port, 1))  # warm: connections
        pid, ppid = t.serve.popen.pid, t.proxy.popen.pid
        c0, p0, t0 = thread_cpu(pid), thread_cpu(ppid), time.time()
        r = result(lg(t.proxy_port, "--streams", streams, "--steps", 1, "--warmup", 0, "--method", "GET",
                      "--path", f"/bulk?bytes={mb << 20}", "--events", "none"), timeout=900)  # lossy 1 Gbit/s rows move GBs
        wall = time.time() - t0
        c1, p1 = thread_cpu(pid), thread_cpu(ppid)
        cpu = {k: round(100 * (c1[k] - c0.get(k, 0.0)) / wall, 1) for k in c1 if c1[k] - c0.get(k, 0.0) > 0}
        pcpu = {k: round(100 * (p1[k] - p0.get(k, 0.0)) / wall, 1) for k in p1 if p1[k] - p0.get(k, 0.0) > 0}
        mbps = r["MBps"]
        row = {"rtt_ms": rtt, "loss": loss, "rate_mbps": rate, "queue_kb": round(qkb), "downloads": streams,
               "mb_each": mb, "MBps": mbps, "pct_of_bottleneck": round(100 * mbps * 1e6 * 8 / (rate * 1e6), 1),
               "seconds": round(wall, 2), "errors": r["errors"],
               "serve_thread_cpu_pct": dict(sorted(cpu.items(), key=lambda kv: -kv[1])),
               "proxy_thread_cpu_pct": dict(sorted(pcpu.items(), key=lambda kv: -kv[1])),
               "serve_sctp": scrape(sm), "proxy_sctp": scrape(pm)}
        return row


def sse(port, steps):
    return lg(port, "--streams", 8, "--steps", steps, "--warmup", 0, "--warm-conns", 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rtts", default="20,50")
    ap.add_argument("--losses", default="0,0.005,0.02")
    ap.add_argument("--rate-mbps", type=float, default=200)
    ap.add_argument("--queue-kb", type=float, default=0, help="bottleneck queue (0: one BDP)")
    ap.add_argument("--sse-steps", type=int, default=3)
    ap.add_argument("--bulk-mb", type=int, default=4, help="size of each of the 4 background downloads")
    ap.add_argument("--echo-steps", type=int, default=1)
    ap.add_argument("--extra", default="", help="extra flags for both tunnel processes")
    ap.add_argument("--steady-mb", type=int, default=0,
                    help="steady-state goodput rows: downloads of this many MB each (0: off)")
    ap.add_argument("--steady-seconds", type=float, default=0,
                    help="size each steady row to at least this many seconds at its bottleneck rate "
                         "(MB per download = max(--steady-mb, rate x seconds / downloads)), so slow start "
                         "is a small part of the row at high rates")
    ap.add_argument("--steady-streams", type=int, default=4)
    ap.add_argument("--steady-rates", default="200,1000", help="bottleneck Mbit/s of the steady rows")
    ap.add_argument("--steady-rtts", default="20,50")
    ap.add_argument("--steady-losses", default="0,0.005")
    ap.add_argument("--steady-queues", default="0", help="queue KB per steady row (0: one BDP), e.g. 0,16")
    ap.add_argument("--relay", action="store_true", help="rows through the native TURN relay's emulated link")
    ap.add_argument("--policy", choices=["default", "keep"], default="default",
                    help="serve's congestion response: default, or keep (TUNNEL_SCTP_CC=beta=100)")
    ap.add_argument("--timeline", action="store_true",
                    help="sample both sides' SCTP/UDP/DTLS gauges every 0.5 s during sse+bulk and echo (row['timeline'])")
    ap.add_argument("--logs", default=None, help="write each row's serve/proxy/relay logs to this directory")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    heartbeat()
    LOGDIR[0] = a.logs
    ensure_native()
    mport = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(mport), "--interval-ms", "10", "--tokens", "100",
                          "--threads", "2"])
    mock.wait_for("Mock LLM server running", 10)
    from p2p_llm_tunnel_amd.utils.boxinfo import identity
    res = {"box": identity(), "host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "mtu": 1200, "rate_mbps": a.rate_mbps, "extra": a.extra, "relay": a.relay, "policy": a.policy,
           "rows": [], "steady": []}
    policy_env = {"TUNNEL_SCTP_CC": "beta=100"} if a.policy == "keep" else {}
    extra = ["--no-jumbo-loopback"] + [x for x in a.extra.split() if x]
    try:
        if a.steady_mb:
            for rate in [float(x) for x in a.steady_rates.split(",") if x]:
                for rtt in [float(x) for x in a.steady_rtts.split(",") if x]:
                    for loss in [float(x) for x in a.steady_losses.split(",") if x]:
                        for q in [float(x) for x in a.steady_queues.split(",") if x != ""]:
                            qkb = q or max(64.0, rate * 1e6 / 8 * rtt / 1e3 / 1024)
                            mb = max(a.steady_mb, int(rate / 8 * a.steady_seconds / a.steady_streams))
                            row = steady_row(mport, rtt, loss, rate, qkb, mb, a.steady_streams, extra)
                            res["steady"].append(row)
                            print(json.dumps(row), file=sys.stderr, flush=True)
        for rtt in [float(x) for x in a.rtts.split(",") if x]:
            for loss in [float(x) for x in a.losses.split(",") if x]:
                qkb = a.queue_kb or max(64.0, a.rate_mbps * 1e6 / 8 * rtt / 1e3 / 1024)
                env = {"RUST_LOG": "info,tunnel::sctp=debug,tunnel::ice=debug,tunnel::rtc=debug,tunnel::turn=debug"
                       if a.logs else "info", **policy_env}
                PHASE[0] = f"rtt {rtt} loss {loss}: tunnel start"
                print(json.dumps({"rtt_ms": rtt, "loss": loss, "phase": "tunnel start"}), file=sys.stderr, flush=True)
                relay, turn = None, []
                if a.relay:
                    sys.path.insert(0, os.path.join(ROOT, "bench"))
                    from bench_fairness import NativeRelay
                    relay = NativeRelay(a.rate_mbps, rtt / 2, qkb, loss)
                    turn = ["--turn", relay.url, "--turn-user", "u", "--turn-pass", "p", "--ice-relay-only"]
                else:
                    env["TUNNEL_FAULT"] = f"rtt_ms={rtt},rate_mbps={a.rate_mbps},queue_kb={qkb},loss={loss}"
                sm, pm = free_port(), free_port()
                with Tunnel(f"http://127.0.0.1:{mport}", transport="webrtc",
                            serve_extra=extra + turn + ["--metrics-listen", f"127.0.0.1:{sm}"],
                            proxy_extra=extra + ["--metrics-listen", f"127.0.0.1:{pm}"], env=env,
                            room=f"wan-{os.getpid()}-{time.time_ns()}") as t:
                    TUNNEL[0] = t
                    def progress(what):  # one line per phase: a long lossy row is not silent
                        PHASE[0] = f"rtt {rtt} loss {loss}: {what}"
                        print(json.dumps({"rtt_ms": rtt, "loss": loss, "phase": what}), file=sys.stderr, flush=True)
                    progress("warm")
                    result(sse(t.proxy_port, 1))  # warm: connections, cwnd
                    progress("sse")
                    alone = result(sse(t.proxy_port, a.sse_steps))
                    progress("sse+bulk")
                    bulk = lg(t.proxy_port, "--streams", 4, "--steps", 1, "--warmup", 0, "--method", "GET",
                              "--path", f"/bulk?bytes={a.bulk_mb << 20}", "--events", "none")
                    tl = Timeline({"serve": sm, "proxy": pm}) if a.timeline else None
                    time.sleep(0.5)
                    mixed = result(sse(t.proxy_port, a.sse_steps))
                    bulk_r = result(bulk)
                    progress("echo")
                    if tl:
                        tl.rows.append({"t": round(time.time() - tl.t0, 2), "phase": "echo"})
                    t0 = time.time()
                    echo = result(lg(t.proxy_port, "--streams", 8, "--steps", a.echo_steps, "--warmup", 0,
                                     "--post-bytes", 1 << 20))
                    timeline = tl.stop() if tl else None
                    row = {"rtt_ms": rtt, "loss": loss, "queue_kb": round(qkb),
                           "sse_itl_p50_ms": alone["p50_itl_ms"], "sse_itl_p99_ms": alone["p99_itl_ms"],
                           "sse_itl_max_ms": alone["max_itl_ms"], "sse_ttft_p50_ms": alone["p50_ttft_ms"],
                           "mixed_itl_p50_ms": mixed["p50_itl_ms"], "mixed_itl_p99_ms": mixed["p99_itl_ms"],
                           "mixed_itl_p999_ms": mixed["p999_itl_ms"], "mixed_itl_max_ms": mixed["max_itl_ms"],
                           "bulk_bg_MBps": bulk_r["MBps"], "echo_req_s": echo["req_s"],
                           "echo_MBps_each_way": echo["req_s"] * 1.048576,
                           "errors": alone["errors"] + mixed["errors"] + bulk_r["errors"] + echo["errors"],
                           "echo_wall_s": round(time.time() - t0, 2),
                           "serve_sctp": scrape(sm), "proxy_sctp": scrape(pm),
                           "path": t.serve.wait_for("WebRTC connection established", 1).split(" via ", 1)[-1]}
                    if timeline is not None:
                        row["timeline"] = timeline
                    if a.logs:
                        os.makedirs(a.logs, exist_ok=True)
                        tag = f"rtt{rtt:g}_loss{loss:g}_{len(res['rows'])}"
                        for proc in (t.serve, t.proxy):
                            with open(os.path.join(a.logs, f"{tag}_{proc.name}.log"), "w") as f:
                                f.write(proc.text() + "\n")
                if relay:
                    relay.stop()
                    row["relay"] = relay.stats
                    if a.logs:
                        with open(os.path.join(a.logs, f"{tag}_relay.log"), "w") as f:
                            f.write(relay.proc.text() + "\n")
                res["rows"].append(row)
                if a.out:  # the rows so far, in case a later one never ends
                    with open(a.out, "w") as f:
                        f.write(json.dumps(res, indent=1) + "\n")
                    print(json.dumps(row), file=sys.stderr, flush=True)
    finally:
        mock.stop()
    doc = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(doc + "\n")
    print(doc)


if __name__ == "__main__":
    main()
