#!/usr/bin/env python3
"""Two tunnels sharing one bottleneck: is the SCTP congestion response fair?

Both tunnels' serve sides reach their proxies through ONE TURN server whose
relay towards peers is an emulated link (rate, drop-tail queue of one BDP,
one-way delay, Bernoulli loss): the native ``tunnel-relay``
(native/bin/relay_main.cc, default) or, with ``--relay python``, the Python
one of utils/turn_server.py (``Link``; it tops out near 17 MB/s), so the two
associations' downloads compete for the same queue — unlike the per-agent WAN
emulator (native/rtc/ice.cc), which gives every association a link of its own.

Each tunnel runs one download loop (GET /bulk from the native mock, repeated
for --seconds) and the two start together. Reported per row: each flow's
MB/s, its share, Jain's fairness index (x1 + x2)^2 / (2 (x1^2 + x2^2)), the
link's utilisation and drops.

Competitors (--pairs): ``default:default`` (two tunnels with the shipped
loss response) and ``default:reno`` (the second serve with
TUNNEL_SCTP_CC=reno: every loss cuts cwnd
by half, no delay response — a Reno-like competitor); a single policy (e.g.
``reno``) runs one flow alone, the reference for how much a competitor harms
it. ``keep`` is round 3's default (random losses keep cwnd:
TUNNEL_SCTP_CC=beta=100).

    python bench/bench_fairness.py --rates 50,200 --rtt-ms 20 --losses 0,0.005 --seconds 20
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.build import ensure_native  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port, spawn  # noqa: E402
from p2p_llm_tunnel_amd.utils.turn_server import Link, TurnServer  # noqa: E402

POLICIES = {
    "default": {},
    "reno": {"TUNNEL_SCTP_CC": "reno"},
    "keep": {"TUNNEL_SCTP_CC": "beta=100"},
}


def jain(xs):
    s, q = sum(xs), sum(x * x for x in xs)
    return s * s / (len(xs) * q) if q else 0.0


class NativeRelay:
    """tunnel-relay as a subprocess with the TurnServer surface run_row uses."""

    def __init__(self, rate, delay_ms, queue_kb, loss):
        self.proc = spawn("relay", [binary("tunnel-relay"), "--rate-mbps", str(rate), "--delay-ms", str(delay_ms),
                                    "--queue-kb", str(queue_kb), "--loss", str(loss)])
        line = self.proc.wait_for(r"relay listening on turn:", 10)
        self.url = line.split("relay listening on ", 1)[1].split()[0]
        self.stats = {}

    def stop(self):
        self.proc.stop()
        for line in reversed(self.proc.lines):
            if line.startswith("{"):
                self.stats = json.loads(line)
                break


def run_row(rate, rtt_ms, loss, pair, seconds, mb, mtu_extra, relay="native", queue_kb=0):
    queue_kb = queue_kb or max(32, int(rate * 1e6 / 8 * rtt_ms / 1e3 / 1024))
    link = None
    if relay == "native":
        turn = NativeRelay(rate, rtt_ms / 2, queue_kb, loss)
    else:
        link = Link(rate_mbps=rate, delay_ms=rtt_ms / 2, queue_kb=queue_kb, loss=loss)
        turn = TurnServer(user="u", password="p", link=link).start()
    port = free_port()
    mock = spawn("mock", [binary("tunnel-mock"), "--port", str(port)])
    mock.wait_for("Mock LLM server running", 10)
    tunnels = []
    try:
        for i, pol in enumerate(pair):
            serve_extra = ["--turn", turn.url, "--turn-user", "u", "--turn-pass", "p", "--ice-relay-only"] + mtu_extra
            # "betaNN": the random-loss cut to NN % (TUNNEL_SCTP_CC=beta=NN)
            env = dict(POLICIES[pol]) if pol in POLICIES else {"TUNNEL_SCTP_CC": "beta=" + pol[4:]}
            t = Tunnel(f"http://127.0.0.1:{port}", transport="webrtc", serve_extra=serve_extra,
                       proxy_extra=list(mtu_extra), env=env,
                       room=f"fair-{os.getpid()}-{i}-{time.time_ns()}")
            tunnels.append(t.start(timeout=60))
        paths = [t.serve.wait_for("WebRTC connection established", 5).split(" via ", 1)[-1] for t in tunnels]
        procs = [subprocess.Popen([binary("tunnel-loadgen"), "--target", f"127.0.0.1:{t.proxy_port}", "--streams", "1",
                                   "--steps", str(1 << 20), "--warmup", "0", "--method", "GET", "--path",
                                   f"/bulk?bytes={mb << 20}", "--events", "none", "--duration-s", str(seconds)],
                                  stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for t in tunnels]
        outs = []
        for p in procs:
            out, _ = p.communicate(timeout=seconds + 120)
            outs.append(json.loads(out.strip().splitlines()[-1]))
    finally:
        for t in tunnels:
            t.stop()
        mock.stop()
        turn.stop()
    mbps = [o["body_bytes"] / o["seconds"] / 1e6 if o["seconds"] else 0.0 for o in outs]
    cap = rate * 1e6 / 8 / 1e6
    two = len(mbps) == 2
    return {"rate_mbps": rate, "rtt_ms": rtt_ms, "loss": loss, "pair": ":".join(pair), "paths": paths,
            "MBps": [round(x, 3) for x in mbps], "share": [round(x / sum(mbps), 3) if sum(mbps) else 0 for x in mbps],
            "jain": round(jain(mbps), 4) if two else None, "utilisation": round(sum(mbps) / cap, 3),
            "ratio_first_to_second": round(mbps[0] / mbps[1], 3) if two and mbps[1] else None,
            "errors": [o["errors"] for o in outs], "relay": relay,
            "link": link.stats if link is not None else turn.stats.get("link", {}), "queue_kb": queue_kb}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="50,200")
    ap.add_argument("--rtt-ms", type=float, default=20.0)
    ap.add_argument("--losses", default="0,0.005")
    ap.add_argument("--pairs", default="default:default,default:reno")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--mb", type=int, default=8, help="size of each download in the loop")
    ap.add_argument("--jumbo", action="store_true", help="allow the jumbo path (default: 1200-byte MTU)")
    ap.add_argument("--relay", choices=["native", "python"], default="native")
    ap.add_argument("--queue-kb", type=float, default=0, help="bottleneck queue (default: one BDP, at least 32 KiB)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ensure_native()
    mtu_extra = [] if a.jumbo else ["--no-jumbo-loopback"]
    rows = []
    for rate in [float(x) for x in a.rates.split(",")]:
        for loss in [float(x) for x in a.losses.split(",")]:
            for pair in a.pairs.split(","):
                r = run_row(rate, a.rtt_ms, loss, pair.split(":"), a.seconds, a.mb, mtu_extra, a.relay, a.queue_kb)
                rows.append(r)
                print(json.dumps(r), file=sys.stderr, flush=True)
    from p2p_llm_tunnel_amd.utils.boxinfo import identity
    res = {"bench": "fairness", "rows": rows, "box": identity()}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
