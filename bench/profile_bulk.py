#!/usr/bin/env python3
"""64 streams x 1 MB POST echoed through a tunnel (BASELINE config #3), with
per-process CPU accounting, SCTP gauges and optional sampling profiles.

    python bench/profile_bulk.py [--transport webrtc|tcp] [--streams 64] [--steps 3]
                                 [--profile-dir DIR]   # TUNNEL_PROFILE dumps + reports

The profile dumps come from native/core/profiler.cc and are symbolised with
scripts/profile_report.py.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import start_mock  # noqa: E402
from p2p_llm_tunnel_amd import binary  # noqa: E402
from p2p_llm_tunnel_amd.utils.procs import Tunnel, free_port  # noqa: E402


def cpu_s(pid: int) -> float:
    st = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
    return (int(st[11]) + int(st[12])) / os.sysconf("SC_CLK_TCK")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="webrtc")
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--mb", type=int, default=1)
    ap.add_argument("--profile-dir", default=None)
    ap.add_argument("--extra", default="", help="extra flags for both tunnel processes, e.g. --no-jumbo-loopback")
    ap.add_argument("--serve-extra", default="", help="extra flags for serve only, e.g. --stream-body-threshold 65536")
    ap.add_argument("--mock-threads", type=int, default=int(os.environ.get("P2PT_MOCK_THREADS", "1")),
                    help="reactor threads of the echo upstream (one thread saturates at ~2500 req/s of this row)")
    ap.add_argument("--pin", action="store_true", help="pin loadgen / mock / serve / proxy to disjoint CPUs")
    ap.add_argument("--timeline", action="store_true",
                    help="per-thread CPU utilisation in 2 ms intervals (TUNNEL_THREAD_TIMELINE), summarised per thread")
    a = ap.parse_args()
    extra = [x for x in a.extra.split() if x]
    serve_only = [x for x in a.serve_extra.split() if x]
    from p2p_llm_tunnel_amd.utils import netstat
    from p2p_llm_tunnel_amd.utils.pinning import cgroup_cpu_stat, cpu_plan, cpu_stat_delta
    plan = cpu_plan() if a.pin else {}
    env = None
    if a.profile_dir:
        os.makedirs(a.profile_dir, exist_ok=True)
        env = {"TUNNEL_PROFILE": os.path.join(os.path.abspath(a.profile_dir), "tunnel.%p.prof@2000")}
    tl_dir = None
    if a.timeline:
        from p2p_llm_tunnel_amd.utils import timeline
        tl_dir, tl_env = timeline.new_dir()
        env = dict(env or {}, **tl_env)
    mock, port = start_mock("native", 100, 5, plan.get("mock"), a.mock_threads)
    ms, mp = free_port(), free_port()
    out = {}
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport=a.transport, env=env,
                    serve_extra=["--metrics-listen", f"127.0.0.1:{ms}"] + extra + serve_only +
                    (["--cpu-affinity", plan["serve"]] if plan else []),
                    proxy_extra=["--metrics-listen", f"127.0.0.1:{mp}"] + extra +
                    (["--cpu-affinity", plan["proxy"]] if plan else [])) as t:
            def run(target):
                r = subprocess.run((["taskset", "-c", plan["loadgen"]] if plan else []) +
                                   [binary("tunnel-loadgen"), "--target", f"127.0.0.1:{target}", "--streams",
                                    str(a.streams), "--steps", str(a.steps), "--warmup", "1", "--post-bytes",
                                    str(a.mb << 20)], capture_output=True, text=True, timeout=600)
                return json.loads(r.stdout.strip().splitlines()[-1])
            pids = {"serve": t.serve.popen.pid, "proxy": t.proxy.popen.pid, "mock": mock.popen.pid}
            c0 = {k: cpu_s(v) for k, v in pids.items()}
            g0, k0 = cgroup_cpu_stat(), netstat.snapshot()
            t0 = time.time()
            tr = run(t.proxy_port)
            wall = time.time() - t0
            c1 = {k: cpu_s(v) for k, v in pids.items()}
            g1, k1 = cgroup_cpu_stat(), netstat.snapshot()
            dr = run(port)
            g2, k2 = cgroup_cpu_stat(), netstat.snapshot()
            out = {"transport": a.transport, "extra": a.extra, "mock_threads": a.mock_threads, "serve_extra": a.serve_extra, "pinned": plan, "path": t.serve.wait_for("WebRTC connection established", 1)
                   .split(" via ", 1)[-1] if a.transport == "webrtc" else "", "streams": a.streams, "body_mb": a.mb, "steps": a.steps,
                   "tunneled_req_s": tr["req_s"], "direct_req_s": dr["req_s"],
                   "tunneled_MBps_each_way": tr["req_s"] * a.mb * 1.048576, "errors": tr["errors"] + dr["errors"],
                   "wall_s_incl_warmup": round(wall, 3),
                   "cpu_s_incl_warmup": {k: round(c1[k] - c0[k], 3) for k in pids}, "pids": pids,
                   "tunneled_cgroup": cpu_stat_delta(g0, g1), "direct_cgroup": cpu_stat_delta(g1, g2),
                   "kernel_tunneled": netstat.delta(k0, k1), "kernel_direct": netstat.delta(k1, k2),
                   "tunneled_step_ms": tr.get("step_ms"), "direct_step_ms": dr.get("step_ms")}
            for name, p in (("serve", ms), ("proxy", mp)):
                txt = urllib.request.urlopen(f"http://127.0.0.1:{p}/metrics", timeout=5).read().decode()
                out[f"{name}_sctp"] = {l.split()[0]: float(l.split()[1]) for l in txt.splitlines()
                                       if l.startswith(("tunnel_sctp", "tunnel_dtls", "tunnel_udp"))}
            # Loss the stack could not see and self-inflicted drops, both sides.
            out["loss"] = {k: sum(out[f"{n}_sctp"].get(m, 0.0) for n in ("serve", "proxy")) for k, m in (
                ("udp_rx_overflow", "tunnel_udp_rx_overflow_total"), ("lane_send_drops", "tunnel_dtls_lane_send_drops"),
                ("udp_send_drops", "tunnel_udp_send_drops"),
                ("lane_send_waits", "tunnel_dtls_lane_send_waits"), ("reader_waits", "tunnel_udp_reader_waits"), ("reader_escapes", "tunnel_udp_reader_escapes"),
                ("fast_retransmits", "tunnel_sctp_fast_retransmits"), ("retransmits", "tunnel_sctp_retransmits"),
                ("t3_expirations", "tunnel_sctp_t3_expirations"), ("tlp_probes", "tunnel_sctp_tlp_probes"),
                ("rack_marks", "tunnel_sctp_rack_marks"), ("spurious_undos", "tunnel_sctp_spurious_undos"),
                ("probe_ambiguous", "tunnel_sctp_probe_ambiguous"), ("dup_tsns_received", "tunnel_sctp_dup_tsns_received"), ("late_tsns_received", "tunnel_sctp_late_tsns_received"),
                ("rwnd_drops", "tunnel_sctp_rwnd_drops"), ("dtls_rx_dropped", "tunnel_dtls_rx_dropped"))}
    finally:
        mock.stop()
    if tl_dir and out:
        # Share of each thread's active 2 ms intervals (>= 10 % CPU) spent at
        # >= 90 % / >= 75 % CPU, over the process's life (warm-up, tunneled and
        # direct runs; the direct run adds idle intervals only).
        out["timeline"] = timeline.summarise(tl_dir, out.get("pids", {}))
    from p2p_llm_tunnel_amd.utils.boxinfo import identity
    out["box"] = identity()
    print(json.dumps(out))
    if a.profile_dir:
        for f in sorted(glob.glob(os.path.join(a.profile_dir, "tunnel.*.prof"))):
            rep = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "profile_report.py"), f, "--top", "25"],
                                 capture_output=True, text=True).stdout
            with open(f[:-5] + ".txt", "w") as fh:
                fh.write(rep)


if __name__ == "__main__":
    main()
