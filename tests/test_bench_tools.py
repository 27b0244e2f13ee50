"""The host-benchmark tooling: the A/B runner (bench/ab.py), CPU plans for
pinned runs, per-thread timelines, kernel counter deltas and the tunnel's
per-thread CPU pinning switch (TUNNEL_PIN_THREADS with --cpu-affinity)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import ab  # noqa: E402
from p2p_llm_tunnel_amd.utils import netstat, pinning, timeline  # noqa: E402


def test_ab_variants_and_key_numbers():
    v = ab.parse_variants("base: co:TUNNEL_COALESCE_US=0 both:A=1,B=2")
    assert v == [("base", {}), ("co", {"TUNNEL_COALESCE_US": "0"}), ("both", {"A": "1", "B": "2"})]
    k = ab.key_numbers("bulk", {"tunneled_req_s": 1500.0, "direct_req_s": 2000.0})
    assert k == {"tunneled_req_s": 1500.0, "direct_req_s": 2000.0, "ratio": 0.75}
    node = {"runs": [{"streams": 256, "added_p50_ttft_ms": 0.3, "tunneled_p99_ttft_ms": 1.6,
                      "direct_p99_ttft_ms": 0.4, "events_ratio": 0.99}]}
    assert ab.key_numbers("node", node)["s256.added_p50_ttft_ms"] == 0.3


def test_ab_stops_on_a_failed_run(tmp_path):
    # an argument the bench rejects: the A/B ends with exit 1, nothing retried
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "ab.py"), "node", "--reps", "2",
                        "--out", str(tmp_path), "--", "--no-such-flag"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "exit 2" in r.stdout and r.stdout.count("rep ") == 1


def test_cpu_plan_splits_sixteen(monkeypatch):
    plan = pinning.cpu_plan(list(range(16)), by_side=False)
    assert plan == {"loadgen": "0-1", "mock": "2-3", "serve": "4-9", "proxy": "10-15"}
    # two 8-CPU L3 domains: client side on one, server side on the other
    monkeypatch.setattr(pinning, "l3_groups", lambda cpus: [cpus[:8], cpus[8:]])
    monkeypatch.delenv("P2PT_PIN_PLAN", raising=False)
    assert pinning.cpu_plan(list(range(16))) == {"loadgen": "0-1", "mock": "2-3", "serve": "4-9", "proxy": "10-15"}
    monkeypatch.setenv("P2PT_PIN_PLAN", "side")
    assert pinning.cpu_plan(list(range(16)))["proxy"] == "2-7"
    plan = pinning.cpu_plan(list(range(16)), by_side="auto")
    assert plan == {"loadgen": "0-1", "proxy": "2-7", "serve": "8-13", "mock": "14-15"}
    assert pinning.cpu_plan([0, 1, 2]) == {}
    assert pinning.parse_cpus("0-2,5") == [0, 1, 2, 5]


def test_cgroup_and_netstat_deltas():
    a = {"usage_usec": 10, "nr_periods": 1, "nr_throttled": 0, "throttled_usec": 0}
    b = {"usage_usec": 25, "nr_periods": 3, "nr_throttled": 1, "throttled_usec": 7}
    assert pinning.cpu_stat_delta(a, b) == {"usage_usec": 15, "nr_periods": 2, "nr_throttled": 1, "throttled_usec": 7}
    snap = netstat.snapshot()
    assert isinstance(snap, dict)
    if snap:  # Linux: the TCP MIB is there
        assert "Tcp.RetransSegs" in snap
        assert netstat.delta(snap, snap)["Tcp.RetransSegs"] == 0
        assert netstat.delta(snap, snap, everything=True) == {}


def test_timeline_summary(tmp_path):
    d = {"threads": [{"tag": 0, "busy_s": 1.5, "hist": [10, 2, 2, 2, 2, 4]},
                     {"tag": 93, "busy_s": 0.5, "hist": [20, 4, 0, 0, 0, 0]}]}
    with open(tmp_path / "tl.42.json", "w") as f:
        json.dump(d, f)
    s = timeline.summarise(str(tmp_path), {"serve": 42, "proxy": 43})
    assert s["serve.assoc"]["active_intervals"] == 12
    assert s["serve.assoc"]["sat90_share_of_active"] == round(4 / 12, 3)
    assert s["serve.tx_send"]["sat75_share_of_active"] == 0.0
    assert not any(k.startswith("proxy.") for k in s)


@pytest.mark.skipif(not sys.platform.startswith("linux"), reason="sched_setaffinity")
def test_tunnel_threads_pinned_one_cpu_each(mock_upstream):
    """With --cpu-affinity the tunnel's threads each take one CPU of the set
    (the association thread the first); TUNNEL_PIN_THREADS=0 leaves them
    floating over the whole set."""
    from p2p_llm_tunnel_amd.utils.procs import Tunnel
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 3:
        pytest.skip("needs 3 CPUs")
    spec = ",".join(str(c) for c in cpus[:3])

    def thread_sets(pid):
        out = {}
        for tid in os.listdir(f"/proc/{pid}/task"):
            out[tid] = frozenset(os.sched_getaffinity(int(tid)))
        return out

    with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--cpu-affinity", spec, "--workers", "2"]) as t:
        sets = thread_sets(t.serve.popen.pid)
        assert frozenset([cpus[0]]) in sets.values()          # the association thread
        assert all(len(s) == 1 for s in sets.values())        # every thread on one CPU
        assert set().union(*sets.values()) <= set(cpus[:3])
    with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--cpu-affinity", spec],
                env={"TUNNEL_PIN_THREADS": "0"}) as t:
        sets = thread_sets(t.serve.popen.pid)
        assert all(s == frozenset(cpus[:3]) for s in sets.values())
    if len(cpus) >= 6:
        # auto workers follow the set given (6 CPUs, one per thread: the
        # association thread, reader and TX stages take four, 1 worker), not
        # the one CPU the association thread pinned itself to first
        spec6 = ",".join(str(c) for c in cpus[:6])
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--cpu-affinity", spec6]) as t:
            pid = t.serve.popen.pid
            names = [open(f"/proc/{pid}/task/{tid}/comm").read().strip() for tid in os.listdir(f"/proc/{pid}/task")]
            assert sum(n.startswith("p2pt-w") for n in names) == 1, names
        with Tunnel(mock_upstream, transport="webrtc", serve_extra=["--cpu-affinity", spec6],
                    env={"TUNNEL_PIN_THREADS": "0"}) as t:  # floating threads: half the CPUs less one
            pid = t.serve.popen.pid
            names = [open(f"/proc/{pid}/task/{tid}/comm").read().strip() for tid in os.listdir(f"/proc/{pid}/task")]
            assert sum(n.startswith("p2pt-w") for n in names) == 2, names
