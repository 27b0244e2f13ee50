"""bench.py contract: one JSON line from rank 0 with the driver's keys, value =
whole-job req/s aggregated over ranks (weak scaling), on 1 and 2 ranks
(torch.distributed.run, gloo; the tunnel workload itself is host-side)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(argv, timeout=300):
    out = subprocess.run(argv, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                         env={**os.environ, "MASTER_ADDR": "127.0.0.1"})
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _check(d, n, steps, warmup):
    assert KEYS <= set(d)
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["scaling"] == "weak" and d["higher_is_better"] is True and d["errors"] == 0
    assert d["config"]["global_batch"] == 8 * n
    # 8 streams per rank, one 5-token completion (~0.5 s) per step: ~16 req/s per rank
    assert 12 * n < d["value"] < 17 * n
    assert abs(d["value"] - 8 * n * steps / (d["ms_per_step"] * steps / 1e3)) < 1e-6 * d["value"]


def test_bench_single_rank():
    d = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--curve", "1", "--curve-steps", "1"])
    _check(d, 1, 2, 1)
    assert "1" in d["curve_rank0"] and "8" in d["curve_rank0"]
    assert d["curve_steps"] == 1
    # The host the numbers came from (rows move 20-40 % between boxes).
    assert {"cpu_model", "host_hash", "governor", "deepest_idle", "cpus_allowed", "cgroup_cpus", "io_uring"} <= set(d["box"])
    assert d["config"]["assoc"] == int(os.environ.get("TUNNEL_ASSOC", "3"))


def test_bench_curve_points_default_to_the_headline_steps():
    d = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--curve", "2", "--no-jumbo-extra"])
    _check(d, 1, 2, 1)
    assert d["curve_steps"] == 2


def test_bench_two_ranks_torchrun():
    from p2p_llm_tunnel_amd.utils.procs import free_port
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
              "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
              "--curve", "", "--curve-steps", "1"])
    _check(d, 2, 2, 1)
