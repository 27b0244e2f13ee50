"""Identity of the host a benchmark ran on.

Rows of the same build move 20-40 % between the pool's boxes
(profiles/README.md), so every bench JSON records which box it came from:
CPU model, a hash of the hostname (not the name itself), the cpufreq
governor, the deepest enabled idle state with its exit latency, the CPUs this
process may use, the cgroup CPU quota, and whether io_uring is available to
unprivileged processes (docs/ROUND6.md, node row).

    python -m p2p_llm_tunnel_amd.utils.boxinfo     # one JSON line
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import socket


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_model() -> str | None:
    txt = _read("/proc/cpuinfo") or ""
    for line in txt.splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return None


def governor() -> str | None:
    return _read("/sys/devices/system/cpu/cpu0/cpufreq/scaling_governor")


def deepest_idle_state(cpu: int = 0) -> dict | None:
    """The deepest cpuidle state not disabled on `cpu`: name and exit latency (us)."""
    base = f"/sys/devices/system/cpu/cpu{cpu}/cpuidle"
    best = None
    try:
        states = sorted(os.listdir(base), key=lambda s: int(s[5:]) if s[5:].isdigit() else -1)
    except OSError:
        return None
    for s in states:
        if not s.startswith("state"):
            continue
        if _read(f"{base}/{s}/disable") == "1":
            continue
        lat = _read(f"{base}/{s}/latency")
        best = {"name": _read(f"{base}/{s}/name"), "exit_latency_us": int(lat) if lat and lat.isdigit() else None}
    return best


def cgroup_cpu_quota() -> float | None:
    """CPUs the cgroup may use (cpu.max quota / period), None when unlimited."""
    txt = _read("/sys/fs/cgroup/cpu.max")
    if not txt:
        return None
    q, _, p = txt.partition(" ")
    if q == "max" or not p:
        return None
    try:
        return round(int(q) / int(p), 2)
    except ValueError:
        return None


def io_uring_allowed() -> str:
    """'yes', or why not ('ENOSYS', 'EPERM', ...): io_uring_setup(2) with 8 entries."""
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        params = (ctypes.c_uint8 * 120)()
        fd = libc.syscall(425, 8, ctypes.byref(params))  # __NR_io_uring_setup (x86_64)
        if fd >= 0:
            os.close(fd)
            return "yes"
        import errno
        return errno.errorcode.get(ctypes.get_errno(), str(ctypes.get_errno()))
    except Exception as e:  # pragma: no cover
        return f"error: {e}"


def identity() -> dict:
    host = socket.gethostname()
    aff = sorted(os.sched_getaffinity(0))
    return {
        "cpu_model": cpu_model(),
        "host_hash": hashlib.sha256(host.encode()).hexdigest()[:12],
        "governor": governor(),
        "deepest_idle": deepest_idle_state(aff[0] if aff else 0),
        "cpus_allowed": len(aff),
        "cgroup_cpus": cgroup_cpu_quota(),
        "io_uring": io_uring_allowed(),
    }


if __name__ == "__main__":
    print(json.dumps(identity()))
