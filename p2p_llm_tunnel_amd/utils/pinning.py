"""Disjoint CPU sets for the processes of a benchmark on one host.

The bulk and node rows run four kinds of process on one box — the load
generator, the mock upstream, ``tunnel serve`` and ``tunnel proxy`` — and
left to the scheduler they share and migrate between cores, which made the
direct leg of one row move by 40 % between repetitions.
``cpu_plan()`` splits the CPUs this process may use (``P2PT_CPUS`` overrides,
e.g. ``0-15``; at most ``P2PT_CPU_BUDGET``, default 16, the pool's share per
GPU) into one set per role, in the same proportions on every box:

    loadgen 1/8, mock 1/8, serve 3/8, proxy 3/8   (16 CPUs: 2 / 2 / 6 / 6)

When the CPUs span two L3 domains (two CCDs), the client side (loadgen,
proxy) takes one and the server side (serve, mock) the other (cpu_plan).

Each tunnel process holds an association thread, a DTLS TX lane, a socket
reader, an RX lane and its HTTP workers; the load generator and the mock are
single reactors (the direct leg runs on exactly their CPUs too).
"""
from __future__ import annotations

import os


def parse_cpus(spec: str) -> list[int]:
    out: list[int] = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.extend(range(int(lo), int(hi) + 1))
        else:
            out.append(int(part))
    return out


def fmt_cpus(cpus: list[int]) -> str:
    cpus = sorted(cpus)
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def available_cpus() -> list[int]:
    spec = os.environ.get("P2PT_CPUS")
    cpus = parse_cpus(spec) if spec else sorted(os.sched_getaffinity(0))
    budget = int(os.environ.get("P2PT_CPU_BUDGET", "16"))
    return cpus[:budget]


def l3_groups(cpus: list[int]) -> list[list[int]]:
    """cpus grouped by shared L3 (one CCD on EPYC), in order; one group when
    the topology is unknown."""
    groups: dict[str, list[int]] = {}
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                key = f.read().strip()
        except OSError:
            key = ""
        groups.setdefault(key, []).append(c)
    return list(groups.values())


def cpu_plan(cpus: list[int] | None = None, by_side=None) -> dict[str, str]:
    """Role -> CPU list string (taskset / --cpu-affinity syntax); {} with fewer than 4 CPUs.

    Default (P2PT_PIN_PLAN=order, or by_side False): the split above, in CPU
    order: load generator and mock on the first CPUs. On the pool's 16-CPU
    budget over two 8-core CCDs (own L3 each) that keeps the direct leg
    (load generator <-> mock) inside one L3 while the tunneled leg crosses
    between them.
    by_side True (P2PT_PIN_PLAN=side; "auto": when the CPUs span exactly two
    L3 domains of equal size): the client side (load generator, proxy) on
    one L3, the server side (serve, mock) on the other, as two machines would
    be, so the direct leg and the tunnel each cross once. On the host that
    moves the direct leg more than the tunnel (2660 -> 1850 req/s against
    1760 -> 1810 at 1200 MTU; profiles/r04/plan26), so the published rows use
    the default."""
    cpus = available_cpus() if cpus is None else list(cpus)
    n = len(cpus)
    if n < 4:
        return {}
    mode = os.environ.get("P2PT_PIN_PLAN", "order")
    if by_side is None:  # P2PT_PIN_PLAN: order (default), order75 (serve one CPU more), side, auto
        by_side = {"order": False, "order75": False, "side": True}.get(mode, "auto")
    groups = l3_groups(cpus) if by_side else [cpus]
    if by_side == "auto":
        by_side = len(groups) == 2 and len(groups[0]) == len(groups[1]) and len(groups[0]) >= 4
    if by_side and len(groups) == 2:
        a, b = groups
        k = max(1, len(a) // 4)
        plan = {"loadgen": a[:k], "proxy": a[k:], "serve": b[:len(b) - k], "mock": b[len(b) - k:]}
        return {k_: fmt_cpus(v) for k_, v in plan.items()}
    lg = max(1, n // 8)
    mk = max(1, n // 8)
    rest = n - lg - mk
    sv = rest // 2 + (1 if mode == "order75" and rest >= 10 else 0)
    plan = {"loadgen": cpus[:lg], "mock": cpus[lg:lg + mk], "serve": cpus[lg + mk:lg + mk + sv],
            "proxy": cpus[lg + mk + sv:]}
    return {k: fmt_cpus(v) for k, v in plan.items()}


def cgroup_cpu_stat() -> dict[str, int]:
    """The job cgroup's CPU accounting (cgroup v2 ``cpu.stat``): ``usage_usec``
    (CPU time of every process in the job), ``nr_periods``, ``nr_throttled`` and
    ``throttled_usec``. On the GPU pool the job's quota is 16 CPUs
    (``cpu.max`` 1600000/100000): a burst past it stalls EVERY process of the
    job, loadgen and mock included, until the next 100 ms period — a tail that
    is no stage's own. {} where the file is absent."""
    out: dict[str, int] = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if v.strip().isdigit():
                    out[k] = int(v)
    except OSError:
        pass
    return out


def cpu_stat_delta(a: dict[str, int], b: dict[str, int]) -> dict[str, int]:
    """b - a for the throttling keys of two cgroup_cpu_stat() snapshots."""
    keys = ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec")
    return {k: b[k] - a[k] for k in keys if k in a and k in b}


def physical_cores(cpus: list[int]) -> list[int]:
    """The first hardware thread of every core among cpus (SMT siblings dropped)."""
    out, seen = [], set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                key = f.read().strip()
        except OSError:
            key = str(c)
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def cpu_busy(sample_s: float = 0.3) -> dict[int, float]:
    """Per-CPU busy share over a short sample of /proc/stat (0..1)."""
    import time

    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    parts = line.split()
                    v = [int(x) for x in parts[1:]]
                    idle = v[3] + (v[4] if len(v) > 4 else 0)
                    out[int(parts[0][3:])] = (sum(v), idle)
        return out

    try:
        a = snap()
        time.sleep(sample_s)
        b = snap()
    except OSError:
        return {}
    busy = {}
    for c, (tot, idle) in b.items():
        if c in a:
            dt, di = tot - a[c][0], idle - a[c][1]
            busy[c] = 1.0 - di / dt if dt > 0 else 0.0
    return busy


def ccd_plan(cpus: list[int] | None = None, busy: dict[int, float] | None = None) -> dict[str, str]:
    """The headline's layout: every process of the benchmark on the cores of
    ONE L3 domain (a CCD on EPYC), one core per role thread — load generator,
    mock, serve (association thread first), proxy — so no hop of either leg
    crosses an L3 or a socket, and the direct leg (load generator <-> mock)
    gets the same placement as the tunneled one.

    The pool's jobs have a 16-CPU quota but may run on any of the host's 256
    CPUs, and other jobs run on some of them: the CCD is the idlest one
    (/proc/stat over 0.3 s, SMT siblings included, CPU 0's CCD avoided).
    Pinned to CPUs 0-7 regardless, steps stalled ~10 ms behind other runnable
    work in both legs (profiles/r05/b03); on the idlest CCD they still did in
    3 of 12 runs (b04), so bench.py leaves placement to the scheduler by
    default. {} when no L3 domain has 6 cores."""
    cpus = sorted(os.sched_getaffinity(0)) if cpus is None else list(cpus)
    busy = cpu_busy() if busy is None else busy
    best, best_load = None, None
    for g in l3_groups(cpus):
        cores = physical_cores(g)
        if len(cores) < 6:
            continue
        load = max((busy.get(c, 0.0) for c in g), default=0.0) + (1.0 if 0 in g else 0.0)
        if best is None or load < best_load:
            best, best_load = cores, load
    if not best:
        return {}
    n = len(best)
    sv = (n - 2 + 1) // 2
    return {"loadgen": fmt_cpus(best[:1]), "mock": fmt_cpus(best[1:2]),
            "serve": fmt_cpus(best[2:2 + sv]), "proxy": fmt_cpus(best[2 + sv:])}


def l3_set_plan(cpus: list[int] | None = None, busy: dict[int, float] | None = None) -> dict[str, str]:
    """Every role on the same CPU SET: one hardware thread of each core of the
    idlest L3 domain (the SMT siblings left out), and the scheduler places the
    threads within it. Unlike one CPU per role (ccd_plan), a thread whose CPU
    another job's work takes is moved to a free one of the set instead of
    waiting behind it; unlike no pinning, no hop leaves the L3 and no thread
    runs on the sibling of a busy core (a run whose every hop was 30-40 %
    slower than another's, mock and client included: profiles/r05/b05)."""
    cpus = sorted(os.sched_getaffinity(0)) if cpus is None else list(cpus)
    busy = cpu_busy() if busy is None else busy
    best, best_load = None, None
    for g in l3_groups(cpus):
        cores = physical_cores(g)
        if len(cores) < 6:
            continue
        load = max((busy.get(c, 0.0) for c in g), default=0.0) + (1.0 if 0 in g else 0.0)
        if best is None or load < best_load:
            best, best_load = cores, load
    if not best:
        return {}
    s = fmt_cpus(best)
    return {"loadgen": s, "mock": s, "serve": s, "proxy": s, "set": True}


def where(pid: int) -> list[int]:
    """The CPU each thread of a process last ran on."""
    out = []
    try:
        for t in os.listdir(f"/proc/{pid}/task"):
            with open(f"/proc/{pid}/task/{t}/stat") as f:
                out.append(int(f.read().rsplit(")", 1)[1].split()[36]))
    except (OSError, ValueError, IndexError):
        pass
    return sorted(out)


def numa_nodes() -> dict[int, list[int]]:
    """NUMA node -> its CPUs (one node holding every CPU where sysfs has none)."""
    out: dict[int, list[int]] = {}
    base = "/sys/devices/system/node"
    try:
        for name in sorted(os.listdir(base)):
            if name.startswith("node") and name[4:].isdigit():
                with open(os.path.join(base, name, "cpulist")) as f:
                    out[int(name[4:])] = parse_cpus(f.read().strip())
    except OSError:
        pass
    return out or {0: sorted(os.sched_getaffinity(0))}


def numa_plan(busy: dict[int, float] | None = None) -> dict:
    """Every role on the CPUs of ONE NUMA node (one socket here: 64 cores and
    their SMT siblings), the node with the most idle CPUs; threads placed by
    the scheduler within it. Left to the scheduler over both sockets, runs
    whose threads ended up split across the sockets were the slow ones (the
    round trip of a frame through a remote L3; profiles/r05/b06, b07
    cpus_rank0); one CPU per role stalled behind other jobs' work (b03, b04),
    which a 128-CPU set avoids."""
    allowed = set(os.sched_getaffinity(0))
    busy = cpu_busy() if busy is None else busy
    best, best_idle = None, -1.0
    for node, cpus in numa_nodes().items():
        cpus = [c for c in cpus if c in allowed]
        if not cpus:
            continue
        idle = sum(1.0 - busy.get(c, 0.0) for c in cpus)
        if idle > best_idle:
            best, best_idle = cpus, idle
    if not best:
        return {}
    s = fmt_cpus(best)
    return {"loadgen": s, "mock": s, "serve": s, "proxy": s, "set": True}
