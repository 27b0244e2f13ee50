"""Per-thread CPU utilisation timelines of tunnel processes.

``TUNNEL_THREAD_TIMELINE=<dir>/tl.%p.json`` makes a tunnel process sample the
CPU clocks of its registered threads every 2 ms and write, at exit, a
histogram per thread of those intervals by utilisation (<10, <25, <50, <75,
<90, >=90 %; native/core/profiler.cc). ``summarise()`` turns the files of a
run's processes into one row per thread: busy seconds, active intervals
(>= 10 %) and the share of them at >= 90 % / >= 75 % CPU — which stage of the
pipeline saturates.
"""
from __future__ import annotations

import json
import os
import tempfile

# Thread tags (native/rtc/datapath.cc Lane/RxReader, native/tunnel/workers.cc).
NAMES = {0: "assoc", 90: "tx_seal", 94: "tx_seal2", 93: "tx_send", 91: "rx_lane", 92: "udp_reader"}


def new_dir() -> tuple[str, dict[str, str]]:
    """A scratch directory and the environment that points the tunnel at it."""
    d = tempfile.mkdtemp(prefix="p2pt-timeline-")
    return d, {"TUNNEL_THREAD_TIMELINE": os.path.join(d, "tl.%p.json")}


def summarise(tl_dir: str, pids: dict[str, int]) -> dict[str, dict]:
    """{"<role>.<thread>": {busy_s, active_intervals, sat90_share_of_active,
    sat75_share_of_active}} for each role -> pid whose file exists."""
    out: dict[str, dict] = {}
    for role, pid in pids.items():
        f = os.path.join(tl_dir, f"tl.{pid}.json")
        if not os.path.exists(f):
            continue
        with open(f) as fh:
            d = json.load(fh)
        for t in d["threads"]:
            h = t["hist"]
            busy = sum(h[1:])
            out[f"{role}.{NAMES.get(t['tag'], 'worker%d' % t['tag'])}"] = {
                "busy_s": t["busy_s"], "active_intervals": busy,
                "sat90_share_of_active": round(h[5] / busy, 3) if busy else 0.0,
                "sat75_share_of_active": round((h[4] + h[5]) / busy, 3) if busy else 0.0}
    return out
