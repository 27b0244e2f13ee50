"""Kernel TCP/UDP counters of this network namespace (/proc/net/snmp and
/proc/net/netstat), for benchmarks that cross loopback TCP: a segment the
kernel drops on loopback (receive backlog over its limit, receive queue
pruned under memory pressure) is retransmitted only after TCP's minimum RTO,
200 ms — a stall no tunnel counter can see.
"""
from __future__ import annotations

KEYS = ("Tcp.RetransSegs", "TcpExt.TCPTimeouts", "TcpExt.TCPLossProbes", "TcpExt.TCPBacklogDrop",
        "TcpExt.TCPRcvQDrop", "TcpExt.PruneCalled", "TcpExt.RcvPruned", "TcpExt.TCPOFODrop",
        "TcpExt.TCPZeroWindowDrop", "TcpExt.TCPFastRetrans", "TcpExt.TCPSpuriousRTOs", "TcpExt.TCPMemoryPressures",
        "TcpExt.ListenOverflows", "TcpExt.ListenDrops", "TcpExt.TCPFromZeroWindowAdv", "TcpExt.TCPToZeroWindowAdv",
        "Udp.RcvbufErrors", "Udp.SndbufErrors", "Udp.InErrors")


def snapshot() -> dict[str, int]:
    out: dict[str, int] = {}
    for path in ("/proc/net/snmp", "/proc/net/netstat"):
        try:
            with open(path) as f:
                lines = f.read().splitlines()
        except OSError:
            continue
        for names, vals in zip(lines[::2], lines[1::2]):
            n, v = names.split(), vals.split()
            if not n or n[0] != v[0]:
                continue
            proto = n[0].rstrip(":")
            for k, x in zip(n[1:], v[1:]):
                try:
                    out[f"{proto}.{k}"] = int(x)
                except ValueError:
                    pass
    return out


def delta(a: dict[str, int], b: dict[str, int], everything: bool = False) -> dict[str, int]:
    """b - a over KEYS (keys missing on this kernel are left out); with
    everything=True, every counter that moved."""
    if everything:
        return {k: b[k] - a[k] for k in sorted(b) if k in a and b[k] != a[k]}
    return {k: b[k] - a[k] for k in KEYS if k in a and k in b}
