#!/usr/bin/env python3
"""Symbolise a TUNNEL_PROFILE dump (native/core/profiler.cc) and print self /
inclusive tables.

    TUNNEL_PROFILE=/tmp/serve.prof build/bin/tunnel serve ...
    python scripts/profile_report.py /tmp/serve.prof [--top 40]

Each dump line is ``count addr0 addr1 ...`` where addr0 is the interrupted PC,
addr1 the word at the stack pointer (caller of a frameless leaf, heuristic) and
the rest frame-pointer return addresses, all as ``module+0xoffset``.
"""
from __future__ import annotations

import argparse
import bisect
import collections
import os
import subprocess

def _dynsyms(mod: str) -> tuple[list[int], list[str]]:
    r = subprocess.run(["nm", "-D", "--defined-only", mod], capture_output=True, text=True)
    syms = sorted((int(p[0], 16), p[2].split("@")[0]) for p in (l.split() for l in r.stdout.splitlines())
                  if len(p) == 3 and p[1] in "tTwWiI")
    return [a for a, _ in syms], [n for _, n in syms]


def symbolise(addrs: set[tuple[str, int]]) -> dict[tuple[str, int], str]:
    """addr2line for modules with symbols; nearest exported symbol otherwise
    (glibc's memcpy variants are local symbols: they show as '<export>+off')."""
    by_mod: dict[str, list[int]] = collections.defaultdict(list)
    for mod, off in addrs:
        by_mod[mod].append(off)
    out: dict[tuple[str, int], str] = {}
    for mod, offs in by_mod.items():
        base = os.path.basename(mod)
        if mod == "?" or not os.path.exists(mod):
            for o in offs:
                out[(mod, o)] = f"{base}+{o:#x}"
            continue
        r = subprocess.run(["addr2line", "-f", "-C", "-e", mod] + [f"{o:#x}" for o in offs],
                           capture_output=True, text=True)
        lines = r.stdout.splitlines()
        ea, en = None, None
        for i, o in enumerate(offs):
            fn = lines[2 * i] if 2 * i < len(lines) else "??"
            if fn == "??":
                if ea is None:
                    ea, en = _dynsyms(mod)
                k = bisect.bisect_right(ea, o) - 1
                fn = f"{base}:{en[k]}+{o - ea[k]:#x}" if k >= 0 else f"{base}+{o:#x}"
            out[(mod, o)] = fn if len(fn) < 140 else fn[:137] + "..."
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--thread", default=None,
                    help="only samples of this thread tag (0 = main reactor, k = worker k; 'workers' = all k > 0)")
    ap.add_argument("--leaf", default=None,
                    help="also list the fp-chain callers (frames 2..4) of samples whose leaf contains this text")
    a = ap.parse_args()
    per_thread = collections.Counter()
    stacks = []
    header = ""
    for line in open(a.dump):
        if line.startswith("#"):
            header = line.strip()
            continue
        parts = line.split()
        cnt = int(parts[0])
        tag = 0
        if len(parts) > 1 and parts[1].startswith("T") and "+" not in parts[1]:
            tag = int(parts[1][1:])
            parts = [parts[0]] + parts[2:]
        per_thread[tag] += cnt
        if a.thread is not None and not (a.thread == "workers" and tag > 0) and a.thread != str(tag):
            continue
        frames = []
        for i, tok in enumerate(parts[1:]):
            mod, off = tok.rsplit("+", 1)
            off = int(off, 16)
            if i >= 1 and off:
                off -= 1  # return address -> call site
            frames.append((mod, off))
        stacks.append((cnt, frames))
    addrs = {f for _, fr in stacks for f in fr}
    names = symbolise(addrs)
    total = sum(c for c, _ in stacks) or 1
    self_t = collections.Counter()
    incl = collections.Counter()
    leaf_caller = collections.Counter()
    for cnt, fr in stacks:
        leaf = names[fr[0]]
        self_t[leaf] += cnt
        seen = set()
        # frame 1 is a heuristic (valid when the leaf had no frame of its own)
        for i, f in enumerate(fr):
            n = names[f]
            if n in seen:
                continue
            seen.add(n)
            incl[n] += cnt
        if len(fr) > 1:
            leaf_caller[(leaf, names[fr[1]])] += cnt
    print(header)
    allt = sum(per_thread.values()) or 1
    print("threads (samples %): " + ", ".join(f"T{t} {100 * c / allt:.1f}" for t, c in sorted(per_thread.items())))
    if a.thread is not None:
        print(f"(tables below: thread {a.thread} only)")
    print(f"\n{'self %':>7}  function")
    for n, c in self_t.most_common(a.top):
        print(f"{100 * c / total:7.2f}  {n}")
    print(f"\n{'incl %':>7}  function")
    for n, c in incl.most_common(a.top):
        print(f"{100 * c / total:7.2f}  {n}")
    print(f"\n{'%':>7}  leaf <- caller")
    for (l, cl), c in leaf_caller.most_common(a.top):
        print(f"{100 * c / total:7.2f}  {l}  <-  {cl}")
    if a.leaf:
        chains = collections.Counter()
        for cnt, fr in stacks:
            if a.leaf in names[fr[0]]:
                chain = [names[f][:70] for f in fr[2:5] if not names[f].startswith("?")]
                chains[" <- ".join(chain) or "?"] += cnt
        print(f"\n{'%':>7}  callers of leaves matching {a.leaf!r} (fp chain)")
        for ch, c in chains.most_common(a.top):
            print(f"{100 * c / total:7.2f}  {ch}")


if __name__ == "__main__":
    main()
