"""Per-position kernel timing of a repeated step from a rocprofv3 kernel trace.

    python scripts/rocprof_steps.py RESULTS.db [--marker k_embed] [--label small_b1]

Dispatches are ordered by start time and cut into steps at each ``--marker``
kernel (the first kernel of a decode step). For every position in the step it
prints the median duration and the median gap from the previous kernel's end
(the dependent-launch boundary), then the step's median span, its summed kernel
time and summed gaps.
"""
import argparse
import sqlite3
import statistics


def dispatches(db):
    names = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
    for view in ("kernels", "rocpd_kernel_dispatch"):
        if view in names:
            cols = [r[1] for r in db.execute(f"pragma table_info({view})")]
            nm = next(c for c in ("kernel_name", "name", "display_name") if c in cols)
            st = next(c for c in ("start", "start_ns", "begin") if c in cols)
            en = next(c for c in ("end", "end_ns", "stop") if c in cols)
            rows = db.execute(f'select "{nm}", "{st}", "{en}" from {view} order by "{st}"').fetchall()
            return [(str(n), int(s), int(e)) for n, s, e in rows]
    raise SystemExit(f"no kernel dispatch view in {names}")


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return (name.split("(")[0] if "(" in name else name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_embed")
    ap.add_argument("--label", default="")
    ap.add_argument("--skip", type=int, default=3, help="leading steps to drop (warm-up)")
    a = ap.parse_args()
    d = dispatches(sqlite3.connect(a.db))
    steps, cur = [], None
    for n, s, e in d:
        if a.marker in n:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((n, s, e))
    steps = steps[a.skip:-1] if len(steps) > a.skip + 1 else steps
    L = statistics.mode(len(s) for s in steps)
    steps = [s for s in steps if len(s) == L]
    print(f"### {a.label} ({len(steps)} steps of {L} kernels; µs, medians)\n")
    print("| # | kernel | duration | gap before |")
    print("|---:|---|---:|---:|")
    tot_k = tot_g = 0.0
    for i in range(L):
        dur = statistics.median((s[i][2] - s[i][1]) / 1e3 for s in steps)
        gap = statistics.median((s[i][1] - s[i - 1][2]) / 1e3 for s in steps) if i else 0.0
        tot_k += dur
        tot_g += gap
        print(f"| {i} | {short(steps[0][i][0])} | {dur:.2f} | {gap:.2f} |")
    span = statistics.median((s[-1][2] - s[0][1]) / 1e3 for s in steps)
    print(f"\nstep span {span:.1f} µs = kernels {tot_k:.1f} + gaps {tot_g:.1f} (medians per position)\n")


if __name__ == "__main__":
    main()
