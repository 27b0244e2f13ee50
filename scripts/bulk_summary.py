#!/usr/bin/env python3
"""Median and min-max per path of bulk runs (profile_bulk.py JSON files named
<path>_<rep>.json in DIR): tunneled req/s, direct req/s, tunneled/direct."""
import glob
import json
import os
import statistics
import sys


def main(d):
    rows = {}
    for f in sorted(glob.glob(os.path.join(d, "*_*.json"))):
        name = os.path.basename(f).rsplit("_", 1)[0]
        j = json.load(open(f))
        rows.setdefault(name, []).append(j)
    out = {}
    for name, runs in rows.items():
        t = [r["tunneled_req_s"] for r in runs]
        dd = [r["direct_req_s"] for r in runs]
        q = [a / b for a, b in zip(t, dd)]

        def s(v):
            return {"median": round(statistics.median(v), 3), "min": round(min(v), 3), "max": round(max(v), 3)}
        out[name] = {"runs": len(runs), "steps": runs[0].get("steps"), "tunneled_req_s": s(t), "direct_req_s": s(dd),
                     "ratio": s(q), "errors": sum(r["errors"] for r in runs)}
        print(f"{name:6s} n={len(runs)} tunneled {s(t)['median']:.0f} [{s(t)['min']:.0f}-{s(t)['max']:.0f}]  "
              f"direct {s(dd)['median']:.0f} [{s(dd)['min']:.0f}-{s(dd)['max']:.0f}]  "
              f"ratio {s(q)['median']:.3f} [{s(q)['min']:.3f}-{s(q)['max']:.3f}]")
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
