#!/usr/bin/env python3
"""Interleaved A/B runs of the host benchmarks under environment variants.

One entry point for what used to be a shell runner per experiment: each
repetition runs every variant once, in turn, on the same box, so a slow box
or a noisy minute hits all variants alike; the summary gives the median and
min-max of each variant's key numbers.

    python bench/ab.py KIND --variants "base: co0:TUNNEL_COALESCE_US=0" --reps 3 \\
        --out gpurun_out/ab/x [--paths std,jumbo] [-- extra args for the bench]

KIND and what one run is:
  bulk   bench/profile_bulk.py, once per --paths entry (std = 1200-byte MTU,
         jumbo = same-host 16 KiB packets, tcp = the TCP transport): the
         64 x 1 MB echo, tunneled then direct. Key: tunneled/direct req/s.
  wf     scripts/ttft_breakdown.py --bulk-echo (per path): the same row with
         per-request stamps (waterfall, slowest steps). Key: req/s ratio.
  node   bench/bench_node.py --reps 1: one serve over 8 mocks, N SSE streams
         of 1 ms tokens. Key: added p50 TTFT, tunneled / direct p99 TTFT.
  mixed  bench/bench_mixed.py --reps 1: SSE next to 8 x 64 MB downloads.
         Key: SSE TTFT p99 per transport, bulk ratio, proxy RSS.
  head   bench.py: the headline (8 streams). Key: added p50 / p99 TTFT.

A variant is "label:VAR=v,VAR2=w" ("label:" for the environment as is). A
run that fails or times out ends the whole A/B (exit status 1): nothing is
retried. Per-run JSON lands in --out as <label>.<path>_<rep>.json.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_variants(spec: str) -> list[tuple[str, dict[str, str]]]:
    out = []
    for v in spec.split():
        label, _, envs = v.partition(":")
        env = {}
        for kv in [x for x in envs.split(",") if x]:
            k, _, val = kv.partition("=")
            env[k] = val
        out.append((label, env))
    return out


def command(kind: str, path: str, out_file: str, a, extra: list[str]) -> tuple[list[str], bool]:
    """argv of one run and whether it writes its JSON to stdout (else to out_file)."""
    py = sys.executable
    if kind == "bulk":
        x = "--no-jumbo-loopback" if path == "std" else ""
        argv = [py, "bench/profile_bulk.py", "--transport", "tcp" if path == "tcp" else "webrtc",
                "--steps", str(a.steps), f"--extra={x}"]
        if a.pin:
            argv.append("--pin")
        if a.timeline:
            argv.append("--timeline")
        return argv + extra, True
    if kind == "wf":
        argv = [py, "scripts/ttft_breakdown.py", "--bulk-echo", "--steps", str(a.steps)]
        if path == "std":
            argv.append("--extra=--no-jumbo-loopback")
        if a.pin:
            argv.append("--pin")
        return argv + extra, True
    if kind == "node":
        return [py, "bench/bench_node.py", "--reps", "1", "--out", out_file] + extra, False
    if kind == "mixed":
        return [py, "bench/bench_mixed.py", "--reps", "1", "--out", out_file] + extra, False
    if kind == "head":
        return [py, "bench.py", "--out", out_file] + extra, False
    raise SystemExit(f"unknown kind {kind}")


def key_numbers(kind: str, d: dict) -> dict[str, float]:
    if kind == "bulk":
        return {"tunneled_req_s": d["tunneled_req_s"], "direct_req_s": d["direct_req_s"],
                "ratio": d["tunneled_req_s"] / d["direct_req_s"]}
    if kind == "wf":
        return {"tunneled_req_s": d["tunneled"]["req_s"], "direct_req_s": d["direct"]["req_s"], "ratio": d["ratio"]}
    if kind == "node":
        out = {}
        for r in d["runs"]:
            s = r["streams"]
            out.update({f"s{s}.added_p50_ttft_ms": r["added_p50_ttft_ms"],
                        f"s{s}.tunneled_p99_ttft_ms": r["tunneled_p99_ttft_ms"],
                        f"s{s}.direct_p99_ttft_ms": r["direct_p99_ttft_ms"],
                        f"s{s}.events_ratio": r["events_ratio"]})
        return out
    if kind == "mixed":
        out = {}
        for r in d["runs"]:
            t = r["transport"]
            out.update({f"{t}.tunneled_ttft_p99_ms": r["tunneled_ttft_p99_ms"],
                        f"{t}.direct_ttft_p99_ms": r["direct_ttft_p99_ms"], f"{t}.bulk_ratio": r["bulk_ratio"],
                        f"{t}.proxy_rss_peak_mib": r["proxy_rss_peak_mib"]})
        return out
    if kind == "head":
        return {"value": d["value"], "added_p50_ttft_ms": d["added_p50_ttft_ms"],
                "added_p99_ttft_ms": d["added_p99_ttft_ms"]}
    return {}


def main():
    argv = sys.argv[1:]
    extra: list[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("kind", choices=["bulk", "wf", "node", "mixed", "head"])
    ap.add_argument("--variants", default="base:", help='"label:VAR=v,VAR2=w label2: ..."')
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--paths", default="std,jumbo", help="bulk / wf: std, jumbo, tcp")
    ap.add_argument("--steps", type=int, default=150, help="bulk / wf: timed steps per run (150: ~10 s tunneled)")
    ap.add_argument("--pin", action="store_true", help="bulk / wf: disjoint CPUs per process")
    ap.add_argument("--timeline", action="store_true", help="bulk: per-thread CPU timeline")
    ap.add_argument("--timeout", type=int, default=300, help="seconds per run")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    variants = parse_variants(a.variants)
    paths = [p for p in a.paths.split(",") if p] if a.kind in ("bulk", "wf") else [""]
    results: dict[str, list[dict]] = {}
    err = open(os.path.join(a.out, "err.log"), "a")
    for rep in range(1, a.reps + 1):
        for label, env in variants:
            for path in paths:
                name = f"{label}.{path}" if path else label
                out_file = os.path.join(a.out, f"{name}_{rep}.json")
                cmd, to_stdout = command(a.kind, path, out_file, a, extra)
                t0 = time.time()
                try:
                    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, **env), stdout=subprocess.PIPE,
                                       stderr=err, text=True, timeout=a.timeout)
                except subprocess.TimeoutExpired:
                    print(f"{name} rep {rep}: timed out after {a.timeout} s", flush=True)
                    sys.exit(1)
                if r.returncode != 0:
                    print(f"{name} rep {rep}: exit {r.returncode} (see {a.out}/err.log)", flush=True)
                    sys.exit(1)
                if to_stdout:
                    with open(out_file, "w") as f:
                        f.write(r.stdout.strip().splitlines()[-1] if a.kind == "bulk" else r.stdout)
                with open(out_file) as f:
                    d = json.load(f)
                k = key_numbers(a.kind, d)
                results.setdefault(name, []).append(k)
                print(f"{name} rep {rep} ({time.time() - t0:.0f} s): " +
                      ", ".join(f"{kk} {v:.3f}" for kk, v in k.items()), flush=True)
    summary = {}
    lines = []
    for name, runs in results.items():
        row = {}
        for kk in runs[0]:
            v = sorted(r[kk] for r in runs if kk in r)
            row[kk] = {"median": round(statistics.median(v), 4), "min": round(v[0], 4), "max": round(v[-1], 4)}
        summary[name] = {"runs": len(runs), **row}
        lines.append(f"{name} n={len(runs)} " + "  ".join(
            f"{kk} {x['median']:.3f} [{x['min']:.3f}-{x['max']:.3f}]" for kk, x in row.items()))
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump({"kind": a.kind, "variants": a.variants, "reps": a.reps, "extra": extra, "rows": summary}, f, indent=1)
    with open(os.path.join(a.out, "summary.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
