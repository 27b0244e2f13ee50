"""Summarise a rocprofv3 rocpd database (kernel-trace) into a markdown table.

    python scripts/rocprof_summary.py gpurun_out/prof_decode/decode_results.db > profiles/decode_kernels.md
"""
import sqlite3
import sys


def short(name: str) -> str:
    if name.startswith("Cijk_"):
        return "hipBLASLt GEMM " + name.split("_MT")[1].split("_")[0] if "_MT" in name else "hipBLASLt GEMM"
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    if "(" in name:
        name = name.split("(")[0]
    return name[:80]


def main(path):
    db = sqlite3.connect(path)
    rows = list(db.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    print(f"Source: `{path}` (rocprofv3 --kernel-trace --stats; durations in µs)\n")
    print("| kernel | calls | total µs | avg µs | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in rows:
        print(f"| {short(name)} | {calls} | {tot:.1f} | {avg:.2f} | {pct:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
