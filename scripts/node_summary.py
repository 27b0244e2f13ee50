"""One line per row of a bench/bench_node.py result: tunneled/direct events/s, TTFT, ITL, tunnel CPU.

Rows from repeated runs (--reps) carry {median, min, max} per field: printed
as median [min-max]."""
import json
import sys


def f(v, fmt="%.2f"):
    if isinstance(v, dict):
        return (fmt + " [" + fmt + "-" + fmt + "]") % (v["median"], v["min"], v["max"])
    return fmt % v if v is not None else "-"


d = json.load(open(sys.argv[1]))
print("cpus", d["cpus"])
for r in d["rows"]:
    print(r["workers"], r["streams"], "ev/s", f(r["tunneled_events_s"], "%.0f"), "/", f(r["direct_events_s"], "%.0f"),
          "ratio", f(r["events_ratio"], "%.3f"),
          "| ttft added p50", f(r.get("added_p50_ttft_ms")), "p99 tunneled", f(r.get("tunneled_p99_ttft_ms")),
          "direct", f(r.get("direct_p99_ttft_ms")),
          "| itl p99", f(r.get("tunneled_p99_itl_ms")), "/", f(r.get("direct_p99_itl_ms")),
          "| cpu s/p", f(r.get("serve_cpu_s")), "/", f(r.get("proxy_cpu_s")), "| err", r.get("errors", r.get("tunneled_errors")))
