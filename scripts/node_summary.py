"""One line per row of a bench/bench_node.py result: tunneled/direct events/s, TTFT, ITL, tunnel CPU."""
import json,sys
d = json.load(open(sys.argv[1]))
print("cpus", d["cpus"])
for r in d["rows"]:
    print(r["workers"], r["streams"], "ev/s %.0f/%.0f (%.3f)" % (r["tunneled_events_s"], r["direct_events_s"], r["events_ratio"]),
          "ttft p50 %.2f/%.2f p99 %.2f/%.2f" % (r["tunneled_p50_ttft_ms"], r["direct_p50_ttft_ms"], r["tunneled_p99_ttft_ms"], r["direct_p99_ttft_ms"]),
          "itl p99 %.2f/%.2f" % (r["tunneled_p99_itl_ms"], r["direct_p99_itl_ms"]),
          "cpu s/p %.2f/%.2f" % (r["serve_cpu_s"], r["proxy_cpu_s"]), "t %.2f" % r["seconds"], "err", r["tunneled_errors"])
