# Round 4, thirteenth host batch: is the single-threaded echo upstream the
# bound of the 64 x 1 MB row? (tunneled run: mock at 80-95 % of a core; the
# serve's store-and-forward hands it each body in one burst.) A/B of a 1- and a
# 2-thread mock (its 2 pinned CPUs), both MTUs, with the per-thread timeline.
# First the node row's packet / batch / reader counters at 256 and 1024 streams.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/node13
echo "== node counters"; timeout -k 10 300 python bench/bench_node.py --streams 256,1024 --seconds 10 --reps 1 --metrics --out gpurun_out/r04/node13/node.json > /dev/null 2> gpurun_out/r04/node13/err.log || { tail -5 gpurun_out/r04/node13/err.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04/node13/node.json"))
for r in d["runs"]:
    print(r["streams"], "p50 +%.3f p99 %.2f/%.2f" % (r["added_p50_ttft_ms"], r["tunneled_p99_ttft_ms"], r["direct_p99_ttft_ms"]), "events/s %.0f" % r["tunneled_events_s"])
    print("  serve", r.get("serve_counters")); print("  proxy", r.get("proxy_counters"))
PY
echo "== mock threads A/B"; TAG=r04/mock_ab PIN=1 TIMELINE=1 REPS=3 PATHS="std jumbo" \
  VARIANTS="m1:build:P2PT_MOCK_THREADS=1 m2:build:P2PT_MOCK_THREADS=2" \
  timeout -k 10 900 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/mock_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/mock_ab.log; exit $rc
