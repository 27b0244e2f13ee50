# Round 4, eighth host batch: the headline with the GPU runtime brought up
# before the tunnel (per-step max TTFT), the pinned 64 x 1 MB waterfall on both
# MTUs with the seal -> send TX pipeline, and the node row at 256 / 1024
# streams with the job's cgroup CPU use and quota throttling per leg.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/head_init gpurun_out/r04/wf8 gpurun_out/r04/node8
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --curve "" --no-jumbo-extra --out gpurun_out/r04/head_init/b_$i.json > /dev/null 2>> gpurun_out/r04/head_init/err.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04/head_init/b_$i.json')); print('bench', d['value'], d['added_p50_ttft_ms'], d['added_p99_ttft_ms'], d['step_max_ttft_ms_rank0'])"
done
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 60 --pin $x > gpurun_out/r04/wf8/$m.json 2> gpurun_out/r04/wf8/$m.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04/wf8/$m.json')); print(d['tunneled'], d['direct'], round(d['ratio'],3)); print(d['step_waterfall_ms_median'])"
done
echo "== node"; timeout -k 10 400 python bench/bench_node.py --streams 256,1024 --seconds 10 --reps 3 --out gpurun_out/r04/node8/node.json > /dev/null 2> gpurun_out/r04/node8/err.log || { tail -5 gpurun_out/r04/node8/err.log; exit 1; }
python - <<'EOF'
import json
d = json.load(open("gpurun_out/r04/node8/node.json"))
for r in d["runs"]:
    print(r["streams"], r["rep"], "p50 +%.3f" % r["added_p50_ttft_ms"], "p99 %.2f/%.2f" % (r["tunneled_p99_ttft_ms"], r["direct_p99_ttft_ms"]),
          "cg tun", r.get("tunneled_cgroup"), "cg dir", r.get("direct_cgroup"))
EOF
