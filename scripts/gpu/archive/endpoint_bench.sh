# GPU endpoint through the tunnel: max batch 16 at 1/8/16 streams, then max
# batch 64 at 16/32/64 streams. Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench/bench_gpu_upstream.py --out gpurun_out/gpu_upstream.json > gpurun_out/gpu_upstream.log 2> gpurun_out/gpu_upstream.err || exit $?
timeout -k 10 600 python bench/bench_gpu_upstream.py --max-batch 64 --streams 16,32,64 --out gpurun_out/gpu_upstream_mb64.json > gpurun_out/gpu_upstream_mb64.log 2> gpurun_out/gpu_upstream_mb64.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/gpu_upstream.json", "gpurun_out/gpu_upstream_mb64.json"):
    for r in json.load(open(f))["rows"]:
        print(f[-12:], r["streams"], "tok/s tun", round(r["tunneled_tok_s"]), "dir", round(r["direct_tok_s"]),
              "ttft", r["tunneled_p50_ttft_ms"], r["direct_p50_ttft_ms"], "steps", r["direct_step_ms"][:2])
PY
