# GPU inference endpoint after the asyncio front-end: GPU model tests, then the
# end-to-end tunnel-in-front-of-the-GPU-endpoint benchmark. Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu model tests"; timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_model.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_model.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu upstream e2e"; timeout -k 10 900 python bench/bench_gpu_upstream.py --out gpurun_out/gpu_upstream.json > gpurun_out/gpu_upstream.log 2> gpurun_out/gpu_upstream.err; rc=$?; tail -3 gpurun_out/gpu_upstream.err | cut -c1-300; python - <<'PY'
import json
d = json.load(open("gpurun_out/gpu_upstream.json"))
for r in d["rows"]:
    print(r["streams"], "tok/s tunneled", r["tunneled_tok_s"], "direct", r["direct_tok_s"], "ttft p50", r["tunneled_p50_ttft_ms"], r["direct_p50_ttft_ms"], "errors", r["errors"])
PY
exit $rc
