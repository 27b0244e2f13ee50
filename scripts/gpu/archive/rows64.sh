# 64-row fused steps: GPU op/model tests, then the GPU endpoint through the
# tunnel (bench/bench_gpu_upstream.py). Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_rows64.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_rows64.log | tail -8
[ $rc -eq 0 ] || exit $rc
echo "== gpu upstream e2e"
timeout -k 10 900 python bench/bench_gpu_upstream.py --out gpurun_out/gpu_upstream.json > gpurun_out/gpu_upstream.log 2> gpurun_out/gpu_upstream.err
rc=$?
grep streams gpurun_out/gpu_upstream.err | cut -c1-330
exit $rc
