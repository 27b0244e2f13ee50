set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu upstream e2e"; timeout -k 10 900 python bench/bench_gpu_upstream.py --out gpurun_out/gpu_upstream.json > gpurun_out/gpu_upstream.log 2> gpurun_out/gpu_upstream.err; rc=$?; tail -5 gpurun_out/gpu_upstream.err | cut -c1-400; exit $rc
