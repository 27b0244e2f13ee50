# Correctness (GPU model/op tests) then decode-step timing and a kernel table
# for the tiny and small configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== gpu model/op tests"; timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_decode.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu_decode.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu_decode.log | head -20; exit $rc; }
: > gpurun_out/decode_timing.log
for args in "--batch 1" "--batch 8" "--batch 16" "--config small --batch 1" "--config small --batch 8" "--config small --batch 16"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 200 $args >> gpurun_out/decode_timing.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_timing.log
done
cd /tmp
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py "$@" > $R/gpurun_out/rocprof_$name.log 2>&1 || return 1
  python3 $R/scripts/rocprof_summary.py $(find /tmp/prof_$name -name '*.db' | head -1) > $R/gpurun_out/kernels_$name.md || return 1
  head -12 $R/gpurun_out/kernels_$name.md
  rm -rf /tmp/prof_$name
}
echo "== small b8"; prof small_b8 --config small --batch 8 --steps 50 --ctx 1024 || exit 1
