set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== decode variants"
for args in "" "--unfused" "--eager" "--batch 1" "--batch 16" "--config small --batch 8" "--config small --batch 8 --unfused"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 200 $args >> gpurun_out/decode_variants.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_variants.log
done
cd /tmp
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py "$@" > $R/gpurun_out/rocprof_$name.log 2>&1 || return 1
  python3 $R/scripts/rocprof_summary.py $(find /tmp/prof_$name -name '*.db' | head -1) > $R/gpurun_out/kernels_$name.md || return 1
  head -9 $R/gpurun_out/kernels_$name.md | tail -5
  rm -rf /tmp/prof_$name
}
for ctx in 64 1024; do echo "== graph ctx $ctx"; prof graph_ctx$ctx --steps 50 --ctx $ctx || exit 1; done
echo "== unfused ctx 1024"; prof unfused_ctx1024 --steps 50 --ctx 1024 --unfused || exit 1
