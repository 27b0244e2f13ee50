set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== decode variants"
for args in "" "--unfused" "--eager" "--eager --unfused" "--batch 1" "--batch 1 --unfused" "--batch 16" "--config small --batch 8" "--config small --batch 8 --unfused"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 200 $args >> gpurun_out/decode_variants.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_variants.log
done
echo "== rocprof fused graph"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fused -o fused -- python3 $R/scripts/profile_decode.py --steps 50 > $R/gpurun_out/rocprof_fused.log 2>&1; rc=$?; cd $R; [ $rc -eq 0 ] || { tail -20 gpurun_out/rocprof_fused.log; exit $rc; }
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1; tail -1 gpurun_out/smoke.log
echo "== matrix"; timeout -k 10 900 python bench/bench_tunnel.py --steps 6 --idle-s 30 --busy-poll 50,500 --out gpurun_out/matrix.json > gpurun_out/matrix.log 2> gpurun_out/matrix.err; rc=$?; tail -4 gpurun_out/matrix.err | cut -c1-250; exit $rc
