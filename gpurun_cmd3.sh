set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== gpu tests"; timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== decode eager"; timeout -k 10 120 python scripts/profile_decode.py --steps 100 --eager > gpurun_out/decode_eager.log 2>&1; tail -1 gpurun_out/decode_eager.log
echo "== decode graph"; timeout -k 10 120 python scripts/profile_decode.py --steps 100 > gpurun_out/decode_graph.log 2>&1; tail -1 gpurun_out/decode_graph.log
echo "== rocprof"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_decode_graph -o decode -- python3 $GRAFT_REPO_ROOT/scripts/profile_decode.py --steps 50 > $GRAFT_REPO_ROOT/gpurun_out/rocprof.log 2>&1; rc=$?; tail -1 $GRAFT_REPO_ROOT/gpurun_out/rocprof.log; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || exit $rc
echo "== matrix"; timeout -k 10 900 python bench/bench_tunnel.py --steps 6 --idle-s 30 --out gpurun_out/matrix.json > gpurun_out/matrix.log 2> gpurun_out/matrix.err; rc=$?; tail -3 gpurun_out/matrix.err; exit $rc
