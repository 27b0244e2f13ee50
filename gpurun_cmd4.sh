set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== matrix"; timeout -k 10 900 python bench/bench_tunnel.py --steps 6 --idle-s 30 --out gpurun_out/matrix.json > gpurun_out/matrix.log 2> gpurun_out/matrix.err; rc=$?; tail -4 gpurun_out/matrix.err; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400; exit $rc
