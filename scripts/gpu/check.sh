# Round-end rehearsal on a 1-GPU MI355X box (run via gpurun from the repo root):
# GPU tests, smoke(), headline bench. Build in-tree on the CPU first
# (python -c "import __graft_entry__ as g; g.build()"); the .so files travel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-600; exit $rc
