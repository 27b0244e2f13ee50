# Round 4, third host batch (after zero-copy reassembly and the client fixes):
# window A/B on the 1200-byte 64 x 1 MB echo, a per-thread CPU profile of that
# row, and the pinned waterfall on both MTUs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
echo "== window A/B"; REPS=3 bash scripts/gpu/archive/r04_window_ab.sh > gpurun_out/r04/window_ab.log 2>&1; rc=$?; tail -5 gpurun_out/r04/window_ab.log; [ $rc -eq 0 ] || exit $rc
echo "== threads"; PATHS=std STEPS=100 timeout -k 10 300 bash scripts/gpu/archive/bulk_threads.sh > gpurun_out/r04/threads.log 2>&1; rc=$?; tail -4 gpurun_out/r04/threads.log; [ $rc -eq 0 ] || exit $rc
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 60 --pin $x > gpurun_out/r04/wf3_${m}.json 2> gpurun_out/r04/wf3_${m}.err || exit 1
done
