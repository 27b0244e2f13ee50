# Round 4, fourth host batch: chained reassembly vs one copy, and a capped
# reader burst, on the 1200-byte 64 x 1 MB echo (pinned), then a per-thread
# CPU profile of the row at HEAD and the pinned waterfall on both MTUs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
echo "== chain A/B"; TAG=r04/chain_ab PIN=1 REPS=3 PATHS=std \
  VARIANTS="chain:build: copy:build:TUNNEL_SCTP_CHAIN=0 burst:build:TUNNEL_RX_BURST_KB=256" \
  timeout -k 10 900 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/chain_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/chain_ab.log; [ $rc -eq 0 ] || exit $rc
echo "== threads"; PATHS=std STEPS=100 timeout -k 10 300 bash scripts/gpu/archive/bulk_threads.sh > gpurun_out/r04/threads4.log 2>&1; rc=$?; tail -3 gpurun_out/r04/threads4.log; [ $rc -eq 0 ] || exit $rc
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 60 --pin $x > gpurun_out/r04/wf4_${m}.json 2> gpurun_out/r04/wf4_${m}.err || exit 1
done
