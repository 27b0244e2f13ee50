# Round 4, sixth host batch: which thread saturates in the 64 x 1 MB echo
# (per-thread 2 ms utilisation timeline), with the per-stream flow window A/B
# (256 KiB default vs 1 MiB), both MTUs, pinned; then the 1024-stream node
# profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/head_steps
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --curve "" --no-jumbo-extra --out gpurun_out/r04/head_steps/b_$i.json > /dev/null 2>> gpurun_out/r04/head_steps/err.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04/head_steps/b_$i.json')); print('bench', d['value'], d['added_p50_ttft_ms'], d['added_p99_ttft_ms'], d['step_max_ttft_ms_rank0'])"
done
timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 --extra=--no-jumbo-loopback > gpurun_out/r04/head_steps/ttft8.json 2>> gpurun_out/r04/head_steps/err.log || exit 1
echo "== flow A/B + timeline"; TAG=r04/flow_ab PIN=1 TIMELINE=1 REPS=2 PATHS="std jumbo" \
  VARIANTS="w256:build:TUNNEL_SCTP_CHAIN=0 w1m:build:TUNNEL_SCTP_CHAIN=0,TUNNEL_FLOW_WINDOW_KB=1024" \
  timeout -k 10 900 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/flow_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/flow_ab.log; [ $rc -eq 0 ] || exit $rc
echo "== node prof"; timeout -k 10 400 bash scripts/gpu/archive/r04_node_prof.sh > gpurun_out/r04/node_prof.log 2>&1; rc=$?; tail -3 gpurun_out/r04/node_prof.log; exit $rc
