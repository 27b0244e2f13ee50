# Round 4, second host batch: cut-through A/B on the 64 x 1 MB echo (pinned),
# the 8-stream TTFT hops with the worst requests, node hop stamps at 256 /
# 1024 streams, and the mixed row.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
echo "== bulk ct A/B"; REPS=3 bash scripts/gpu/archive/r04_bulk_ab.sh > gpurun_out/r04/bulk_ct.log 2>&1; rc=$?; tail -4 gpurun_out/r04/bulk_ct.log; [ $rc -eq 0 ] || exit $rc
echo "== ttft8"; timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 --extra=--no-jumbo-loopback > gpurun_out/r04/ttft8_std2.json 2> gpurun_out/r04/ttft8_std2.err || exit 1
echo "== node"; timeout -k 10 400 python bench/bench_node.py --streams 256,1024 --seconds 10 --reps 3 --trace --out gpurun_out/r04/node_trace.json > /dev/null 2> gpurun_out/r04/node_trace.err || exit 1
echo "== mixed"; timeout -k 10 400 python bench/bench_mixed.py --seconds 10 --reps 3 --mock-threads 8 --out gpurun_out/r04/mixed.json > /dev/null 2> gpurun_out/r04/mixed.err; rc=$?; tail -2 gpurun_out/r04/mixed.err; exit $rc
