# Round 4, seventh host batch: the TX lane split into seal -> send stages
# (A/B against the single lane, TUNNEL_TX_PIPELINE=0) with auto workers from
# the pinned CPU count, on the 64 x 1 MB echo (both MTUs, pinned, per-thread
# timeline); the headline with its warm-up on the timed connections (per-step
# max TTFT); the mixed row (8-thread mock).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/head_hold
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --curve "" --no-jumbo-extra --out gpurun_out/r04/head_hold/b_$i.json > /dev/null 2>> gpurun_out/r04/head_hold/err.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04/head_hold/b_$i.json')); print('bench', d['value'], d['added_p50_ttft_ms'], d['added_p99_ttft_ms'], d['step_max_ttft_ms_rank0'])"
done
echo "== pipeline A/B + timeline"; TAG=r04/pipe_ab PIN=1 TIMELINE=1 REPS=2 PATHS="std jumbo" \
  VARIANTS="pipe:build: lane:build:TUNNEL_TX_PIPELINE=0" \
  timeout -k 10 700 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/pipe_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/pipe_ab.log; [ $rc -eq 0 ] || exit $rc
echo "== mixed"; timeout -k 10 300 python bench/bench_mixed.py --seconds 10 --reps 2 --mock-threads 8 --out gpurun_out/r04/mixed7.json > /dev/null 2> gpurun_out/r04/mixed7.err; rc=$?; tail -2 gpurun_out/r04/mixed7.err; exit $rc
