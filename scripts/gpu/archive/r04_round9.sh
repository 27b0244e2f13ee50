# Round 4, ninth host batch: small flushes leave a loaded association loop
# (TUNNEL_INLINE_LOAD_PCT, default 50: seal + sendmmsg on the TX lanes once the
# loop is >= 50 % busy; 100 = always inline as before, 0 = never inline), A/B
# on the node row at 1024 and 256 streams (plus 8 workers at 1024), then the
# 64 x 1 MB echo (pinned, both MTUs) and the headline.
set -o pipefail
export TMPDIR=/tmp
echo "== node 1024"; STREAMS=1024 REPS=2 VARIANTS="dflt: inl100:TUNNEL_INLINE_LOAD_PCT=100 inl0:TUNNEL_INLINE_LOAD_PCT=0 w8:TUNNEL_WORKERS=8" \
  timeout -k 10 600 bash scripts/gpu/archive/node_env_ab.sh > gpurun_out/r04_node1024.log 2>&1; rc=$?; cat gpurun_out/r04_node1024.log | grep -v "^{" | tail -8; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r04/node9 && mv gpurun_out/node_ab gpurun_out/r04/node9/s1024
echo "== node 256"; STREAMS=256 REPS=2 VARIANTS="dflt: inl100:TUNNEL_INLINE_LOAD_PCT=100" \
  timeout -k 10 300 bash scripts/gpu/archive/node_env_ab.sh > gpurun_out/r04_node256.log 2>&1; rc=$?; cat gpurun_out/r04_node256.log | grep -v "^{" | tail -4; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/node_ab gpurun_out/r04/node9/s256
echo "== bulk"; TAG=r04/inl_ab PIN=1 REPS=2 PATHS="std jumbo" VARIANTS="dflt:build: inl100:build:TUNNEL_INLINE_LOAD_PCT=100" \
  timeout -k 10 600 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/inl_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/inl_ab.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r04/head9
timeout -k 10 200 python bench.py --steps 10 --curve "" --no-jumbo-extra --out gpurun_out/r04/head9/b_1.json > /dev/null 2>> gpurun_out/r04/head9/err.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04/head9/b_1.json')); print('bench', d['value'], d['added_p50_ttft_ms'], d['added_p99_ttft_ms'], d['step_max_ttft_ms_rank0'])"
