# Round 4, fourteenth host batch: flush coalescing on a busy association loop
# (TUNNEL_COALESCE_US: while the loop is >= 50 % busy and less than a packet
# is queued, the SCTP flush waits up to that long after the previous one), on
# the node row. At 1024 streams the serve sent 105 k packets/s of ~7 tokens,
# one sendmmsg each (profiles/r04/node13). Then cut-through uploads again (the
# 1-thread echo upstream bounds the direct leg; store-and-forward leaves it idle).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/node14
echo "== node 1024"; NODE_EXTRA=--metrics STREAMS=1024 REPS=3 VARIANTS="off: c50:TUNNEL_COALESCE_US=50 c200:TUNNEL_COALESCE_US=200" \
  timeout -k 10 700 bash scripts/gpu/archive/node_env_ab.sh > gpurun_out/r04/node14/s1024.log 2>&1; rc=$?; grep -v "^{\\|^ \\|^}\\|^\\]" gpurun_out/r04/node14/s1024.log | tail -9; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/node_ab gpurun_out/r04/node14/s1024
echo "== node 256"; NODE_EXTRA=--metrics STREAMS=256 REPS=2 VARIANTS="off: c50:TUNNEL_COALESCE_US=50 c200:TUNNEL_COALESCE_US=200" \
  timeout -k 10 500 bash scripts/gpu/archive/node_env_ab.sh > gpurun_out/r04/node14/s256.log 2>&1; rc=$?; grep -v "^{\\|^ \\|^}\\|^\\]" gpurun_out/r04/node14/s256.log | tail -6; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/node_ab gpurun_out/r04/node14/s256
echo "== cut-through A/B"; TAG=r04/ct14 PIN=1 REPS=2 PATHS="std jumbo" \
  VARIANTS="sf:build: ct:build:TUNNEL_STREAM_BODY_THRESHOLD=65536" \
  timeout -k 10 600 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/r04/ct14.log 2>&1; rc=$?; tail -4 gpurun_out/r04/ct14.log; [ $rc -eq 0 ] || exit $rc
echo "== wf std (credit / flow wait stamps)"; mkdir -p gpurun_out/r04/wf14
timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 100 --pin --extra=--no-jumbo-loopback > gpurun_out/r04/wf14/std.json 2> gpurun_out/r04/wf14/std.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/r04/wf14/std.json')); print(d['tunneled'], d['direct'], round(d['ratio'],3))
for s in d['slowest_steps']: print(s['step end at the client'], s['new connections'], s['straggler'])"
