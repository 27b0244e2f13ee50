# Node row (1 serve over 8 mocks, 1 ms tokens) A/B of tunnel environments at
# one stream count, interleaved per repetition. VARIANTS="label:VAR=v,VAR2=w ...".
#   STREAMS=256 REPS=3 VARIANTS="dflt: old:TUNNEL_SCHED_BYPASS=0" bash scripts/gpu/archive/node_env_ab.sh
# NODE_EXTRA="--metrics" adds bench_node flags (packet / batch counters per run).
set -o pipefail
mkdir -p gpurun_out/node_ab
export TMPDIR=/tmp
for i in $(seq 1 ${REPS:-3}); do
  for v in $VARIANTS; do
    label=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 200 python bench/bench_node.py --streams ${STREAMS:-256} --workers auto --seconds 10 --reps 1 \
      --tokens 64 --lg-threads 4 ${NODE_EXTRA} --out gpurun_out/node_ab/${label}_$i.json 2>> gpurun_out/node_ab/err.log || exit 1
    python3 -c "
import json,sys; r=json.load(open('gpurun_out/node_ab/${label}_$i.json'))['runs'][0]
sc = r.get('serve_counters') or {}
print('$label', $i, r['streams'], round(r['events_ratio'],3), 'ttft p50', r['tunneled_p50_ttft_ms'], r['direct_p50_ttft_ms'], 'p99', r['tunneled_p99_ttft_ms'], r['direct_p99_ttft_ms'], 'serve pkts', sc.get('sctp_packets_sent'), 'cpu', r['serve_cpu_s'], r['proxy_cpu_s'])" | tee -a gpurun_out/node_ab/summary.txt
  done
done
