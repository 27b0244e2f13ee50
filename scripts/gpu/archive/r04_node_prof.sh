# Round 4: where the 1024-stream node row spends its CPU (sampling profile of
# serve and proxy, association thread and workers separately), 10 s run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/node_prof
mkdir -p $O
TUNNEL_PROFILE_HZ=2000 timeout -k 10 300 python bench/bench_node.py --streams 1024 --seconds 10 --reps 1 \
  --profile-dir $O --out $O/node.json > /dev/null 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
for f in $O/*.prof; do
  python scripts/profile_report.py $f --top 30 > ${f%.prof}.txt
  python scripts/profile_report.py $f --top 30 --thread 0 > ${f%.prof}.main.txt
  python scripts/profile_report.py $f --top 30 --thread workers > ${f%.prof}.workers.txt
done
python -c "import json; d=json.load(open('$O/node.json')); r=d['runs'][0]; print({k: r[k] for k in ('events_ratio','tunneled_p99_ttft_ms','direct_p99_ttft_ms','serve_cpu_s','proxy_cpu_s')})"
head -3 $O/*.txt
