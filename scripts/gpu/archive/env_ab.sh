# Environment A/B of the tunnel on the MI355X host (CPU-only work): 64 x 1 MB
# echo (bulk_reps.sh VARIANTS), the mixed row and the TTFT hop breakdown next
# to 8 bulk downloads, per variant. VARS="label:ENV=v,ENV2=w label2:..."
# SKIP_BULK=1 leaves out the 64 x 1 MB part; MIXED_EXTRA passes flags to bench_mixed.py.
# Results under gpurun_out/$TAG/ (default env_ab).
set -o pipefail
TAG=${TAG:-env_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
V=""
for x in $VARS; do V="$V ${x%%:*}:build:${x#*:}"; done
if [ -z "$SKIP_BULK" ]; then
  TAG=$TAG/bulk REPS=${REPS:-3} STEPS=${STEPS:-150} VARIANTS="$V" bash scripts/gpu/archive/bulk_reps.sh || exit 1
fi
for x in $VARS; do
  l=${x%%:*}; e=${x#*:}
  env ${e//,/ } timeout -k 10 300 python bench/bench_mixed.py --seconds ${MIXED_S:-8} --reps ${MIXED_REPS:-3} \
    ${MIXED_EXTRA} --out $OUT/mixed_$l.json > /dev/null 2> $OUT/mixed_$l.err || { tail -5 $OUT/mixed_$l.err; exit 1; }
  for p in jumbo std; do
    xx=""; [ $p = std ] && xx="--no-jumbo-loopback"
    env ${e//,/ } timeout -k 10 200 python scripts/ttft_breakdown.py --requests 80 --bulk 8 --extra="$xx" \
      > $OUT/ttft_${l}_$p.json 2>> $OUT/ttft.err || { tail -5 $OUT/ttft.err; exit 1; }
    python -c "
import json; d = json.load(open('$OUT/ttft_${l}_$p.json'))
print('$l $p', [(k.split(' -> ')[1], v['p50_us'], v['p90_us']) for k, v in d['hops'].items()])"
  done
  python - $OUT/mixed_$l.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for r in d["rows"]:
    g = lambda k: (r.get(k) or {}).get("median")
    print(sys.argv[1].split("/")[-1], r["transport"], "ttft p50", g("tunneled_ttft_p50_ms"), "p99", g("tunneled_ttft_p99_ms"),
          "direct p99", g("direct_ttft_p99_ms"), "itl p99", g("tunneled_itl_p99_ms"), "bulk", g("bulk_MBps"), "ratio", g("bulk_ratio"))
PY
done
