# 64 x 1 MB POST echoed (BASELINE config #3) on the MI355X host: REPS
# alternating runs of each path (jumbo = same-host 16 KiB SCTP packets,
# std = 1200-byte MTU, the path a reference peer negotiates), STEPS timed
# steps each. JSON per run under gpurun_out/$TAG/, one summary line per run.
set -o pipefail
TAG=${TAG:-bulk_reps}
REPS=${REPS:-5}
STEPS=${STEPS:-30}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for i in $(seq 1 $REPS); do
  for p in jumbo std; do
    x="${EXTRA}"
    [ $p = std ] && x="$x --no-jumbo-loopback"
    timeout -k 10 300 python bench/profile_bulk.py --steps $STEPS --extra="$x" > gpurun_out/$TAG/${p}_$i.json 2>> gpurun_out/$TAG/err.log || { tail -5 gpurun_out/$TAG/err.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$TAG/${p}_$i.json')); print('$p $i', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), round(d['tunneled_req_s']/d['direct_req_s'],3), d['cpu_s_incl_warmup'], d['wall_s_incl_warmup'])"
  done
done
