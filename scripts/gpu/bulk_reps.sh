# 64 x 1 MB POST echoed (BASELINE config #3) on the MI355X host: REPS
# alternating runs of each path (jumbo = same-host 16 KiB SCTP packets,
# std = 1200-byte MTU, the path a reference peer negotiates, tcp = the TCP
# transport: the HTTP + framing machinery without DTLS/SCTP), STEPS timed
# steps each (150 steps: ~10 s tunneled + the direct run of the same load).
# JSON per run under gpurun_out/$TAG/; summary: python scripts/bulk_summary.py DIR.
set -o pipefail
TAG=${TAG:-bulk_reps}
REPS=${REPS:-5}
STEPS=${STEPS:-150}
PATHS=${PATHS:-jumbo std}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
# BUILDS="build build-r2": interleave builds of the tunnel (bin dirs) for an
# A/B on one box; file names then carry the build: <build>.<path>_<rep>.json.
BUILDS=${BUILDS:-build}
for i in $(seq 1 $REPS); do
  for b in $BUILDS; do
    for p in $PATHS; do
      x="${EXTRA}"
      t=webrtc
      [ $p = std ] && x="$x --no-jumbo-loopback"
      [ $p = tcp ] && t=tcp
      n=$p
      [ "$BUILDS" != build ] && n=$b.$p
      P2PT_BIN_DIR=$PWD/$b/bin timeout -k 10 300 python bench/profile_bulk.py --transport $t --steps $STEPS --extra="$x" > gpurun_out/$TAG/${n}_$i.json 2>> gpurun_out/$TAG/err.log || { tail -5 gpurun_out/$TAG/err.log; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/$TAG/${n}_$i.json')); print('$n $i', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), round(d['tunneled_req_s']/d['direct_req_s'],3), d['cpu_s_incl_warmup'], d['wall_s_incl_warmup'], flush=True)"
    done
  done
done
python scripts/bulk_summary.py gpurun_out/$TAG | tee gpurun_out/$TAG/summary.txt
