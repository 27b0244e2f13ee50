# 64 x 1 MB POST echoed (BASELINE config #3) on the MI355X host: REPS
# alternating runs of each path (jumbo = same-host 16 KiB SCTP packets,
# std = 1200-byte MTU, the path a reference peer negotiates, tcp = the TCP
# transport: the HTTP + framing machinery without DTLS/SCTP), STEPS timed
# steps each (150 steps: ~10 s tunneled + the direct run of the same load).
# JSON per run under gpurun_out/$TAG/; summary: python scripts/bulk_summary.py DIR.
# PIN=1: loadgen / mock / serve / proxy on disjoint CPUs (utils/pinning.py).
# TIMELINE=1: per-thread CPU utilisation in 2 ms intervals (which stage saturates).
# P2PT_MOCK_THREADS=n (in VARIANTS too): reactor threads of the echo upstream (default 1).
set -o pipefail
TAG=${TAG:-bulk_reps}
REPS=${REPS:-5}
STEPS=${STEPS:-150}
PATHS=${PATHS:-jumbo std}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
# A/B on one box, interleaved: BUILDS="build build-ab" (bin dirs of two builds
# of the tunnel) or VARIANTS="label:bindir:VAR=v,VAR2=w ..." (same or other
# builds under different environments). File names then carry the label:
# <label>.<path>_<rep>.json.
BUILDS=${BUILDS:-build}
if [ -z "$VARIANTS" ]; then
  for b in $BUILDS; do VARIANTS="$VARIANTS $b:$b:"; done
fi
nvar=$(echo $VARIANTS | wc -w)
for i in $(seq 1 $REPS); do
  for v in $VARIANTS; do
    IFS=: read -r label bindir envs <<< "$v"
    for p in $PATHS; do
      x="${EXTRA}"
      t=webrtc
      [ $p = std ] && x="$x --no-jumbo-loopback"
      [ $p = tcp ] && t=tcp
      n=$p
      [ $nvar -gt 1 ] && n=$label.$p
      env ${envs//,/ } P2PT_BIN_DIR=$PWD/$bindir/bin timeout -k 10 300 python bench/profile_bulk.py --transport $t --steps $STEPS --extra="$x" ${PIN:+--pin} ${TIMELINE:+--timeline} > gpurun_out/$TAG/${n}_$i.json 2>> gpurun_out/$TAG/err.log || { tail -5 gpurun_out/$TAG/err.log; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/$TAG/${n}_$i.json')); print('$n $i', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), round(d['tunneled_req_s']/d['direct_req_s'],3), d['cpu_s_incl_warmup'], d.get('loss'), flush=True)"
    done
  done
done
python scripts/bulk_summary.py gpurun_out/$TAG | tee gpurun_out/$TAG/summary.txt
