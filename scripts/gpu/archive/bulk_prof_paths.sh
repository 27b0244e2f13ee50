# Sampling profiles of the 64 x 1 MB echo on the MI355X host, on both paths
# (jumbo and the 1200-byte MTU a reference peer negotiates). Per-thread
# reports under gpurun_out/$TAG/ (thread 0 = association thread, 90/91 = DTLS
# TX/RX lanes, 1.. = HTTP workers).
set -o pipefail
TAG=${TAG:-bulk_prof_paths}
STEPS=${STEPS:-30}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for p in jumbo std; do
  x="${EXTRA}"
  [ $p = std ] && x="$x --no-jumbo-loopback"
  rm -rf /tmp/bp_$p
  timeout -k 10 300 python bench/profile_bulk.py --steps $STEPS --extra="$x" --profile-dir /tmp/bp_$p > gpurun_out/$TAG/$p.json 2>> gpurun_out/$TAG/err.log || { tail -5 gpurun_out/$TAG/err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/$p.json')); print('$p', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), d['cpu_s_incl_warmup'])"
  for f in /tmp/bp_$p/*.prof; do
    b=$(basename $f .prof)
    python scripts/profile_report.py $f --top 30 > gpurun_out/$TAG/${p}_$b.txt
    python scripts/profile_report.py $f --top 30 --thread 0 > gpurun_out/$TAG/${p}_$b.main.txt
  done
done
