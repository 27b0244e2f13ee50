# Sampling profiles of the 64 x 1 MB WebRTC bulk row on the MI355X host, single
# reactor vs worker threads. Reports under gpurun_out/bulk_prof/.
set -o pipefail
mkdir -p gpurun_out/bulk_prof
export TMPDIR=/tmp
for w in 0 auto; do
  rm -rf /tmp/bp_$w
  timeout -k 10 300 python bench/profile_bulk.py --steps ${STEPS:-30} --extra=--workers=$w --profile-dir /tmp/bp_$w > gpurun_out/bulk_prof/w$w.json 2>> gpurun_out/bulk_prof/err.log || { tail -5 gpurun_out/bulk_prof/err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bulk_prof/w$w.json')); print('w=$w', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), d['cpu_s_incl_warmup'])"
  for f in /tmp/bp_$w/*.prof; do
    b=$(basename $f .prof)
    python scripts/profile_report.py $f --top 30 > gpurun_out/bulk_prof/w${w}_$b.txt
    python scripts/profile_report.py $f --top 30 --thread 0 > gpurun_out/bulk_prof/w${w}_$b.main.txt
  done
done
