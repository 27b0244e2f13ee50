# A/B of the 64 x 1 MB WebRTC bulk row on the MI355X host: worker threads
# (0 / auto) x "flow" extension (on / off via TUNNEL_FEATURES), alternating.
set -o pipefail
mkdir -p gpurun_out/bulk_ab
export TMPDIR=/tmp
for i in 1 2 3; do
  for w in 0 auto; do
    for f in flow noflow; do
      if [ $f = noflow ]; then export TUNNEL_FEATURES=sse,cancel; else unset TUNNEL_FEATURES; fi
      timeout -k 10 300 python bench/profile_bulk.py --steps 10 --extra=--workers=$w ${EXTRA:+--extra="$EXTRA"} > gpurun_out/bulk_ab/w${w}_${f}_$i.json 2>> gpurun_out/bulk_ab/err.log || { tail -5 gpurun_out/bulk_ab/err.log; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/bulk_ab/w${w}_${f}_$i.json')); print('w=$w $f $i', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), d['cpu_s_incl_warmup'])"
    done
  done
done
