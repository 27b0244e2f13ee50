# 64 x 1 MB echo over the TCP transport (no DTLS/SCTP: the HTTP + framing
# machinery's own ceiling on this host), REPS runs, beside the WebRTC rows.
set -o pipefail
TAG=${TAG:-bulk_tcp}
REPS=${REPS:-3}
STEPS=${STEPS:-30}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for i in $(seq 1 $REPS); do
  timeout -k 10 300 python bench/profile_bulk.py --transport tcp --steps $STEPS > gpurun_out/$TAG/tcp_$i.json 2>> gpurun_out/$TAG/err.log || { tail -5 gpurun_out/$TAG/err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/tcp_$i.json')); print('tcp $i', round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), round(d['tunneled_req_s']/d['direct_req_s'],3), d['cpu_s_incl_warmup'])"
done
