# BASELINE matrix rows on the MI355X host, jumbo and standard 1200-byte MTU
# WebRTC paths back to back (CPU-only tunnel work). Results: gpurun_out/mtu/.
set -o pipefail
mkdir -p gpurun_out/mtu
export TMPDIR=/tmp
for m in jumbo std; do
  f=""; [ $m = std ] && f=--std-mtu
  echo "== $m"; timeout -k 10 600 python bench/bench_tunnel.py --quick --idle-s 10 --steps 6 $f --out gpurun_out/mtu/matrix_$m.json > /dev/null 2> gpurun_out/mtu/matrix_$m.err || { tail -5 gpurun_out/mtu/matrix_$m.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/mtu/matrix_$m.json'))
for r in d['sse']: print(r['transport'], r['path'][-8:], r['streams'], round(r['tunneled_req_s'],2), round(r['direct_req_s'],2), round(r['added_p50_ttft_ms'],3), r['errors'])
for r in d['post_64x1MB']: print('post', r['transport'], round(r['tunneled_req_s'],1), round(r['direct_req_s'],1))
r=d['idle_burst']; print('idle', r['transport'], r['tunneled_req_s'], round(r['added_p50_ttft_ms'],3))
"
done
