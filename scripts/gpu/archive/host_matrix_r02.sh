# Round-2 host-side matrix on the MI355X box (CPU-only work; the tunnel has no
# GPU compute): headline bench, mixed SSE+bulk HOL row, 64x1MB bulk on the
# jumbo and standard-MTU paths, node topology (1 serve over 8 upstreams).
# Results under gpurun_out/r02/.
set -o pipefail
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
echo "nproc=$(nproc)"
echo "== headline"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --out gpurun_out/r02/bench.json > gpurun_out/r02/bench.log 2>&1 || { tail -5 gpurun_out/r02/bench.log; exit 1; }
cut -c1-400 gpurun_out/r02/bench.json
echo "== mixed"; timeout -k 10 400 python bench/bench_mixed.py --out gpurun_out/r02/mixed.json > /dev/null 2> gpurun_out/r02/mixed.err || { tail -5 gpurun_out/r02/mixed.err; exit 1; }
tail -3 gpurun_out/r02/mixed.err | cut -c1-600
echo "== bulk"
for i in 1 2 3; do
  for x in jumbo std; do
    if [ $x = std ]; then e=--extra=--no-jumbo-loopback; else e=; fi
    timeout -k 10 300 python bench/profile_bulk.py --steps 10 $e > gpurun_out/r02/bulk_${x}_$i.json 2>> gpurun_out/r02/bulk.err || { tail -5 gpurun_out/r02/bulk.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r02/bulk_${x}_$i.json')); print('$x', $i, d['path'], round(d['tunneled_req_s'],1), round(d['direct_req_s'],1), d['cpu_s_incl_warmup'])"
  done
done
echo "== node"; timeout -k 10 400 python bench/bench_node.py --streams 256,512,1024 --workers 0,auto --steps 12 --tokens 64 --lg-threads 4 --out gpurun_out/r02/node.json > /dev/null 2> gpurun_out/r02/node.err || { tail -5 gpurun_out/r02/node.err; exit 1; }
python scripts/node_summary.py gpurun_out/r02/node.json
