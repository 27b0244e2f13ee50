# Round 4, fifth host batch: GPU tests + smoke (HIP tree changed: k_block
# removed, V=32000 sampler cases, stop sequences), then the headline's tail:
# bench.py with the association thread taking the first 16 streams (default)
# against every stream on a worker (TUNNEL_INLINE_STREAMS=0), alternating, and
# the 8-stream hop breakdown of both (warm-up step excluded).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/head_ab
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r04/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r04/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in inline0 default; do
    e=""; [ $v = inline0 ] && e="TUNNEL_INLINE_STREAMS=0"
    env $e timeout -k 10 200 python bench.py --steps 10 --curve "" --no-jumbo-extra --out gpurun_out/r04/head_ab/${v}_$i.json > /dev/null 2>> gpurun_out/r04/head_ab/err.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04/head_ab/${v}_$i.json')); print('$v $i', d['value'], d['added_p50_ttft_ms'], d['added_p99_ttft_ms'], d['p99_ttft_ms'])"
  done
done
for v in inline0 default; do
  e=""; [ $v = inline0 ] && e="TUNNEL_INLINE_STREAMS=0"
  env $e timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 --extra=--no-jumbo-loopback > gpurun_out/r04/head_ab/ttft8_$v.json 2>> gpurun_out/r04/head_ab/err.log || exit 1
done
