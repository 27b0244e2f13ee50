# Round-3 host-side matrix on the MI355X box (CPU-only work: the tunnel has no
# GPU compute). PART=mixed: SSE next to bulk (5 alternating direct/tunneled
# reps of 10 s per path). PART=node: one serve over 8 upstreams at 256/512/1024
# SSE streams (5 x 10 s per point). Results under gpurun_out/r03/.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
echo "nproc=$(nproc)"
case "${PART:-mixed}" in
  mixed)
    timeout -k 10 900 python bench/bench_mixed.py --seconds 10 --reps 5 --out gpurun_out/r03/mixed.json \
      > /dev/null 2> gpurun_out/r03/mixed.err || { tail -5 gpurun_out/r03/mixed.err; exit 1; }
    tail -4 gpurun_out/r03/mixed.err | cut -c1-800
    ;;
  node)
    timeout -k 10 1000 python bench/bench_node.py --streams ${STREAMS:-256,512,1024} --workers auto --seconds 10 --reps 5 \
      --tokens 64 --lg-threads 4 --out gpurun_out/r03/node.json > /dev/null 2> gpurun_out/r03/node.err \
      || { tail -5 gpurun_out/r03/node.err; exit 1; }
    python scripts/node_summary.py gpurun_out/r03/node.json
    ;;
esac
