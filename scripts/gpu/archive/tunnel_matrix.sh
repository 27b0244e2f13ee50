# Tunnel benchmark matrix on the MI355X host (CPU-side networking; no GPU work):
# SSE 1/2/4/8 streams (native + Python mocks, WebRTC + TCP), 64 x 1 MB POST,
# idle -> burst, then a profiled 64 x 1 MB run. Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== matrix"; timeout -k 10 900 python bench/bench_tunnel.py --steps 6 --idle-s 30 --out gpurun_out/matrix.json > gpurun_out/matrix.log 2> gpurun_out/matrix.err; rc=$?; tail -4 gpurun_out/matrix.err | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== bulk profile"; timeout -k 10 300 python bench/profile_bulk.py --steps 10 --profile-dir gpurun_out/bulk_prof > gpurun_out/bulk.json 2> gpurun_out/bulk.err; rc=$?; cut -c1-400 gpurun_out/bulk.json; [ $rc -eq 0 ] || exit $rc
echo "== bulk tcp"; timeout -k 10 300 python bench/profile_bulk.py --steps 10 --transport tcp > gpurun_out/bulk_tcp.json 2>> gpurun_out/bulk.err; rc=$?; cut -c1-300 gpurun_out/bulk_tcp.json; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-500; exit $rc
