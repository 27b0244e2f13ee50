# BASELINE config #3 and the mixed row at HEAD on the MI355X host, defaults
# only: 64 x 1 MB echo (5 alternating reps of ~10 s per path) and SSE next to
# bulk (5 x 10 s, 8-thread mock). Raw files under gpurun_out/head_rows/.
#   bash scripts/gpu/archive/head_rows.sh
set -o pipefail
mkdir -p gpurun_out/head_rows
export TMPDIR=/tmp
echo "== bulk"; TAG=head_rows/bulk REPS=5 timeout -k 10 600 bash scripts/gpu/archive/bulk_reps.sh > gpurun_out/head_rows/bulk.log 2>&1; rc=$?; tail -3 gpurun_out/head_rows/bulk.log; [ $rc -eq 0 ] || exit $rc
echo "== mixed"; timeout -k 10 500 python bench/bench_mixed.py --seconds 10 --reps 5 --mock-threads 8 --out gpurun_out/head_rows/mixed.json > /dev/null 2> gpurun_out/head_rows/mixed.err; rc=$?; tail -3 gpurun_out/head_rows/mixed.err; exit $rc
