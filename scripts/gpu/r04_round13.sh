# Round 4, thirteenth host batch: is the single-threaded echo upstream the
# bound of the 64 x 1 MB row? (tunneled run: mock at 80-95 % of a core; the
# serve's store-and-forward hands it each body in one burst.) A/B of a 1- and a
# 2-thread mock (its 2 pinned CPUs), both MTUs, with the per-thread timeline.
set -o pipefail
export TMPDIR=/tmp
echo "== mock threads A/B"; TAG=r04/mock_ab PIN=1 TIMELINE=1 REPS=3 PATHS="std jumbo" \
  VARIANTS="m1:build:P2PT_MOCK_THREADS=1 m2:build:P2PT_MOCK_THREADS=2" \
  timeout -k 10 900 bash scripts/gpu/bulk_reps.sh > gpurun_out/r04/mock_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r04/mock_ab.log; exit $rc
