# Persistent O/gate-up/down block (P2PT_DECODE_BLOCK): numerics against the
# launched kernels, then wall-clock decode loops (small, batch 1 and 16) with
# the block off and on. Logs under gpurun_out/block/.
set -o pipefail
mkdir -p gpurun_out/block
export TMPDIR=/tmp
# Quick probe first: a step that takes seconds means the dependency waits time out.
for v in 0 256; do
  P2PT_DECODE_BLOCK=$v timeout -k 5 120 python -u scripts/profile_decode.py --config small --batch 1 --eager --steps 3 --warmup 1 \
    >> gpurun_out/block/probe.log 2>&1 || { tail -5 gpurun_out/block/probe.log; exit 1; }
  tail -1 gpurun_out/block/probe.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -k block_kernel -x -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/block/pytest.log 2>&1; rc=$?; tail -n 8 gpurun_out/block/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 1 16; do
  for v in ${BLKS:-0 256 512 768 0}; do
    echo -n "block=$v " >> gpurun_out/block/wall.log
    P2PT_DECODE_BLOCK=$v timeout -k 10 180 python scripts/profile_decode.py --config small --batch $b --loop --steps 400 >> gpurun_out/block/wall.log 2>&1 || exit 1
    tail -1 gpurun_out/block/wall.log
  done
done
