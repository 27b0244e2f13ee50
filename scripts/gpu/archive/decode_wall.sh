# Wall-clock decode loops of the small config at batch 1 and 16 (3 runs each),
# the numbers BASELINE quotes; log under gpurun_out/decode_wall.log.
set -o pipefail
mkdir -p gpurun_out
for b in 1 16; do
  for i in 1 2 3; do
    timeout -k 10 180 python scripts/profile_decode.py --config small --batch $b --loop --steps 400 >> gpurun_out/decode_wall.log 2>&1 || exit 1
    tail -1 gpurun_out/decode_wall.log
  done
done
