# Decode attention span sweep at HEAD: wall-clock of the device-side decode
# loop (small, ctx 1024) under P2PT_ATTN_MINSPAN, 2 interleaved repetitions.
#   bash scripts/gpu/archive/attn_span_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for b in 1 16; do
    for span in 64 128 256 512; do
      out=$(P2PT_ATTN_MINSPAN=$span timeout -k 10 120 python scripts/profile_decode.py --loop --config small --batch $b --steps 400 2>/dev/null | tail -1) || exit 1
      echo "span=$span rep=$rep $out" | tee -a gpurun_out/attn_span_sweep.log
    done
  done
done
