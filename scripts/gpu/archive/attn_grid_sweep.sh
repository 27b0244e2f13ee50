# Decode attention grid sweep at HEAD: wall-clock of the device-side decode
# loop (small, ctx 1024) under the attention grid knobs, 2 interleaved
# repetitions. Each case: "batch ENV=VAL ...".
#   bash scripts/gpu/archive/attn_grid_sweep.sh
set -o pipefail
mkdir -p gpurun_out
CASES=(
  "1 P2PT_ATTN_SLOTS=16" "1 P2PT_ATTN_SLOTS=24" "1 P2PT_ATTN_SLOTS=32"
  "16 P2PT_ATTN_WGS=256" "16 P2PT_ATTN_WGS=512" "16 P2PT_ATTN_WGS=768" "16 P2PT_ATTN_WGS=1024"
  "4 P2PT_ATTN_WGS=256" "4 P2PT_ATTN_WGS=512 P2PT_ATTN_SLOTS=32"
)
for rep in 1 2; do
  for c in "${CASES[@]}"; do
    set -- $c
    b=$1; shift
    out=$(env "$@" timeout -k 10 120 python scripts/profile_decode.py --loop --config small --batch $b --steps 400 2>/dev/null | tail -1) || exit 1
    ms=$(echo "$out" | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"], 4))') || exit 1
    echo "b=$b $* rep=$rep ms_per_step=$ms" | tee -a gpurun_out/attn_grid_sweep.log
  done
done
