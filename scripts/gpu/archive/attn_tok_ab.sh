# A/B of the decode attention piece size (P2PT_ATTN_TOK 32 vs 16: 16 halves
# the K/V registers so two 8-wave workgroups fit a CU), numerics first, then
# wall-clock of the device-side decode loop (small, ctx 1024), interleaved.
#   bash scripts/gpu/archive/attn_tok_ab.sh
set -o pipefail
mkdir -p gpurun_out
P2PT_ATTN_TOK=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_attn_tok16.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_attn_tok16.log; [ $rc -eq 0 ] || exit $rc
CASES=(
  "1 P2PT_ATTN_TOK=32" "1 P2PT_ATTN_TOK=16"
  "4 P2PT_ATTN_TOK=32" "4 P2PT_ATTN_TOK=16"
  "16 P2PT_ATTN_TOK=32" "16 P2PT_ATTN_TOK=16" "16 P2PT_ATTN_TOK=16 P2PT_ATTN_WGS=512"
  "64 P2PT_ATTN_TOK=32" "64 P2PT_ATTN_TOK=16"
)
for rep in 1 2; do
  for c in "${CASES[@]}"; do
    set -- $c
    b=$1; shift
    out=$(env "$@" timeout -k 10 120 python scripts/profile_decode.py --loop --config small --batch $b --steps 400 2>/dev/null | tail -1) || exit 1
    ms=$(echo "$out" | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"], 4))') || exit 1
    echo "b=$b $* rep=$rep ms_per_step=$ms" | tee -a gpurun_out/attn_tok_ab.log
  done
done
