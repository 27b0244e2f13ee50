# Interleaved wall-clock A/B of two in-tree builds of the HIP kernels (and env
# variants) on one box: scripts/profile_decode.py --loop, 3 rounds each.
#   bash scripts/gpu/archive/decode_ab.sh TAG "label|LIB|ENV..." ...   (LIB: file under ops/)
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for cfg in "--config small --batch 1" "--config small --batch 16"; do
  for round in 1 2 3; do
    for v in "$@"; do
      IFS='|' read -r label libf envs <<< "$v"
      out=$(env P2PT_HIP_OPS_LIB=$libf $envs timeout -k 10 120 python scripts/profile_decode.py --loop --steps 400 $cfg 2>/dev/null | tail -1) || exit 1
      echo "$label $out" | tee -a gpurun_out/decode_ab_$TAG.log
    done
  done
done
