# Decode weights through the 256 MB Infinity Cache.
# 1) What the kernels reach when their weights stay resident: the small
#    config at batch 1 against the same layer shapes with 2 layers and an
#    8000-row LM head (213 MB of weights: resident between steps).
# 2) Prefetch workgroups (P2PT_DECODE_PF bit mask, decode_fused.hip
#    prefetch_range): wall-clock loops per mask at batch 1 and 16, then a
#    kernel trace of mask $PFT.
#   bash scripts/gpu/archive/decode_mall.sh [TAG]
set -o pipefail
mkdir -p gpurun_out/decode_mall
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-mall}
O=$R/gpurun_out/decode_mall
for sets in "--set n_layers=2 --set vocab=8000" "--set n_layers=2"; do
  timeout -k 10 180 python scripts/profile_decode.py --config small --batch 1 --loop --steps 400 $sets >> $O/wall_$TAG.log 2>&1 || exit 1
  tail -1 $O/wall_$TAG.log
done
for b in 1 16; do
  for m in ${PFS:-0 1 2 4 8 3 15 0}; do
    echo -n "pf$m " >> $O/wall_$TAG.log
    P2PT_DECODE_PF=$m timeout -k 10 180 python scripts/profile_decode.py --config small --batch $b --loop --steps 400 >> $O/wall_$TAG.log 2>&1 || exit 1
    tail -1 $O/wall_$TAG.log
  done
done
cd /tmp
i=0
for v in "0|--set n_layers=2 --set vocab=8000" "0|" "${PFT:-15}|"; do
  i=$((i+1))
  m=${v%%|*}; sets=${v#*|}
  P2PT_DECODE_PF=$m timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_m$i -o p -- python3 $R/scripts/profile_decode.py --config small --batch 1 --loop --steps 60 $sets > $O/rocprof_$i.log 2>&1 || exit 1
  python3 $R/scripts/rocprof_steps.py $(find /tmp/prof_m$i -name '*.db' | head -1) --label "small b1 pf$m $sets" >> $O/steps_$TAG.md || exit 1
  rm -rf /tmp/prof_m$i
done
grep -E "^###|step span" $O/steps_$TAG.md
