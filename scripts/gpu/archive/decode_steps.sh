# Per-position kernel timing of the fused decode step (rocprofv3 kernel trace):
# small config at batch 1 and 16, tiny at batch 1, plus wall-clock tokens/s.
#   bash scripts/gpu/archive/decode_steps.sh [TAG]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-cur}
for args in "--config small --batch 1" "--config small --batch 16" "--config tiny --batch 1"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 300 $args >> gpurun_out/decode_wall_$TAG.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_wall_$TAG.log
done
cd /tmp
for cfg in "small 1" "small 16" "tiny 1"; do
  set -- $cfg
  name=${1}_b${2}
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py --config $1 --batch $2 --steps 40 --ctx 1024 > $R/gpurun_out/rocprof_${name}_$TAG.log 2>&1 || exit 1
  python3 $R/scripts/rocprof_steps.py $(find /tmp/prof_$name -name '*.db' | head -1) --label "${name} $TAG" >> $R/gpurun_out/steps_$TAG.md || exit 1
  rm -rf /tmp/prof_$name
done
tail -3 $R/gpurun_out/steps_$TAG.md
