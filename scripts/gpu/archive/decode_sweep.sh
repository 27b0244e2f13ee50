# Decode-step tuning sweep on one GPU: numerics tests first, then wall-clock
# of the device-side decode loop (scripts/profile_decode.py --loop) under the
# kernel tunables (P2PT_DECODE_MIN_TILES, P2PT_ATTN_MINSPAN, P2PT_ATTN_SLOTS),
# then a per-position rocprofv3 kernel trace of the default settings.
#   bash scripts/gpu/archive/decode_sweep.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-sweep}
echo "== numerics"
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py tests/test_checkpoint.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_decode_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_decode_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # label, env..., -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  local out
  out=$(env "${envs[@]}" timeout -k 10 120 python scripts/profile_decode.py --loop --steps 400 "$@" 2>/dev/null | tail -1) || return 1
  echo "$label $out" | tee -a gpurun_out/decode_sweep_$TAG.log
}
for cfg in "--config small --batch 1" "--config small --batch 16" "--config small --batch 64" "--config tiny --batch 1" "--config tiny --batch 64"; do
  run "dflt" P2PT_X=0 -- $cfg || exit 1
done
cd /tmp
for cfg in "small 1" "small 16"; do
  set -- $cfg
  name=${1}_b${2}
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py --loop --config $1 --batch $2 --steps 40 --ctx 1024 > $R/gpurun_out/rocprof_${name}_$TAG.log 2>&1 || exit 1
  python3 $R/scripts/rocprof_steps.py $(find /tmp/prof_$name -name '*.db' | head -1) --label "${name} $TAG" >> $R/gpurun_out/steps_$TAG.md || exit 1
  rm -rf /tmp/prof_$name
done
grep "step span" $R/gpurun_out/steps_$TAG.md
