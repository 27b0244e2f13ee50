# Kernel-level profile of the fused decode step on the "small" config (d=2048,
# 8 layers, ffn 5632, vocab 32000; ~0.85 GB of bf16 weights per step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for args in "--config small --batch 1" "--config small --batch 8" "--config small --batch 16"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 200 $args >> gpurun_out/decode_small.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_small.log
done
cd /tmp
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py "$@" > $R/gpurun_out/rocprof_$name.log 2>&1 || return 1
  python3 $R/scripts/rocprof_summary.py $(find /tmp/prof_$name -name '*.db' | head -1) > $R/gpurun_out/kernels_$name.md || return 1
  head -14 $R/gpurun_out/kernels_$name.md
  rm -rf /tmp/prof_$name
}
echo "== small b8"; prof small_b8 --config small --batch 8 --steps 50 --ctx 1024 || exit 1
