set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1 || true
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py "$@" > $R/gpurun_out/rocprof_$name.log 2>&1 || return 1
  python3 $R/scripts/rocprof_summary.py $(find /tmp/prof_$name -name '*.db' | head -1) > $R/gpurun_out/kernels_$name.md || return 1
  grep -E "k_attn|k_skinny|ms_per_step" $R/gpurun_out/kernels_$name.md | head -3
  rm -rf /tmp/prof_$name
}
for ctx in 64 512 1024 2000; do echo "== graph ctx $ctx"; prof graph_ctx$ctx --steps 50 --ctx $ctx || exit 1; done
for ctx in 64 1024; do echo "== eager ctx $ctx"; prof eager_ctx$ctx --steps 50 --ctx $ctx --eager || exit 1; done
