set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1 || true
for ctx in 64 512 1024 2000; do
  echo "== rocprof ctx $ctx"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ctx$ctx -o ctx -- python3 $R/scripts/profile_decode.py --steps 50 --ctx $ctx > $R/gpurun_out/rocprof_ctx$ctx.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/rocprof_ctx$ctx.log
done
for ctx in 64 1024; do
  echo "== eager rocprof ctx $ctx"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_eager_ctx$ctx -o ctx -- python3 $R/scripts/profile_decode.py --steps 50 --ctx $ctx --eager > $R/gpurun_out/rocprof_eager_ctx$ctx.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/rocprof_eager_ctx$ctx.log
done
