# Node topology benchmark on the MI355X host CPU: one tunnel serve over 8
# native mocks (1 ms tokens), 64..1024 SSE streams, worker-thread counts
# compared; then one profiled run at 1024 streams. CPU-only; results under
# gpurun_out/node/.
set -o pipefail
mkdir -p gpurun_out/node
export TMPDIR=/tmp
echo "nproc=$(nproc)"
timeout -k 10 400 python bench/bench_node.py --streams ${STREAMS:-64,256,512,1024} --workers ${WORKERS:-0,2,4,8} \
  --steps ${STEPS:-4} --tokens 64 --lg-threads 4 --out gpurun_out/node/node.json 2> gpurun_out/node/node.err || { tail -20 gpurun_out/node/node.err; exit 1; }
python scripts/node_summary.py gpurun_out/node/node.json
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 python bench/bench_node.py --streams ${PROFILE_STREAMS:-1024} --workers ${PROFILE_WORKERS:-4} \
    --steps ${STEPS:-4} --tokens 64 --lg-threads 4 \
    --profile-dir gpurun_out/node/prof --out gpurun_out/node/node_prof.json 2> gpurun_out/node/prof.err || exit 1
  python scripts/node_summary.py gpurun_out/node/node_prof.json
  for f in gpurun_out/node/prof/*.prof; do
    python scripts/profile_report.py $f --top 25 > ${f%.prof}.txt
    python scripts/profile_report.py $f --top 25 --thread 0 > ${f%.prof}.main.txt
    python scripts/profile_report.py $f --top 25 --thread workers > ${f%.prof}.workers.txt
  done
  head -3 gpurun_out/node/prof/*.txt
fi
