set -o pipefail
mkdir -p gpurun_out
export P2PT_TRANSPORT=tcp
echo "== host"; nproc; python -c "import torch;print(torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))"
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== gpu tests"; timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "not webrtc" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --transport tcp --steps 10 --warmup 2 --out gpurun_out/bench_tcp.json > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; exit $rc
