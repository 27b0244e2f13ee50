# A TinyLlama-1.1B-shaped random checkpoint (2.2 GB bf16, 2 safetensors shards):
# write it, decode-loop timing through the loader, then the endpoint serving it
# through the tunnel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CK=/tmp/tl11
echo "== write checkpoint"; timeout -k 10 300 python scripts/make_synthetic_checkpoint.py --shape tinyllama-1.1b --out $CK > gpurun_out/ck_write.log 2>&1 || exit 1; tail -1 gpurun_out/ck_write.log
echo "== decode loop"
for b in 1 16; do
  timeout -k 10 300 python scripts/profile_decode.py --loop --checkpoint $CK --batch $b --steps 200 2>/dev/null | tail -1 | tee -a gpurun_out/ck_decode.log || exit 1
done
echo "== endpoint through the tunnel"; timeout -k 10 900 python bench/bench_gpu_upstream.py --checkpoint $CK --streams 1,8,16 --out gpurun_out/ck_upstream.json > gpurun_out/ck_upstream.log 2> gpurun_out/ck_upstream.err; rc=$?; tail -3 gpurun_out/ck_upstream.err | cut -c1-300; exit $rc
