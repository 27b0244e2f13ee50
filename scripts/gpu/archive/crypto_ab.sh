# AES-GCM record layer on the MI355X host CPU: microbenchmark, then the
# 64 x 1 MB WebRTC body benchmark with the vector AES-GCM vs OpenSSL EVP
# (TUNNEL_DTLS_EVP=1), alternating runs. CPU-only; results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/crypto
export TMPDIR=/tmp
timeout -k 10 120 ./build/bin/tunnel-cryptobench > gpurun_out/crypto/cryptobench.jsonl || exit $?
cat gpurun_out/crypto/cryptobench.jsonl
for i in 1 2 3; do
  for mode in vector evp; do
    if [ $mode = evp ]; then export TUNNEL_DTLS_EVP=1; else unset TUNNEL_DTLS_EVP; fi
    timeout -k 10 300 python bench/profile_bulk.py --steps 10 > gpurun_out/crypto/bulk_${mode}_$i.json 2>> gpurun_out/crypto/bulk.err || exit $?
    echo "$mode $i $(cut -c1-330 gpurun_out/crypto/bulk_${mode}_$i.json)"
  done
done
unset TUNNEL_DTLS_EVP
timeout -k 10 300 python bench/profile_bulk.py --steps 10 --profile-dir gpurun_out/crypto/prof > gpurun_out/crypto/bulk_prof.json 2>> gpurun_out/crypto/bulk.err || exit $?
for f in gpurun_out/crypto/prof/*.prof; do python scripts/profile_report.py $f --top 12 > ${f%.prof}.txt; done
echo done
