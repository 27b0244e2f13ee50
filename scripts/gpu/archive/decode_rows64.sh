# Fused step timing at 1/8/16 rows (decode) and 32/64 rows (prefill-sized
# steps, several 16-row MFMA tiles), tiny and small configs, plus a rocprofv3
# kernel table of the small config at 64 rows. Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
: > gpurun_out/decode_timing_rows64.log
for args in "--batch 1" "--batch 8" "--batch 16" "--batch 32" "--batch 64" \
            "--config small --batch 1" "--config small --batch 16" "--config small --batch 64"; do
  timeout -k 10 180 python scripts/profile_decode.py --steps 200 $args >> gpurun_out/decode_timing_rows64.log 2>&1 || exit 1
  tail -1 gpurun_out/decode_timing_rows64.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_small64 -o p -- python3 $R/scripts/profile_decode.py --config small --batch 64 --steps 50 > $R/gpurun_out/rocprof_small64.log 2>&1 || exit 1
python3 $R/scripts/rocprof_summary.py $(find /tmp/prof_small64 -name '*.db' | head -1) > $R/gpurun_out/kernels_small_b64.md || exit 1
head -12 $R/gpurun_out/kernels_small_b64.md
rm -rf /tmp/prof_small64
