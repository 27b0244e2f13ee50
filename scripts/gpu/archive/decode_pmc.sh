# HBM bytes per decode kernel (TCC FETCH_SIZE / WRITE_SIZE) on the small config, batch 8.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc1 -o p -- python3 $R/scripts/profile_decode.py --config small --batch 8 --steps 10 --warmup 2 --ctx 1024 > $R/gpurun_out/pmc1.log 2>&1 || { tail -5 $R/gpurun_out/pmc1.log; exit 1; }
f=$(find /tmp/pmc1 -name '*counter_collection.csv' | head -1)
cp "$f" $R/gpurun_out/pmc_fetch.csv
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc2 -o p -- python3 $R/scripts/profile_decode.py --config small --batch 8 --steps 10 --warmup 2 --ctx 1024 > $R/gpurun_out/pmc2.log 2>&1 || { tail -5 $R/gpurun_out/pmc2.log; exit 1; }
f=$(find /tmp/pmc2 -name '*counter_collection.csv' | head -1)
cp "$f" $R/gpurun_out/pmc_write.csv
head -3 $R/gpurun_out/pmc_fetch.csv | cut -c1-400
