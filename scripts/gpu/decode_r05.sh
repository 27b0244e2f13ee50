# Round 5: the GPU endpoint's decode step at HEAD (unchanged this round):
# wall clock of the device-side loop and a per-position rocprofv3 kernel
# trace, small config, batch 1 and 16.
set -o pipefail
mkdir -p gpurun_out/r05/decode
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "--config small --batch 1" "--config small --batch 16"; do
  out=$(timeout -k 10 120 python scripts/profile_decode.py --loop --steps 400 $cfg 2>/dev/null | tail -1) || exit 1
  echo "$cfg $out" | tee -a gpurun_out/r05/decode/decode_wall.log
done
cd /tmp
for cfg in "small 1" "small 16"; do
  set -- $cfg
  name=${1}_b${2}
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py --loop --config $1 --batch $2 --steps 40 --ctx 1024 > $R/gpurun_out/r05/decode/rocprof_${name}.log 2>&1 || exit 1
  python3 $R/scripts/rocprof_steps.py $(find /tmp/prof_$name -name '*.db' | head -1) --label "${name} r05" >> $R/gpurun_out/r05/decode/steps_r05.md || exit 1
  rm -rf /tmp/prof_$name
done
grep "step span" $R/gpurun_out/r05/decode/steps_r05.md
