# Round 6: the GPU endpoint's decode step at HEAD:
# wall clock of the device-side loop and a per-position rocprofv3 kernel
# trace, small config, batch 1 and 16.
set -o pipefail
mkdir -p gpurun_out/r06/decode
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "--config small --batch 1" "--config small --batch 16"; do
  out=$(timeout -k 10 120 python scripts/profile_decode.py --loop --steps 400 $cfg 2>/dev/null | tail -1) || exit 1
  echo "$cfg $out" | tee -a gpurun_out/r06/decode/decode_wall.log
done
cd /tmp
for cfg in "small 1" "small 16"; do
  set -- $cfg
  name=${1}_b${2}
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$name -o p -- python3 $R/scripts/profile_decode.py --loop --config $1 --batch $2 --steps 40 --ctx 1024 > $R/gpurun_out/r06/decode/rocprof_${name}.log 2>&1 || exit 1
  python3 $R/scripts/rocprof_steps.py $(find /tmp/prof_$name -name '*.db' | head -1) --label "${name} r06" >> $R/gpurun_out/r06/decode/steps_r06.md || exit 1
  rm -rf /tmp/prof_$name
done
grep "step span" $R/gpurun_out/r06/decode/steps_r06.md
# Attention grid knobs at batch 1 and 16 (wall clock of the device-side loop).
cd $R
for knob in "P2PT_ATTN_SLOTS=8" "P2PT_ATTN_SLOTS=32" "P2PT_ATTN_MINSPAN=32" "P2PT_ATTN_MINSPAN=128"; do
  for b in 1 16; do
    out=$(env $knob timeout -k 10 120 python scripts/profile_decode.py --loop --steps 400 --config small --batch $b 2>/dev/null | tail -1) || exit 1
    echo "$knob b$b $out" | tee -a gpurun_out/r06/decode/decode_knobs.log
  done
done
