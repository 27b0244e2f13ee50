# Round 4, tenth host batch: the pinned 64 x 1 MB waterfall, twice per MTU,
# with the per-step distribution (mean vs median), the slowest steps' own
# waterfalls and the recovery counters of each run.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/wf10
for i in 1 2; do
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m $i"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 100 --pin $x > gpurun_out/r04/wf10/${m}_$i.json 2> gpurun_out/r04/wf10/${m}_$i.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r04/wf10/${m}_$i.json')); print(d['tunneled'], d['direct'], round(d['ratio'],3)); print(d['recovery'])
for s in d['slowest_steps']: print({k: round(v, 2) for k, v in s.items() if v is not None})"
done
done
