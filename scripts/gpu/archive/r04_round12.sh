# Round 4, twelfth host batch: the 64 x 1 MB waterfall (pinned, both MTUs)
# with each slow step's straggler request and its new-connection count, and
# every kernel network counter that moved per leg.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/wf12
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 100 --pin $x > gpurun_out/r04/wf12/$m.json 2> gpurun_out/r04/wf12/$m.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r04/wf12/$m.json')); print(d['tunneled'], d['direct'], round(d['ratio'],3))
for s in d['slowest_steps']: print(s['step end at the client'], s['new connections'], s['straggler'])"
done
