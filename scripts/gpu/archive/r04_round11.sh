# Round 4, eleventh host batch: the 64 x 1 MB waterfall with the kernel's TCP
# counters per leg (a loopback TCP segment the kernel drops waits out TCP's
# 200 ms minimum RTO), pinned on both MTUs and unpinned at 1200 MTU.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/wf11
for m in std jumbo std_nopin; do
  x=""; p="--pin"; [ $m != jumbo ] && x="--extra=--no-jumbo-loopback"; [ $m = std_nopin ] && p=""
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 100 $p $x > gpurun_out/r04/wf11/$m.json 2> gpurun_out/r04/wf11/$m.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r04/wf11/$m.json')); print(d['tunneled'], d['direct'], round(d['ratio'],3)); print('tun', {k: v for k, v in d['kernel_tunneled'].items() if v}); print('dir', {k: v for k, v in d['kernel_direct'].items() if v})
print({k: v for k, v in d['recovery'].items() if v})"
done
