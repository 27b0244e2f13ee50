# Round-4 first host probe: box facts, the headline, the 8-stream TTFT hops on
# both MTUs, and the 64 x 1 MB echo waterfall (pinned and not) on both MTUs.
set -o pipefail
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
{ nproc; taskset -cp $$; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; lscpu | head -25; sysctl net.core.rmem_max net.core.wmem_max net.core.rmem_default net.ipv4.udp_mem 2>&1; } > gpurun_out/r04/box.txt 2>&1
echo "== bench"; timeout -k 10 200 python bench.py --out gpurun_out/r04/bench_head.json > gpurun_out/r04/bench_head.log 2>&1 || exit 1
for m in std jumbo; do
  x=""; [ $m = std ] && x="--extra=--no-jumbo-loopback"
  echo "== wf $m pinned"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 60 --pin $x > gpurun_out/r04/wf_${m}_pin.json 2> gpurun_out/r04/wf_${m}_pin.err || exit 1
  echo "== wf $m"; timeout -k 10 200 python scripts/ttft_breakdown.py --bulk-echo --steps 60 $x > gpurun_out/r04/wf_${m}.json 2> gpurun_out/r04/wf_${m}.err || exit 1
done
echo "== ttft8"; timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 --extra=--no-jumbo-loopback > gpurun_out/r04/ttft8_std.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 > gpurun_out/r04/ttft8_jumbo.txt 2>&1
