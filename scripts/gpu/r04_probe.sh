set -o pipefail
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
{ nproc; taskset -cp $$; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; lscpu | head -25; numactl -H 2>/dev/null | head -5; sysctl net.core.rmem_max net.core.wmem_max net.core.rmem_default net.ipv4.udp_mem 2>&1; ulimit -a; } > gpurun_out/r04/box.txt 2>&1
timeout -k 10 200 python bench.py --out gpurun_out/r04/bench_head.json > gpurun_out/r04/bench_head.log 2>&1 || exit 1
timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 --extra=--no-jumbo-loopback > gpurun_out/r04/ttft8_std.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/ttft_breakdown.py --streams 8 --requests 400 > gpurun_out/r04/ttft8_jumbo.txt 2>&1
