# Per-thread CPU of the 64 x 1 MB echo row (config #3) on the MI355X host:
# which tunnel thread saturates. Sampling profiles (2 kHz of each thread's CPU
# time) of one run per path; prints each thread's CPU seconds next to the
# tunneled run's wall time. Reports under gpurun_out/bulk_threads/.
set -o pipefail
O=gpurun_out/bulk_threads
mkdir -p $O
export TMPDIR=/tmp
for p in ${PATHS:-std jumbo}; do
  x=""; [ $p = std ] && x="--no-jumbo-loopback"
  rm -rf /tmp/bt_$p
  TUNNEL_PROFILE_HZ=2000 timeout -k 10 300 python bench/profile_bulk.py --steps ${STEPS:-100} --extra="$x" --profile-dir /tmp/bt_$p > $O/$p.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  for f in /tmp/bt_$p/*.prof; do
    b=$(basename $f .prof)
    python scripts/profile_report.py $f --top 30 > $O/${p}_$b.txt
    python scripts/profile_report.py $f --top 30 --thread 0 > $O/${p}_$b.main.txt
  done
  python - $O/$p.json $O/${p}_*.txt <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1]))
tun_s = d["wall_s_incl_warmup"]
print(sys.argv[1].split("/")[-1], "tunneled", round(d["tunneled_req_s"]), "direct", round(d["direct_req_s"]),
      "tunneled run %.1f s" % tun_s, "cpu", d["cpu_s_incl_warmup"])
# Thread shares of the sampled CPU time, scaled to the process's CPU over the
# timed tunneled run (profile_bulk measures it around warmup + the timed steps).
role = {str(v): k for k, v in d.get("pids", {}).items()}
for f in sys.argv[2:]:
    if f.endswith(".main.txt"):
        continue
    t = open(f).read()
    pid = re.search(r"tunnel\.(\d+)", f.split("/")[-1]).group(1)
    r = role.get(pid, pid)
    cpu = d["cpu_s_incl_warmup"].get(r, 0.0)
    th = re.search(r"threads \(samples %\): (.*)", t).group(1)
    parts = [(k, float(v)) for k, v in (x.split() for x in th.split(", "))]
    print("  ", r, "cpu %.1f s:" % cpu, " ".join("%s %.0f%%" % (k, 100 * cpu * v / 100 / tun_s) for k, v in parts),
          "(of one core over the tunneled run)")
PY
done
