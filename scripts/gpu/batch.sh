# Runs a host batch: a plan file of bench/ab.py (or other) command lines, one
# per line ('#' comments allowed), each under its own time limit, stopping at
# the first failure (nothing is retried). Output under gpurun_out/.
#   bash scripts/gpu/batch.sh scripts/gpu/plans/<plan>.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
plan=$1
[ -f "$plan" ] || { echo "no plan $plan"; exit 2; }
while IFS= read -r line || [ -n "$line" ]; do
  case "$line" in ''|'#'*) continue ;; esac
  echo "== $line"
  timeout -k 10 ${STEP_TIMEOUT:-1000} bash -c "$line"; rc=$?
  [ $rc -eq 0 ] || { echo "step failed (exit $rc): $line"; exit $rc; }
done < "$plan"
