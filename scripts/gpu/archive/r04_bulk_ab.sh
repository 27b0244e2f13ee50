# Round 4: 64 x 1 MB echo, pinned, cut-through upload (serve streams bodies
# declared >= 64 KiB from REQ_HEADERS on) against store-and-forward to
# REQ_END, both MTUs, REPS alternating runs of 150 steps each.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04/bulk_ct} PIN=1 REPS=${REPS:-4} VARIANTS="sf:build: ct:build:TUNNEL_STREAM_BODY_THRESHOLD=65536" \
  timeout -k 10 1000 bash scripts/gpu/archive/bulk_reps.sh
