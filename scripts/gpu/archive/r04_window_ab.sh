# Round 4: is the 64 x 1 MB echo at 1200-byte MTU window-bound? The short-path
# queue bound holds cwnd at its 1 MiB floor (SRTT 0.5-0.7 ms under load, so
# <= ~1.7 GB/s per direction); A/B the floor and the bound itself, pinned,
# cut-through upload on, with the client-side fixes (shared request body).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r04/window_ab} PIN=1 REPS=${REPS:-3} PATHS=${PATHS:-std} STEPS=${STEPS:-150} \
  VARIANTS="f1:build:TUNNEL_STREAM_BODY_THRESHOLD=65536 f2:build:TUNNEL_STREAM_BODY_THRESHOLD=65536,TUNNEL_SCTP_QUEUE_FLOOR_KB=2048 f4:build:TUNNEL_STREAM_BODY_THRESHOLD=65536,TUNNEL_SCTP_QUEUE_FLOOR_KB=4096 qoff:build:TUNNEL_STREAM_BODY_THRESHOLD=65536,TUNNEL_SCTP_QUEUE_US=0" \
  timeout -k 10 1000 bash scripts/gpu/archive/bulk_reps.sh
