#!/usr/bin/env bash
# End-to-end smoke of the whole stack with curl (behavioural equivalent of the
# reference's scripts/test-local.sh and scripts/test-tunnel.sh).
#
#   scripts/e2e.sh                 # local signal server on a free port
#   scripts/e2e.sh --public        # the public signal server (needs internet)
#   SIGNAL=ws://host:8787 scripts/e2e.sh
#
# Starts the mock LLM upstream, (optionally) the C++ signal server, `tunnel
# serve` and `tunnel proxy`, waits on their readiness log lines rather than
# fixed sleeps, then checks /v1/models, /health and a streamed chat completion
# through the proxy. Logs go to $LOGDIR (default: a fresh temp dir).
set -euo pipefail

ROOT="$(cd "$(dirname "$0")/.." && pwd)"
BIN="$ROOT/build/bin"
LOGDIR="${LOGDIR:-$(mktemp -d /tmp/p2pt-e2e.XXXXXX)}"
ROOM="e2e-$$-$RANDOM"
PUBLIC=0
[ "${1:-}" = "--public" ] && PUBLIC=1

green() { printf '\033[0;32m%s\033[0m\n' "$*"; }
red() { printf '\033[0;31m%s\033[0m\n' "$*"; }

free_port() { python3 -c 'import socket; s=socket.socket(); s.bind(("127.0.0.1",0)); print(s.getsockname()[1])'; }

PIDS=()
cleanup() {
  for p in "${PIDS[@]:-}"; do [ -n "$p" ] && kill "$p" 2>/dev/null || true; done
  wait 2>/dev/null || true
}
trap cleanup EXIT

wait_log() {  # file pattern timeout_s
  local deadline=$((SECONDS + $3))
  until grep -q "$2" "$1" 2>/dev/null; do
    if [ $SECONDS -ge $deadline ]; then
      red "timed out waiting for '$2' in $1"; tail -20 "$1" || true; exit 1
    fi
    sleep 0.05
  done
}

[ -x "$BIN/tunnel" ] || { echo "building native tree..."; cmake -S "$ROOT" -B "$ROOT/build" -G Ninja -DCMAKE_BUILD_TYPE=Release >/dev/null && cmake --build "$ROOT/build" >/dev/null; }

UP_PORT=$(free_port)
PROXY_PORT=$(free_port)
green "[1/5] mock upstream on :$UP_PORT"
python3 -m p2p_llm_tunnel_amd.utils.mock_llm --port "$UP_PORT" --threaded >"$LOGDIR/upstream.log" 2>&1 &
PIDS+=($!)
for _ in $(seq 100); do curl -sf "http://127.0.0.1:$UP_PORT/health" >/dev/null && break; sleep 0.05; done

if [ -n "${SIGNAL:-}" ]; then
  green "[2/5] using signal server $SIGNAL"
elif [ $PUBLIC = 1 ]; then
  SIGNAL=wss://signal-server.fly.dev
  green "[2/5] using public signal server $SIGNAL"
else
  SIG_PORT=$(free_port)
  SIGNAL="ws://127.0.0.1:$SIG_PORT"
  green "[2/5] local signal server on :$SIG_PORT"
  "$BIN/tunnel-signal" --listen 127.0.0.1 --port "$SIG_PORT" >"$LOGDIR/signal.log" 2>&1 &
  PIDS+=($!)
  wait_log "$LOGDIR/signal.log" "listening" 10
fi

green "[3/5] tunnel serve (room $ROOM)"
RUST_LOG=info "$BIN/tunnel" serve --signal "$SIGNAL" --room "$ROOM" \
  --upstream "http://127.0.0.1:$UP_PORT" >"$LOGDIR/serve.log" 2>&1 &
PIDS+=($!)

green "[4/5] tunnel proxy on :$PROXY_PORT"
RUST_LOG=info "$BIN/tunnel" proxy --signal "$SIGNAL" --room "$ROOM" \
  --listen "127.0.0.1:$PROXY_PORT" >"$LOGDIR/proxy.log" 2>&1 &
PIDS+=($!)
wait_log "$LOGDIR/serve.log" "sent AGREE, tunnel ready" 60
wait_log "$LOGDIR/proxy.log" "proxy listening on" 60

green "[5/5] requests through the tunnel"
fail=0
models=$(curl -s "http://127.0.0.1:$PROXY_PORT/v1/models")
if echo "$models" | grep -q test-model; then green "  ok  /v1/models"; else red "  FAIL /v1/models: $models"; fail=1; fi
health=$(curl -s "http://127.0.0.1:$PROXY_PORT/health")
if [ "$health" = ok ]; then green "  ok  /health"; else red "  FAIL /health: $health"; fail=1; fi
sse=$(curl -sN -H 'content-type: application/json' \
  -d '{"model":"test-model","stream":true,"messages":[{"role":"user","content":"hi"}]}' \
  "http://127.0.0.1:$PROXY_PORT/v1/chat/completions")
events=$(echo "$sse" | grep -c '^data: ' || true)
if [ "$events" -eq 7 ] && echo "$sse" | grep -q 'data: \[DONE\]'; then
  green "  ok  streamed chat completion ($events events)"
else
  red "  FAIL streamed chat completion ($events events)"; fail=1
fi

if [ $fail = 0 ]; then green "=== all checks passed (logs: $LOGDIR) ==="; else
  red "--- serve.log ---"; tail -20 "$LOGDIR/serve.log"; red "--- proxy.log ---"; tail -20 "$LOGDIR/proxy.log"; exit 1
fi
