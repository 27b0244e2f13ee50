#!/bin/bash
# Runs the native test suite once per non-default state of every TUNNEL_*
# switch that selects a code path (README "Environment switches"), so no
# switch guards a datapath the default run leaves untested.
#   bash scripts/switch_matrix.sh [build/bin/native_tests] > profiles/r05/switch_matrix.txt
set -o pipefail
bin=${1:-build/bin/native_tests}
rc=0
for sw in "" TUNNEL_RX_READER=0 TUNNEL_RX_READER=1 TUNNEL_COALESCE_US=0 TUNNEL_SCTP_CC=reno TUNNEL_SCTP_CC=beta=100 \
          TUNNEL_DTLS_RECORDS=evp TUNNEL_UDP_OFFLOAD=none TUNNEL_FEATURES=sse TUNNEL_PIN_THREADS=0; do
  start=$(date +%s)
  out=$(env $sw timeout -k 10 900 "$bin" 2>&1); r=$?
  summary=$(echo "$out" | tail -1)
  fails=$(echo "$out" | grep '^FAIL' | tr '\n' ' ')
  echo "${sw:-defaults}: $summary ($(( $(date +%s) - start )) s) ${fails}"
  [ $r -eq 0 ] || rc=1
done
exit $rc
