#!/usr/bin/env bash
# Local helper (runs in the dev container, never on the GPU box): one gpurun call,
# re-submitted only when gpurun reports an infrastructure-side failure ("transient"
# status or exit 3 = no box free; exit 2 only for "already running" / back-off refusals).
# A command that ran and failed is never retried.  Honours gpurun's back-off hint.
#   GPURUN_ATTEMPTS=n scripts/gpurun_retry.sh <timeout-seconds> '<command>'
T="$1"; shift
LOG=$(mktemp)
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1 | tee "$LOG"
  rc=${PIPESTATUS[0]}
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = 3 ] || [ "$st" = transient ] || grep -q "already running" "$LOG"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$LOG" | tail -1 | grep -o "[0-9]*")
    wait_s=$(( ${wait_s:-90} + 10 ))
    [ "$wait_s" -lt 60 ] && wait_s=60
    echo "[gpurun_retry] infrastructure failure (rc=$rc status=$st), attempt $attempt; waiting ${wait_s}s" >&2
    sleep "$wait_s"
    continue
  fi
  rm -f "$LOG"
  exit $rc
done
rm -f "$LOG"
exit $rc
