#!/usr/bin/env bash
# Local helper (runs in the dev container, never on the GPU box): one gpurun call,
# re-submitted only when gpurun reports an infrastructure-side failure ("transient"
# status or exit 3 = no box free).  A command that ran and failed is never retried.
#   scripts/gpurun_retry.sh <timeout-seconds> '<command>'
T="$1"; shift
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = 3 ] || [ "$st" = transient ]; then
    echo "[gpurun_retry] infrastructure failure (rc=$rc status=$st), attempt $attempt; waiting" >&2
    sleep 90
    continue
  fi
  exit $rc
done
exit $rc
