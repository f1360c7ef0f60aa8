#!/usr/bin/env bash
# A/B: LDS-DMA uniform kernel (ENET_CRC_UNIFORM=dma) vs the register-ring kernel (regs, the default).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-abregs}"
mkdir -p "$OUT"
cd "$ROOT"
(rocm-smi --showuniqueid 2>/dev/null | grep -i "unique" | head -1) || true
for i in 1 2 3 4; do
  for v in dma regs; do
    ENET_CRC_UNIFORM=$v timeout -k 10 200 python bench.py --cpu-seconds 0 --no-e2e --steps 40 > "$OUT/bench_${v}_$i.json" 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['shard_2m']['kernel_ms'], d['mtu_1392']['kernel_ms'])" "$OUT/bench_${v}_$i.json" "$v run $i"
  done
done
