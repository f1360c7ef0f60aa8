#!/bin/bash
# Per-launch clock and address-translation counters over the G2 series after an idle gap
# (VERDICT r4 item 2): one pass per counter group, each its own rocprofv3 run.  Then packed vs
# line-aligned datagrams (item 5): A/B times and read requests per layout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05_tlb}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for counters in "GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY SQ_BUSY_CYCLES TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
                "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/pass$i" -o run --output-format csv \
    -- python3 "$ROOT/scripts/exp_ramp_pmc.py" --launches 200 > "$OUT/pass$i.log" 2>&1 || exit $?
  echo "[tlb] pass $i done" >&2
done
# packed vs line-aligned datagrams: A/B, then read requests per layout
timeout -k 10 240 python3 "$ROOT/scripts/exp_layout.py" --blocks 12 > "$OUT/layout_ab.txt" 2>&1 || exit $?
echo "[tlb] layout A/B done" >&2
for lay in packed aligned; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/rdreq_$lay" -o run --output-format csv \
    -- python3 "$ROOT/scripts/exp_layout.py" --only $lay --blocks 1 --launches 5 > "$OUT/rdreq_$lay.log" 2>&1 || exit $?
done
echo "[tlb] layout rdreq done" >&2
cd "$ROOT"
for lay in packed aligned; do
  PMC_FILTER=crc32_ragged_jobs python3 scripts/pmc_summary.py "$OUT/rdreq_$lay" > "$OUT/rdreq_${lay}_summary.txt" 2>&1
done
for d in "$OUT"/pass*/; do
  python3 scripts/ramp_pmc_summary.py "$d" > "${d%/}_summary.txt" 2>&1
done
echo "[tlb] done" >&2
