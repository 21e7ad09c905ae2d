#!/bin/bash
# MFMA utilisation of the BA Schur kernel (north_star: "MFMA utilisation reported against gfx950
# peak"): one rocprofv3 --pmc pass (SQ MFMA counters + GRBM_GUI_ACTIVE, within the per-pass slot
# limits: <= 8 SQ, <= 2 GRBM) over a short bench run, summarised per kernel by
# profiles/summarize_mfma.py.   gpurun -- 'bash tools/mfma_pmc.sh <tag>'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/mfma_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
CTRS=""
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE; do
  grep -qw "$c" "$OUT/counters_list.txt" && CTRS="$CTRS $c"
done
echo "counters:$CTRS"
[ -n "$CTRS" ] || { echo "no MFMA counters listed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d /tmp/p_mfma -o mfma -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0 > /dev/null 2> "$OUT/pmc.err" || { echo "pmc pass failed"; tail -5 "$OUT/pmc.err"; exit 1; }
python3 "$R/profiles/summarize_mfma.py" /tmp/p_mfma "$OUT"
