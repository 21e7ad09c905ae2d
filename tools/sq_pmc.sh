#!/bin/bash
# One rocprofv3 --pmc pass (<= 8 SQ + GRBM_GUI_ACTIVE) over a command, summarised per kernel
# by profiles/summarize_pmc.py.   gpurun -- 'bash tools/sq_pmc.sh <tag> <shape> "<ctrs>" <cmd...>'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SHAPE=$2; CTRS=$3; shift 3
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d /tmp/p_$TAG -o p -- "$@" > "$OUT/cmd.out" 2> "$OUT/pmc.err" || { echo "pmc pass failed"; tail -5 "$OUT/pmc.err"; exit 1; }
python3 "$R/profiles/summarize_pmc.py" /tmp/p_$TAG "$OUT/pmc.csv" "$SHAPE" k_
