#!/bin/bash
# Timing-only refine variants (FVO_PNP_EXP=1: stop after the init reductions, 2: after the DLT)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pnpexp"
cd /tmp && export TMPDIR=/tmp
for e in 0 1 2; do
  FVO_PNP_EXP=$e timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_pe$e -o pe -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0 --overlap-sgbm 0 > "$R/gpurun_out/pnpexp/b$e.json" 2> "$R/gpurun_out/pnpexp/b$e.err" || { tail -5 "$R/gpurun_out/pnpexp/b$e.err"; exit 1; }
  f=$(find /tmp/p_pe$e -name "*kernel_stats.csv" | head -1)
  echo "EXP=$e"; python3 "$R/tools/kstats.py" "$f" k_pnp_refine
done
