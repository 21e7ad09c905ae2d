#!/bin/bash
# rocprofv3 collection for the committed profiles (run on the GPU box via gpurun):
#   gpurun -- 'bash profiles/collect.sh <tag> <shape> [bench args...]'
# with <shape> = bench.py's shape_key (e.g. 960x600_n1000_b64_k10) for the bench args.
#   pass 1: kernel trace + stats;  passes 2/3: FETCH_SIZE / WRITE_SIZE (separate passes:
#   MI355X_MICROARCH.md §HBM, TCC FETCH_SIZE and WRITE_SIZE cannot share one);  pass 4: SQ
#   VALU counters;  pass 5: MFMA counters of the BA Schur kernel.
# Each pass runs under its own time limit; summaries of libfvo kernels only, keyed by shape.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; SHAPE=$2; shift 2
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-frames 0 --ate-frames 0 $*"
run() {  # run <name> <rocprof args...>
  local n=$1; shift
  timeout -s KILL 420 rocprofv3 "$@" --output-format csv -d /tmp/p_$n -o $n -- python3 "$R/bench.py" $ARGS \
    > "$OUT/$n.out" 2> "$OUT/$n.err" || { echo "pass $n failed"; tail -3 "$OUT/$n.err"; exit 1; }
}
run trace --kernel-trace --stats
# counters on libfvo's kernels only (all in anonymous namespaces): instrumenting the synthetic
# renderer's torch kernels crashed rocprofv3's PMC passes at 1080p
KF=(--kernel-include-regex 'anonymous namespace\)::k_')
run fetch --pmc FETCH_SIZE --kernel-trace "${KF[@]}"
run write --pmc WRITE_SIZE --kernel-trace "${KF[@]}"
run valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace "${KF[@]}"
run mfma --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace "${KF[@]}"
python3 "$R/profiles/summarize.py" /tmp/p_trace /tmp/p_fetch /tmp/p_write "$OUT" "$SHAPE" &&
python3 "$R/profiles/summarize_pmc.py" /tmp/p_valu "$OUT/valu_per_kernel.csv" "$SHAPE" k_ > /dev/null &&
python3 "$R/profiles/summarize_mfma.py" /tmp/p_mfma "$OUT" "$SHAPE" > /dev/null &&
cp "$OUT/trace.out" "$OUT/bench_under_trace.json" && echo "profiles in $OUT"
