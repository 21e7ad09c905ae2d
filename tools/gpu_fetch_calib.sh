# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.hip; run on the GPU box):
#   gpurun -- 'bash tools/gpu_fetch_calib.sh'
# pass 1: the program alone (bytes + HIP-event times), passes 2/3: FETCH_SIZE / WRITE_SIZE
# (separate passes, MI355X_MICROARCH.md §HBM), then tools/fetch_calib_summary.py joins them into
# gpurun_out/fetch_calib/fetch_calib.csv (factor = counter bytes / bytes the pattern moves).
set -uo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/fetch_calib
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$R/tools/fetch_calib" > "$OUT/run.jsonl" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/fc_$c -o $c -- "$R/tools/fetch_calib" \
    > "$OUT/$c.out" 2>&1 || { echo "pass $c failed"; tail -5 "$OUT/$c.out"; exit 1; }
done
python3 "$R/tools/fetch_calib_summary.py" "$OUT/run.jsonl" /tmp/fc_FETCH_SIZE /tmp/fc_WRITE_SIZE "$OUT/fetch_calib.csv"
