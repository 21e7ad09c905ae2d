# SGBM library A/B (tooling): the SGBM parity tests on the in-tree library, then
# tools/bench_sgbm.py alternating the in-tree library and exp/libfvo_${VARIANT:-base}.so, $REPS times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgab
export TMPDIR=/tmp
rm -f gpurun_out/sgab/ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k sgbm -x -q --timeout 120 --timeout-method thread > gpurun_out/sgab/parity.log 2>&1 || { tail -30 gpurun_out/sgab/parity.log; exit 1; }
tail -1 gpurun_out/sgab/parity.log
for rep in $(seq ${REPS:-3}); do
  for v in tree ${VARIANT:-base}; do
    lib=""; [ "$v" = tree ] || lib=exp/libfvo_$v.so
    echo -n "$v " >> gpurun_out/sgab/ab.log
    FVO_LIB=$lib timeout -k 10 120 python tools/bench_sgbm.py 2>/dev/null | tail -1 >> gpurun_out/sgab/ab.log || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/sgab/ab.log"):
    v, j = l.split(" ", 1); d = json.loads(j)
    print(v, d["call_ms"], d["kernels_ms"])
PY
