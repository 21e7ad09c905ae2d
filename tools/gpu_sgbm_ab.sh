# SGBM schedule A/B on the GPU box (tooling): SGBM parity tests, then tools/bench_sgbm.py twice per
# variant, VARIANTS = space-separated env settings with commas between assignments, e.g.
# VARIANTS="FVO_SG_MODE=classic FVO_SG_MODE=split,FVO_SG_CHUNKS=8".
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgab
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_natural.py -x -v -k "sgbm" --timeout 120 --timeout-method thread > gpurun_out/sgab/tests.log 2>&1 || exit 1
for v in ${VARIANTS:-FVO_SG_MODE=classic FVO_SG_MODE=split}; do
  for rep in 1 2; do
    echo -n "$v " >> gpurun_out/sgab/bench.log
    env $(echo $v | tr ',' ' ') timeout -k 10 120 python tools/bench_sgbm.py 2>/dev/null | tail -1 >> gpurun_out/sgab/bench.log || exit 1
  done
done
exit 0
