# SGBM schedule A/B on the GPU box (tooling): SGBM parity tests, then tools/bench_sgbm.py twice per
# variant, VARIANTS = space-separated tools/bench_sgbm.py argument sets with commas between
# arguments, e.g. VARIANTS="--mode=classic --mode=lpath --mode=classic,--lanes=4".
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgab
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_natural.py -x -v -k "sgbm" --timeout 120 --timeout-method thread > gpurun_out/sgab/tests.log 2>&1 || exit 1
for v in ${VARIANTS:---mode=classic --mode=lpath}; do
  for rep in 1 2; do
    echo -n "$v " >> gpurun_out/sgab/bench.log
    timeout -k 10 120 python tools/bench_sgbm.py $(echo $v | tr ',' ' ') 2>/dev/null | tail -1 >> gpurun_out/sgab/bench.log || exit 1
  done
done
exit 0
