# SGBM A/B on the GPU box (tooling): parity tests of the SGBM kernels, then tools/bench_sgbm.py
# per variant argument set (VARIANTS="--mode=classic --lanes=4" ...).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sg
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_parity_configs.py -x -v -k "sgbm or disparity or config or middlebury" --timeout 200 --timeout-method thread > gpurun_out/sg/tests.log 2>&1 || exit 1
for v in ${VARIANTS:---mode=classic}; do
  for rep in 1 2; do
    timeout -k 10 120 python tools/bench_sgbm.py $(echo $v | tr ',' ' ') >> "gpurun_out/sg/bench_$(echo $v | tr -c "A-Za-z0-9=_.\n" "_").log" 2>&1 || exit 1
  done
done
exit 0
