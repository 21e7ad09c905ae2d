# BA change check (tooling): the BA parity tests, the stamped variant's phase times and an
# A/B of tools/bench_ba.py against exp/libfvo_babase.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/batry
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ba.py tests/test_parity_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/batry/tests.log 2>&1 || { tail -40 gpurun_out/batry/tests.log; exit 1; }
tail -2 gpurun_out/batry/tests.log
# (stamps: tools/gpu_ba_stamp.sh)
rm -f gpurun_out/bav/bench.log
VARIANTS=babase HD=1 bash tools/gpu_ba_variants.sh || exit 1
cat gpurun_out/bav/bench.log
