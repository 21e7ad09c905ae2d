set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ba
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_parity_configs.py tests/test_frontend_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ba/tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_ba.py > gpurun_out/ba/bench600.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_ba.py --hd > gpurun_out/ba/bench1080.log 2>&1 || exit 1
for sh in 600 1080; do
  flag=""; [ $sh = 1080 ] && flag="--hd"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof$sh -o run -- python tools/bench_ba.py $flag > gpurun_out/ba/prof$sh.log 2>&1 || exit 1
  find /tmp/prof$sh -name "*kernel_stats.csv" -exec cp {} gpurun_out/ba/kstats_$sh.csv \;
done
[ -n "$WITH_BENCH" ] && { timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-frames 0 > gpurun_out/ba/bench_full.log 2>&1 || exit 1; }
exit 0
