# Kernel trace of the BA stage at 1080p (tooling): tools/bench_ba.py --hd under rocprofv3
# --kernel-trace, the last step's per-queue chain (tools/ba_chain.py) into gpurun_out/bachain/chain.txt.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/bachain
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex 'k_ba_' --output-format csv \
  -d /tmp/bach -o ba -- python3 $R/tools/bench_ba.py ${BA_ARGS:---hd} > /tmp/bach_bench.out 2>&1 || { tail -c 20000 /tmp/bach_bench.out; exit 1; }
f=$(find /tmp/bach -name "*kernel_trace.csv" | head -1)
tail -c 4000 /tmp/bach_bench.out > $R/gpurun_out/bachain/bench_ba.out
ls -la "$f"
python3 $R/tools/ba_chain.py "$f" > $R/gpurun_out/bachain/chain.txt || exit 1
exit 0
