# Kernel trace of the BA stage alone at 1080p (tooling): tools/bench_ba.py --hd under rocprofv3
# --kernel-trace --stats, per-kernel stats of the k_ba_ kernels into gpurun_out/batrace/.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/batrace
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_ba_' --output-format csv \
  -d /tmp/batr -o ba -- python3 $R/tools/bench_ba.py ${BA_ARGS:---hd} > $R/gpurun_out/batrace/bench_ba.out 2>&1 || exit 1
find /tmp/batr -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/batrace/ \;
exit 0
