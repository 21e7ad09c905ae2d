# HBM traffic of the SGBM kernels per schedule (tooling, run on the GPU box via gpurun):
# for each schedule in $MODES, tools/bench_sgbm.py (64 pairs, 960x600, D 96) under a kernel-trace
# pass and separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md: they cannot share one),
# summarised by profiles/summarize.py into gpurun_out/sgtraffic_<mode>/ (pmc_per_kernel.csv,
# kernel_stats.csv), shape key 960x600_b64_d96_<mode>.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-classic lpath}; do
  for pass in trace fetch write; do
    case $pass in
      trace) opt="--kernel-trace --stats" ;;
      fetch) opt="--pmc FETCH_SIZE --kernel-trace" ;;
      write) opt="--pmc WRITE_SIZE --kernel-trace" ;;
    esac
    timeout -s KILL 180 rocprofv3 $opt --kernel-include-regex 'k_sg_' --output-format csv \
      -d /tmp/sgt_${m}_$pass -o $pass -- python3 $R/tools/bench_sgbm.py --mode $m > $R/gpurun_out/sgt_${m}_$pass.out 2>&1 || exit 1
  done
  python3 $R/profiles/summarize.py /tmp/sgt_${m}_trace /tmp/sgt_${m}_fetch /tmp/sgt_${m}_write \
    $R/gpurun_out/sgtraffic_$m 960x600_b64_d96_$m || exit 1
done
exit 0
