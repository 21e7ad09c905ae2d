# SQ counters of the SGBM kernels per schedule (tooling): one rocprofv3 --pmc pass of
# tools/bench_sgbm.py per schedule in $MODES; CSVs under gpurun_out/sgpmc/<mode>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgpmc
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-classic lpath}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --kernel-include-regex 'k_sg_' --output-format csv -d /tmp/sgpmc_$m -o pmc -- python3 $R/tools/bench_sgbm.py --mode $m > $R/gpurun_out/sgpmc/$m.out 2>&1 || exit 1
  mkdir -p $R/gpurun_out/sgpmc/$m && find /tmp/sgpmc_$m -name "*counter_collection.csv" -exec cp {} $R/gpurun_out/sgpmc/$m/ \;
done
exit 0
