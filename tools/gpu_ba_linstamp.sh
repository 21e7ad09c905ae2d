# Phase timing of a stamped k_ba_lin variant (tooling): tools/bench_ba.py --hd under
# FVO_LIB=exp/libfvo_stamp.so; the kernel's printf lines -> gpurun_out/bastamp/lin.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bastamp
export TMPDIR=/tmp
FVO_LIB=exp/libfvo_stamp.so timeout -k 10 150 python tools/bench_ba.py ${BA_ARGS:---hd} > /tmp/st.out 2>&1 || { tail -20 /tmp/st.out; exit 1; }
grep LIN_STAMP /tmp/st.out | tail -64 > gpurun_out/bastamp/lin.txt
tail -1 /tmp/st.out >> gpurun_out/bastamp/lin.txt
