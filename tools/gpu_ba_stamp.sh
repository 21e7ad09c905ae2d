# Phase timing of a stamped BA variant (tooling): tools/bench_ba.py under FVO_LIB=exp/libfvo_stamp.so,
# the kernel's printf lines (s_memrealtime ticks, 10 ns) -> gpurun_out/bastamp/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bastamp
export TMPDIR=/tmp
for flag in --hd ""; do
  FVO_LIB=exp/libfvo_stamp.so timeout -k 10 150 python tools/bench_ba.py $flag > /tmp/st.out 2>&1 || { tail -20 /tmp/st.out; exit 1; }
  grep STAMP /tmp/st.out | tail -60 > gpurun_out/bastamp/stamps${flag}.txt
  tail -1 /tmp/st.out >> gpurun_out/bastamp/stamps${flag}.txt
done
