set -uo pipefail
for v in "FVO_SG_EXP=0" "FVO_SG_EXP=1" "FVO_SG_EXP=2" "FVO_SG_EXP=3"; do
  echo "$v"; env $v timeout -k 10 120 python -u tools/bench_sgbm.py || exit 1
done
