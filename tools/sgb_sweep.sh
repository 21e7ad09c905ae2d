set -uo pipefail
for c in 64:1:1 64:2:1 64:4:1 32:4:1 16:4:1 64:4:2 64:4:4; do
  IFS=: read -r cb pf ch <<< "$c"
  FVO_SG_CB=$cb FVO_SG_PF=$pf FVO_SG_CHUNKS=$ch timeout -k 10 200 python -u tools/bench_sgbm.py || exit 1
done
