set -uo pipefail
for c in ${CFGS:-8:32:4:1:1 8:32:8:1:1 8:32:8:2:1}; do
  IFS=: read -r g cb hg pf ch <<< "$c"
  FVO_SG_G=$g FVO_SG_CB=$cb FVO_SG_HG=$hg FVO_SG_PF=$pf FVO_SG_CHUNKS=$ch timeout -k 10 200 python -u tools/bench_sgbm.py || exit 1
done
