#!/bin/bash
# SGBM launch-variant sweep on the GPU box: parity of the variants, then the bench's stage
# times per variant (cb:pf:chunks = FVO_SG_CB / FVO_SG_PF / FVO_SG_CHUNKS).
#   gpurun -- 'bash tools/sg_sweep.sh "64:1:1 64:2:1 64:4:1 32:2:1 16:2:1 64:2:2 64:4:4"'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
CFGS=${1:-"64:1:1 64:2:1 64:4:1 32:4:1 16:4:1 64:4:2 64:4:4"}
timeout -k 10 500 python -u -m pytest "$R/tests/test_gpu_parity.py" -k "sgbm" -x -v --timeout 200 --timeout-method thread > "$R/gpurun_out/sweep_tests.txt" 2>&1 || { echo "sgbm tests failed rc=$?"; tail -30 "$R/gpurun_out/sweep_tests.txt"; exit 1; }
tail -2 "$R/gpurun_out/sweep_tests.txt"
for c in $CFGS; do
  IFS=: read -r cb pf ch <<< "$c"
  FVO_SG_CB=$cb FVO_SG_PF=$pf FVO_SG_CHUNKS=$ch timeout -k 10 300 python -u "$R/bench.py" --steps 5 --warmup 2 --ate-frames 0 --cpu-frames 0 > "$R/gpurun_out/sweep_$c.json" 2> "$R/gpurun_out/sweep_$c.err" || { echo "bench failed $c"; tail -20 "$R/gpurun_out/sweep_$c.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'vert', s.get('sgbm_vert'), 'horiz', s.get('sgbm_horiz'), 'med', s.get('sgbm_median'))" "$R/gpurun_out/sweep_$c.json" "$c"
done
echo done
