#!/bin/bash
# SGBM variant check: parity tests of SGBM under each env setting, then bench_sgbm per setting.
#   gpurun -- 'bash tools/gpu_sgv.sh <tag> "<env assignments per variant>" ...'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p "$R/gpurun_out"
for v in "$@"; do
  env $v timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_parity.py" "$R/tests/test_natural.py" -k "sgbm" -x -q --timeout 200 --timeout-method thread > "$R/gpurun_out/sgv_tests_$TAG.log" 2>&1 || { echo "sgbm tests failed: $v"; tail -30 "$R/gpurun_out/sgv_tests_$TAG.log"; exit 1; }
  echo "$v: $(tail -1 $R/gpurun_out/sgv_tests_$TAG.log)"
done
for v in "$@"; do
  env $v timeout -k 10 120 python -u "$R/tools/bench_sgbm.py" || { echo "bench_sgbm failed: $v"; exit 1; }
done
