#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, rocprof summaries.
#   gpurun -- 'bash tools/gpu_check.sh <tag> [tests|bench|prof ...]'
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}; shift || true
STEPS=${*:-tests bench prof}
mkdir -p "$R/gpurun_out"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 500 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 120 --timeout-method thread > "$R/gpurun_out/gpu_tests_$TAG.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$R/gpurun_out/gpu_tests_$TAG.log"; exit 1; } ;;
    bench) timeout -k 10 400 python -u "$R/bench.py" > "$R/gpurun_out/bench_$TAG.json" 2> "$R/gpurun_out/bench_$TAG.err" || { echo "bench failed rc=$?"; tail -30 "$R/gpurun_out/bench_$TAG.err"; exit 1; } ; cat "$R/gpurun_out/bench_$TAG.json" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    prof) bash "$R/profiles/collect.sh" "$TAG" || { echo "prof failed"; exit 1; } ;;
  esac
done
tail -3 "$R/gpurun_out/gpu_tests_$TAG.log" 2>/dev/null
echo done
