#!/bin/bash
# BA iteration on the GPU box: BA parity tests, then the BA / PnP stage times (tools/bench_ba.py)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 300 python -u -m pytest "$R/tests/test_ba.py" -x -q --timeout 200 --timeout-method thread > "$R/gpurun_out/ba_tests.log" 2>&1 || { echo "ba tests failed"; tail -30 "$R/gpurun_out/ba_tests.log"; exit 1; }
tail -1 "$R/gpurun_out/ba_tests.log"
for i in 1 2 3; do timeout -k 10 120 python -u "$R/tools/bench_ba.py" || { echo "bench_ba failed"; exit 1; }; done
