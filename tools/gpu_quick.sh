set -uo pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cv2_compat.py tests/test_ba.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pn_t.txt 2>&1; tail -3 gpurun_out/pn_t.txt
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-frames 0 > gpurun_out/pn_b.json 2> gpurun_out/pn_b.err || { tail -20 gpurun_out/pn_b.err; exit 1; }
cat gpurun_out/pn_b.json
