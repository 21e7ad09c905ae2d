set -uo pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/all_t.txt 2>&1; tail -3 gpurun_out/all_t.txt
timeout -k 10 600 python -u bench.py --width 1920 --height 1080 --nfeatures 2000 --ba-window 20 --batch 32 --steps 5 --warmup 2 --ate-frames 100 --cpu-frames 2 --ba-max-landmarks 8192 --ba-max-obs 65536 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo c5 fail; tail -20 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
