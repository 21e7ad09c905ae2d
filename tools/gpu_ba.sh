set -uo pipefail
timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_t.txt 2>&1; tail -3 gpurun_out/ba_t.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --ate-frames 0 --cpu-frames 0 > gpurun_out/ba_b.json 2> gpurun_out/ba_b.err || { tail -20 gpurun_out/ba_b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ba_b.json')); print(d['value'], d['stages_ms_per_step'])"
timeout -k 10 400 python -u bench.py --width 1920 --height 1080 --nfeatures 2000 --ba-window 20 --batch 32 --steps 5 --warmup 2 --ate-frames 0 --cpu-frames 0 --ba-max-landmarks 8192 --ba-max-obs 65536 > gpurun_out/ba_c5.json 2> gpurun_out/ba_c5.err || { tail -20 gpurun_out/ba_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ba_c5.json')); print(d['value'], d['stages_ms_per_step'])"
