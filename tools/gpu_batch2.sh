#!/bin/bash
# frames-per-step sweep of the default bench (no ATE / CPU legs)
set -uo pipefail
mkdir -p gpurun_out
for b in 64 96 128; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --ate-frames 0 --cpu-frames 0 --batch $b > gpurun_out/batch_$b.json 2> gpurun_out/batch_$b.err || { tail -5 gpurun_out/batch_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/batch_$b.json'));print($b,d['value'],d['ms_per_step'],d.get('workspace_gb'))"
done
