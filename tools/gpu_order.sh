set -uo pipefail
mkdir -p gpurun_out
for v in "0" "1"; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --ate-frames 0 --cpu-frames 0 --sgbm-last $v > gpurun_out/ord_$v.json 2> gpurun_out/ord_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ord_$v.json'));print('$v',d['value'],d['ms_per_step'])"
done
FVO_SG_CHUNKS=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --ate-frames 0 --cpu-frames 0 --sgbm-last 1 > gpurun_out/ord_c2.json 2> gpurun_out/ord_c2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ord_c2.json'));print('c2',d['value'],d['ms_per_step'])"
