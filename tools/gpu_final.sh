# Round-end evidence on the GPU box (tooling): the GPU test suite, smoke(), the default bench
# line (with the CPU baseline and ATE), the configs[4] line and the mono line, each under its own
# time limit, chained so that a failure stops the run.  -> gpurun_out/final/
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 400 python bench.py --width 1920 --height 1080 --nfeatures 2000 --ba-window 20 --batch 32 --ba-max-landmarks 8192 --ba-max-obs 65536 --cpu-frames 0 --ate-frames 0 > $O/bench_1080p.json 2> $O/bench_1080p.err || { tail -20 $O/bench_1080p.err; exit 1; }
timeout -k 10 300 python tools/bench_mono.py > $O/bench_mono.json 2> $O/bench_mono.err || { tail -20 $O/bench_mono.err; exit 1; }
for f in bench bench_1080p bench_mono; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d.get('value'), d.get('ms_per_step'))"; done
