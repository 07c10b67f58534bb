#!/bin/bash
# round 3 final check: full GPU suite, smoke, bench lines for every workload (C3 with its CPU baseline,
# C3 without depth, C2 forward, C5), rocprofv3 passes for C3 and C5 at this build
set -o pipefail
OUT=gpurun_out/r3y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --no-depth > $OUT/bench_c3_nodepth.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config C2 > $OUT/bench_c2.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config C5 --steps 20 --warmup 5 > $OUT/bench_c5.log 2>&1 || exit 1
for f in c3 c3_nodepth c2 c5; do tail -1 $OUT/bench_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['unit'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['bound'], d['roofline']['frac'], (d['roofline']['valu'] or {}).get('frac'))"; done
bash tools/profile.sh r3 > gpurun_out/prof_r3.log 2>&1 || { tail -5 gpurun_out/prof_r3.log; exit 1; }
bash tools/profile.sh r3_c5 --config C5 > gpurun_out/prof_r3_c5.log 2>&1 || exit 1
echo profiles done
