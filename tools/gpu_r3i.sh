#!/bin/bash
# round 3 (re-entry): full GPU suite + smoke at HEAD, then the bench lines of
# every BASELINE.md measurement row (C3, C3 --no-depth, C2 forward-only, C5).
set -o pipefail
OUT=gpurun_out/r3i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 400 python bench.py --no-depth > $OUT/bench_c3_nodepth.json 2> $OUT/bench_c3_nodepth.err || exit 1
timeout -k 10 400 python bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 600 python bench.py --config C5 --steps 20 --warmup 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
for f in $OUT/bench_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], (d['cpu_baseline'] or {}).get('value'))"; done
# A/B against the previous library (ab_libs/base.so): C3 stage medians, then C5 bench lines
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
bash tools/c5_ab.sh > $OUT/ab_c5.txt 2>&1 || exit 1
cat $OUT/ab_c5.txt
