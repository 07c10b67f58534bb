#!/bin/bash
# round 3: repeat C5 lines with the folded ranges / segment table (default) and without (prev), after one
# outlier line in r3ah; then the full GPU suite and smoke on the default
set -o pipefail
OUT=gpurun_out/r3ai
mkdir -p $OUT
for lib in default default ab_libs/prev.so default ab_libs/prev.so default; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C5 --steps 40 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('C5 $lib', d['value'], 'tile_lists', s['tile_lists'], 'render_fwd', s['render_fwd'])"
done
unset GSR_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_c3.log 2>&1 || exit 1
tail -1 $OUT/bench_c3.log | cut -c1-120
