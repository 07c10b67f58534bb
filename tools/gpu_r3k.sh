#!/bin/bash
# round 3: compacted phase-3 fallback in render_fwd: parity (C2/C3 refinement vs the
# reference passes, small-scene suites), counters, and C2 / C3 A/B against
# ab_libs/base.so (previous) and ab_libs/hn2.so (looser conditioning threshold)
set -o pipefail
OUT=gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "c2 or refinement or small or long or stats" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/render_stats.py 100000 800 800 > $OUT/stats_c2.txt 2>&1 || exit 1
cat $OUT/stats_c2.txt
for lib in default ab_libs/base.so ab_libs/hn2.so default ab_libs/base.so ab_libs/hn2.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 10 --no-cpu-baseline > $OUT/c2.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/c2.log').read().strip().splitlines()[-1]); print('C2 $lib', d['value'], {k:v for k,v in d['roofline']['stage_ms'].items() if v})"
done
unset GSR_LIB
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
