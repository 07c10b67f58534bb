#!/bin/bash
# round 3: composite with the lazy m0 / word-boundary mask flush (ab_libs/lazy1.so): parity with that
# library, then C3 and C2 A/B against the default (GSR_COMP_LAZY 0)
set -o pipefail
OUT=gpurun_out/r3m
mkdir -p $OUT
GSR_LIB=$(pwd)/ab_libs/lazy1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -x -q --timeout 300 --timeout-method thread -k "not c5" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/lazy1.so default ab_libs/lazy1.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 10 --no-cpu-baseline > $OUT/c2.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/c2.log').read().strip().splitlines()[-1]); print('C2 $lib', d['value'], {k:v for k,v in d['roofline']['stage_ms'].items() if v})"
done
unset GSR_LIB
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
bash tools/ab_libs.sh 10 > $OUT/ab_c3b.txt 2>&1 || exit 1
cat $OUT/ab_c3b.txt
