#!/bin/bash
# round 3: the staged per-Gaussian backward at 2 / 4 waves per SIMD (default 3): C5 / C3 lines
set -o pipefail
OUT=gpurun_out/r3ag
mkdir -p $OUT
for lib in ab_libs/pb2.so ab_libs/pb4.so; do
  export GSR_LIB=$(pwd)/$lib
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "small or sg or yardstick" > $OUT/parity.log 2>&1
  rc=$?; echo "$lib $(tail -1 $OUT/parity.log)"; [ $rc -eq 0 ] || exit $rc
done
for lib in default ab_libs/pb2.so ab_libs/pb4.so default ab_libs/pb2.so ab_libs/pb4.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C5 C3; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'preprocess_bwd', s['preprocess_bwd'])"
  done
done
