#!/bin/bash
# round 3: backward splat loop unrolled by 2 (bwdu2) vs not (default): parity of the backward, C3 / C5 / no-depth
set -o pipefail
OUT=gpurun_out/r3ac
mkdir -p $OUT
export GSR_LIB=$(pwd)/ab_libs/bwdu2.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "small or clamp or warm or yardstick or c3_full" > $OUT/parity.log 2>&1
rc=$?; tail -1 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/bwdu2.so default ab_libs/bwdu2.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in "--config C3" "--config C5" "--no-depth"; do
    timeout -k 10 200 python bench.py $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_bwd', s['render_bwd'])"
  done
done
