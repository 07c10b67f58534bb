#!/bin/bash
# round 3: backward raster skipping the pixel pair (tile half) with no valid pixel in the wave (default)
# vs every pair always (noskip): parity suite, C3 / C5 lines
set -o pipefail
OUT=gpurun_out/r3v
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/noskip.so default ab_libs/noskip.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 40 --warmup 10 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_bwd', s['render_bwd'])"
  done
  timeout -k 10 200 python bench.py --no-depth --steps 40 --warmup 10 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('C3-nodepth $lib', d['value'], 'render_bwd', s['render_bwd'])"
done
