#!/bin/bash
# round 3: render_fwd knobs re-swept at the final layout: composite batch 64 / 256 (default 128), resident
# cache 320 (default 256), 5 waves per SIMD (default 6): C3 / C2 lines (parity of each build first)
set -o pipefail
OUT=gpurun_out/r3ae
mkdir -p $OUT
for lib in ab_libs/b64.so ab_libs/b256.so ab_libs/r320.so ab_libs/w5.so; do
  export GSR_LIB=$(pwd)/$lib
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "small or long or clamp" > $OUT/parity.log 2>&1
  rc=$?; echo "$lib $(tail -1 $OUT/parity.log)"; [ $rc -eq 0 ] || exit $rc
done
for lib in default ab_libs/b64.so ab_libs/b256.so ab_libs/r320.so ab_libs/w5.so default ab_libs/b64.so ab_libs/b256.so ab_libs/r320.so ab_libs/w5.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C2; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_fwd', s['render_fwd'])"
  done
done
