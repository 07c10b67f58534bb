#!/bin/bash
# round 3: forward LPT tile order for grids of <= 4096 tiles (default) vs none (nolpt): the full GPU suite
# (every small parity case now runs the ordered forward), then C2 forward and C3 lines
set -o pipefail
OUT=gpurun_out/r3u
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/nolpt.so default ab_libs/nolpt.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C2 C3; do
    timeout -k 10 200 python bench.py --config $wl --steps 50 --warmup 10 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_fwd', s['render_fwd'])"
  done
done
