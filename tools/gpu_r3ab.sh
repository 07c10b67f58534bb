#!/bin/bash
# round 3: tiles-pass launch sizes: coop emission blocks per XCD 64 / 192 (default 128), tiles_count blocks
# 4096 / 16384 (default 8192): C3 / C5 tile_lists
set -o pipefail
OUT=gpurun_out/r3ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "binning or lists" > $OUT/parity.log 2>&1
rc=$?; tail -1 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/coop64.so ab_libs/coop192.so ab_libs/tb4k.so ab_libs/tb16k.so default ab_libs/coop64.so ab_libs/coop192.so ab_libs/tb4k.so ab_libs/tb16k.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'tile_lists', s['tile_lists'])"
  done
done
