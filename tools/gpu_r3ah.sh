#!/bin/bash
# round 3: tile ranges written by the coop emission kernel and the segment table built inside tiles_count (default) vs their own launches (prev):
# list / binning parity, C3 / C5 lines
set -o pipefail
OUT=gpurun_out/r3ah
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -x -q --timeout 300 --timeout-method thread -k "binning or lists or c3_full or c5 or c2_forward or ties or small or long or sample or query or integrate or sdf" > $OUT/parity.log 2>&1
rc=$?; tail -1 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/prev.so default ab_libs/prev.so default ab_libs/prev.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 40 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'tile_lists', s['tile_lists'])"
  done
done
