#!/bin/bash
# round 3: depth-sort tile shapes (threads x keys per lane) against 1024 x 4 (default): sort tests per build,
# depth_order stage at C3 / C5; then a HIP runtime-API trace of the C3 step (the host path between the K
# readback and the tile-list launches)
set -o pipefail
OUT=gpurun_out/r3w
mkdir -p $OUT
for lib in default ab_libs/t512i8.so ab_libs/t1024i8.so ab_libs/t512i16.so ab_libs/t256i16.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "depth_ties or depth_sort" > $OUT/sort_tests.log 2>&1
  rc=$?; echo "$lib sort tests: $(tail -1 $OUT/sort_tests.log)"; [ $rc -eq 0 ] || exit $rc
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'depth_order', s['depth_order'])"
  done
done
unset GSR_LIB
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $ROOT/$OUT/rt -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $ROOT/$OUT/rt.log 2>&1) || { tail -5 $OUT/rt.log; exit 1; }
ls $OUT/rt
