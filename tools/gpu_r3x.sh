#!/bin/bash
# round 3: depth-sort tiles of 1024 x 8 keys (default) vs x4 (before), x12, x16 (sort tests per build);
# count/histogram grid of 512 / 1024 blocks (kh512, kh1024) vs 256; the SH 3 + SG 7 preprocess at 3 waves per
# SIMD (pre3w, 20 VGPRs spilled) vs 2: C3 / C5 lines; then the full GPU suite and smoke on the default build
set -o pipefail
OUT=gpurun_out/r3x
mkdir -p $OUT
for lib in default ab_libs/t1024i12.so ab_libs/t1024i16.so ab_libs/kh512.so ab_libs/kh1024.so ab_libs/pre3w.so default ab_libs/kh512.so ab_libs/kh1024.so ab_libs/pre3w.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "depth_ties or depth_sort" > $OUT/sort_tests.log 2>&1
  rc=$?; echo "$lib sort tests: $(tail -1 $OUT/sort_tests.log)"; [ $rc -eq 0 ] || exit $rc
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'depth_order', s['depth_order'], 'scan', s['scan'], 'preprocess', s['preprocess'])"
  done
done
unset GSR_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
