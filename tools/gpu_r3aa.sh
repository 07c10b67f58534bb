#!/bin/bash
# round 3: the SH 3 + SG 7 forward preprocess with its colour rows staged through LDS by LDS-DMA (default,
# one-wave blocks) vs per-lane row loads (prenostage): SG / C5 parity, C5 lines
set -o pipefail
OUT=gpurun_out/r3aa
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py -x -q --timeout 300 --timeout-method thread -k "sg or c5 or small or yardstick or sample" > $OUT/parity.log 2>&1
rc=$?; tail -2 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/prenostage.so default ab_libs/prenostage.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C5 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('C5 $lib', d['value'], 'preprocess', s['preprocess'])"
done
