#!/bin/bash
# round 3: is render_bwd bound by its L2 atomics? timing-only build with plain stores (ab_libs/bwdstores.so)
set -o pipefail
OUT=gpurun_out/r3s
mkdir -p $OUT
for lib in default ab_libs/bwdstores.so default ab_libs/bwdstores.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_bwd', s['render_bwd'], 'preprocess_bwd', s['preprocess_bwd'])"
  done
done
