#!/bin/bash
# round 3: rows_emit single-chunk path (default: running slots read from the scan directly, no LDS staging
# or ping-pong) vs the chunked path (chunks): list parity, C3 / C5 lines, per-kernel trace at C5
set -o pipefail
OUT=gpurun_out/r3z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -x -q --timeout 300 --timeout-method thread -k "binning or lists or c3_full or c5 or c2_forward or ties or small or long or sample or query or integrate or sdf" > $OUT/parity.log 2>&1
rc=$?; tail -2 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/chunks.so default ab_libs/chunks.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'tile_lists', s['tile_lists'])"
  done
done
unset GSR_LIB
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/kt_C5/trace -o run -- python3 $ROOT/bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline > $ROOT/$OUT/kt_C5.log 2>&1) || exit 1
python3 tools/kreport.py $OUT/kt_C5 12
