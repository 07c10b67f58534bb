#!/bin/bash
# Development A/B of library builds at C2 (forward-only) and C3: bench.py's per-launch stage times for the
# default lib and each ab_libs/*.so.  bash tools/ab_c2.sh [steps]
set -o pipefail
S=${1:-50}
for lib in default ab_libs/*.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for cfg in C2 C3; do
    timeout -k 10 300 python bench.py --config $cfg --steps $S --warmup 5 --no-cpu-baseline > gpurun_out/abc2.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/abc2.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib $cfg', d['ms_per_step'], d.get('stage_ms')); break"
  done
done
