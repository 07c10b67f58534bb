#!/bin/bash
# Development A/B of library builds: stage medians of tools/ab_option.py for each ab_libs/*.so and the default lib.
# bash tools/ab_libs.sh [steps]
set -o pipefail
S=${1:-20}
for lib in default ab_libs/*.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python tools/ab_option.py 1 0 $S > gpurun_out/ablib.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/ablib.log'):
    if l.startswith('{\"option\"'):
        d = json.loads(l); print('$lib', {k: round(v, 4) for k, v in d['stage_ms_median'].items()}); break"
done
