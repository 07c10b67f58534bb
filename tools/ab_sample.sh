#!/bin/bash
# Development A/B of library builds on the sample bench: sample_fwd / sample_bwd per-launch times for the default
# lib and each ab_libs/*.so, interleaved over R rounds.  bash tools/ab_sample.sh [rounds] [steps]
set -o pipefail
R=${1:-2}
S=${2:-30}
for r in $(seq $R); do
  for lib in default ab_libs/*.so; do
    if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
    timeout -k 10 200 python tools/bench_sample.py $S > gpurun_out/absample.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/absample.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib', d['ms_per_call'], d['stage_ms']['sample_fwd'], d['stage_ms']['sample_bwd'], flush=True); break"
  done
done
