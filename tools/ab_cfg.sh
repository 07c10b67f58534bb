#!/bin/bash
# Development A/B of library builds over bench.py configs: per-launch stage times for the default lib and each
# ab_libs/*.so, interleaved over R rounds.  bash tools/ab_cfg.sh R STEPS CFG... (CFG: C2 C3 C5 e2e)
set -o pipefail
R=$1; S=$2; shift 2
mkdir -p gpurun_out
for r in $(seq $R); do
  for lib in default ab_libs/*.so; do
    if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
    for cfg in "$@"; do
      if [ "$cfg" = e2e ]; then A="--e2e"; else A="--config $cfg"; fi
      timeout -k 10 300 python bench.py $A --steps $S --warmup 5 --no-cpu-baseline > gpurun_out/abcfg.log 2>&1 || exit 1
      python3 -c "
import json
for l in open('gpurun_out/abcfg.log'):
    if l.startswith('{'):
        d = json.loads(l); st = d.get('stage_ms') or d.get('roofline', {}).get('stage_ms') or d.get('roofline', {}).get('stage_ms_per_step')
        print('$lib $cfg', d['ms_per_step'], {k: v for k, v in (st or {}).items() if v}, d.get('components_ms', ''), flush=True); break"
    done
  done
done
