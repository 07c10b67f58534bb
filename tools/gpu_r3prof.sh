#!/bin/bash
# round 3: rocprofv3 passes (tools/profile.sh) for every bench workload: C3, C3 --no-depth, C2, C5
set -o pipefail
bash tools/profile.sh r3 > gpurun_out/prof_r3.log 2>&1 || { tail -5 gpurun_out/prof_r3.log; exit 1; }
bash tools/profile.sh r3_nodepth --no-depth > gpurun_out/prof_r3_nodepth.log 2>&1 || exit 1
bash tools/profile.sh r3_c2 --config C2 > gpurun_out/prof_r3_c2.log 2>&1 || exit 1
bash tools/profile.sh r3_c5 --config C5 > gpurun_out/prof_r3_c5.log 2>&1 || exit 1
echo profiles done
