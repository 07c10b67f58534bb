#!/bin/bash
# round 3 measurement record: bench lines for every BASELINE workload, then the
# rocprofv3 passes per workload (tools/profile.sh), all under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/r3
for wl in "C3:" "C3nd:--no-depth" "C2:--config C2" "C5:--config C5"; do
  name=${wl%%:*}; args=${wl#*:}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/r3/bench_$name.json 2> gpurun_out/r3/bench_$name.log || { tail -20 gpurun_out/r3/bench_$name.log; exit 1; }
  echo "$name: $(head -c 300 gpurun_out/r3/bench_$name.json)"
done
for wl in "r3:" "r3_nodepth:--no-depth" "r3_c2:--config C2" "r3_c5:--config C5"; do
  tag=${wl%%:*}; args=${wl#*:}
  bash tools/profile.sh $tag $args > gpurun_out/r3/profile_$tag.log 2>&1 || { tail -20 gpurun_out/r3/profile_$tag.log; exit 1; }
  echo "profiled $tag"
done
