set -o pipefail
mkdir -p gpurun_out/r6jj
for r in 1 2; do
for lib in default ab_libs/*.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python tools/bench_optim.py > gpurun_out/r6jj/o.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/r6jj/o.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$lib', d['fused_event_ms'], d['fused_GBps'], flush=True)"
done
done
unset GSR_LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_optim.py > gpurun_out/r6jj/t.log 2>&1; tail -2 gpurun_out/r6jj/t.log
