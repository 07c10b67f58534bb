#!/bin/bash
# round 3: render_fwd with the spill-free median-depth phases: forward parity
# (render, sample, query paths), stage A/B against the previous kernel
# (ab_libs/fwd_orig.so), and one WRITE_SIZE pass of each.
set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -q -k "not c5" --timeout 300 --timeout-method thread > gpurun_out/r3h/parity.log 2>&1
rc=$?; tail -4 gpurun_out/r3h/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh 10 || exit 1
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for lib in default fwd_orig; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$ROOT/ab_libs/$lib.so; fi
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/r3h/write_$lib -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --stage-steps 1 > $ROOT/gpurun_out/r3h/write_$lib.log 2>&1 || exit 1
done
echo done
