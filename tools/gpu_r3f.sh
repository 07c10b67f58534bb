#!/bin/bash
# round 3: preprocess_bwd staged rows with LDS-DMA lobe loads: parity, then A/B of the staged kernel's occupancy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "row_store or small" --timeout 120 --timeout-method thread > gpurun_out/r3f_parity.log 2>&1
rc=$?; tail -4 gpurun_out/r3f_parity.log; [ $rc -eq 0 ] || exit $rc
for lib in default ab_libs/dma2.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for cfg in C5 C3; do
    timeout -k 10 300 python -u tools/bench_pbwd.py $cfg 10 > gpurun_out/pbwd.log 2>&1 || { tail -20 gpurun_out/pbwd.log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/pbwd.log)"
  done
done
bash tools/ab_libs.sh 10
