#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg/md_clamp.py > gpurun_out/md_clamp.log 2>&1; rc=$?; cat gpurun_out/md_clamp.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_pbwd.py C5 10 > gpurun_out/pbwd_c5.log 2>&1 || { tail -20 gpurun_out/pbwd_c5.log; exit 1; }
tail -1 gpurun_out/pbwd_c5.log
timeout -k 10 300 python -u tools/bench_pbwd.py C3 20 > gpurun_out/pbwd_c3.log 2>&1 || { tail -20 gpurun_out/pbwd_c3.log; exit 1; }
tail -1 gpurun_out/pbwd_c3.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "row_store" --timeout 120 --timeout-method thread > gpurun_out/r3d_parity.log 2>&1
rc=$?; tail -5 gpurun_out/r3d_parity.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/dbg/c3_grad_detail.py c3 > gpurun_out/c3_detail.log 2>&1; rc=$?; tail -30 gpurun_out/c3_detail.log; exit $rc
