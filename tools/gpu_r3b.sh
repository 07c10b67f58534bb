#!/bin/bash
# round 3: view-exchange GPU tests, backward timing, small parity tests, then the
# GPU-vs-oracle gradient report with the injected forward state.
# A test assertion failure (pytest rc 1) lets the later steps run; anything else stops.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3b_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_pbwd.py C5 10 > gpurun_out/pbwd_c5.log 2>&1 || { tail -20 gpurun_out/pbwd_c5.log; exit 1; }
tail -1 gpurun_out/pbwd_c5.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "small or yardstick" --timeout 120 --timeout-method thread -s > gpurun_out/r3b_parity.log 2>&1
rc=$?; tail -5 gpurun_out/r3b_parity.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 1000 python -u tools/dbg/grad_report.py smallv c3 c5 > gpurun_out/grad_report2.log 2>&1
rc=$?
tail -4 gpurun_out/grad_report2.log
exit $rc
