#!/bin/bash
# round 3: contract/fixture GPU tests, then the per-gradient GPU-vs-oracle report (small, C3, C5)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_ssim.py tests/test_gpu_depth_normal.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -3 gpurun_out/r3a_tests.log
timeout -k 10 900 python -u tools/dbg/grad_report.py small c3 c5 > gpurun_out/grad_report.log 2>&1
rc=$?
tail -8 gpurun_out/grad_report.log
exit $rc
