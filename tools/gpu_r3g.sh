#!/bin/bash
# round 3: the whole GPU suite + smoke (after the A/B retirement)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -s > gpurun_out/r3g_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3g_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g_smoke.log 2>&1
rc2=$?; tail -4 gpurun_out/r3g_smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
