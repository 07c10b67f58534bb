#!/bin/bash
# One GPU session: build check, smoke, parity check, bench.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python tools/gpu_check.py > gpurun_out/check.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/smoke.log; tail -60 gpurun_out/check.log; tail -3 gpurun_out/bench.log
exit $rc
