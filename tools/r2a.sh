set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
bash tools/profile.sh r2
rc=$?
tail -3 gpurun_out/smoke.log; tail -8 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench.log
exit $rc
