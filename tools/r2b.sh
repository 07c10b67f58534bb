set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_r2b.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r2b.log 2>&1 && tail -1 gpurun_out/bench_r2b.log | cut -c1-600
