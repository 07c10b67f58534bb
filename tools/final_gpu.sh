#!/bin/bash
# End-of-round GPU record (development): GPU suite, smoke, bench lines (C3 default, e2e, sample_depth), profiles.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-200 $O/bench_c3.json
timeout -k 10 300 python bench.py --e2e --steps 30 --warmup 5 > $O/bench_e2e.json 2> $O/bench_e2e.err || exit 1
cut -c1-200 $O/bench_e2e.json
SAMPLE_STATS=1 timeout -k 10 200 python tools/bench_sample.py 30 > $O/sample.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/sample.txt | cut -c1-200
bash tools/profile.sh r6fin > $O/prof.txt 2>&1 || { tail -5 $O/prof.txt; exit 1; }
echo profiled
