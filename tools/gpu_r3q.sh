#!/bin/bash
# round 3: rows pass gathering the preprocess's footprint record, rows-pass record prefetch, tiles pass with
# the LDS segment table + next-segment prefetch + double-buffered masks (default build), against HEAD
# (ab_libs/base.so) and 128/256-Gaussian row segments above 2M Gaussians (big128/big256): list parity,
# C3 stage medians, C5 bench lines, per-kernel traces and WRITE_SIZE at C3; then the full GPU suite,
# smoke and the C3 bench line
set -o pipefail
OUT=gpurun_out/r3q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py tests/test_gpu_query.py -x -q --timeout 300 --timeout-method thread -k "binning or lists or c3_full or c2_forward or ties or small or long or sample or query or integrate or sdf" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
for lib in default ab_libs/base.so ab_libs/big128.so ab_libs/big256.so default; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]); print('C5 $lib', d['value'], {k:v for k,v in d['roofline']['stage_ms'].items() if v})"
done
unset GSR_LIB
ROOT=$(pwd)
for wl in C3 C5; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/kt_$wl/trace -o run -- python3 $ROOT/bench.py --config $wl --steps 10 --warmup 3 --no-cpu-baseline > $ROOT/$OUT/kt_$wl.log 2>&1) || exit 1
  python3 tools/kreport.py $OUT/kt_$wl 14
done
bash tools/pmc_one.sh r3q/w_c3 WRITE_SIZE || exit 1
bash tools/pmc_one.sh r3q/f_c3 FETCH_SIZE || exit 1
for f in $OUT/w_c3/run_counter_collection.csv $OUT/f_c3/run_counter_collection.csv; do python3 -c "
import csv, collections
t=collections.defaultdict(float); n=collections.defaultdict(set)
for r in csv.DictReader(open('$f')):
    k=r['Kernel_Name'].split('(')[0][-30:]
    if 'tiles_' in k or 'rows_' in k or 'preprocess_fwd' in k:
        t[k]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
print('$f KiB', {k: round(v/len(n[k])) for k,v in t.items()})"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log
