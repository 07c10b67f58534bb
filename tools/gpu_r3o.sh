#!/bin/bash
# round 3: whole-workgroup tile emission (tiles_emit_coop_kernel, default) vs the single-wave emission
# (ab_libs/wide.so) and 256 blocks per XCD (ab_libs/coop256.so): list parity, stage medians at C3
# and C5, WRITE_SIZE of the list kernels at C3
set -o pipefail
OUT=gpurun_out/r3o
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "binning or lists or c3_full or c2_forward or ties or small or long" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
for lib in default ab_libs/wide.so ab_libs/coop256.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]); print('C5 $lib', d['value'], {k:v for k,v in d['roofline']['stage_ms'].items() if v})"
  n=$(basename $lib .so)
  bash tools/pmc_one.sh r3o/w_$n WRITE_SIZE || exit 1
done
unset GSR_LIB
for f in $OUT/w_*/run_counter_collection.csv; do python3 -c "
import csv, collections
t=collections.defaultdict(float); n=collections.defaultdict(set)
for r in csv.DictReader(open('$f')):
    k=r['Kernel_Name'].split('(')[0][-30:]
    if 'tiles_' in k or 'rows_' in k:
        t[k]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
print('$f', {k: round(v/len(n[k])) for k,v in t.items()})"; done
