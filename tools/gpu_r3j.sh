#!/bin/bash
# round 3: render_fwd counters at C3 and C2; A/B of the preprocess row records
# (default vs ab_libs/norowrec.so vs ab_libs/base.so) at C3 and C5.
set -o pipefail
OUT=gpurun_out/r3j
mkdir -p $OUT
timeout -k 10 200 python tools/render_stats.py > $OUT/stats_c3.txt 2>&1 || exit 1
timeout -k 10 200 python tools/render_stats.py 100000 800 800 > $OUT/stats_c2.txt 2>&1 || exit 1
cat $OUT/stats_c3.txt $OUT/stats_c2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py -x -q --timeout 300 --timeout-method thread -k "not c5" > $OUT/parity.log 2>&1
rc=$?; tail -2 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh 10 > $OUT/ab_c3.txt 2>&1 || exit 1
cat $OUT/ab_c3.txt
AB_LIB=ab_libs/norowrec.so bash tools/c5_ab.sh > $OUT/ab_c5.txt 2>&1 || exit 1
cat $OUT/ab_c5.txt
