#!/bin/bash
# round 3: the §8(f) rows' timing tools at the final build (integrate / evaluate_sdf, distCUDA2, fused Adam,
# NCC, SSIM, depth->normal, sample_depth), one JSON line each into gpurun_out/r3ad/
set -o pipefail
OUT=gpurun_out/r3ad
mkdir -p $OUT
for t in bench_query bench_knn bench_optim bench_ncc bench_ssim bench_depth_normal bench_sample; do
  timeout -k 10 300 python tools/$t.py > $OUT/$t.json 2> $OUT/$t.err || { echo "$t failed"; tail -5 $OUT/$t.err; exit 1; }
  echo "== $t"; cat $OUT/$t.json | cut -c1-400
done
