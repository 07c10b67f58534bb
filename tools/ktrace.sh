#!/bin/bash
# Quick per-kernel look (development): kernel trace + stats, then one --pmc
# pass with the counters given as arguments (default WRITE_SIZE FETCH_SIZE
# are separate passes in profile.sh; this takes one counter list).
# Usage (GPU box, repo root): bash tools/ktrace.sh OUTDIR [COUNTER ...]
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-kt}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
if [ $# -gt 0 ]; then
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc.log 2>&1 || exit $?
fi
