#!/bin/bash
# One rocprofv3 --pmc pass over bench.py (GPU box, repo root): bash tools/pmc_one.sh OUTDIR COUNTER...
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc.log 2>&1
