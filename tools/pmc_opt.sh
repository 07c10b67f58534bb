#!/bin/bash
# One rocprofv3 --pmc pass over tools/run_opt.py (GPU box, repo root): bash tools/pmc_opt.sh OUTDIR OPT VAL COUNTER...
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$1
OPT=$2
VAL=$3
shift 3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o run -- python3 $ROOT/tools/run_opt.py $OPT $VAL 3 > $OUT/pmc.log 2>&1
