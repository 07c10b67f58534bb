#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats  2. --pmc FETCH_SIZE  3. --pmc WRITE_SIZE
#   4. --pmc SQ VALU instruction mix (all, transcendental, FMA/ADD/MUL f32, int32) and VALU cycles
#   4b. --pmc SQ wave / wait cycles, SALU / LDS instructions, LDS-array cycles and bank conflicts
#   5. --pmc L2 requests / busy / tag stalls / hits   6. --pmc TA busy
#   7. kernel trace + stats of tools/bench_sample.py (sample_depth kernels; default workload only)
# (counters in their own passes; never combined with other trace domains).
# Output: gpurun_out/prof_<tag>/..., summarised by tools/pmc_summary.py.
#   bash tools/profile.sh <tag> [bench.py workload args, e.g. --config C5 | --no-depth]
# (the sample_depth pass runs only for the default workload)
set -o pipefail
TAG=${1:-r1}
shift
WL="$*"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# an SQ pass whose counter set the profiler rejects (exit 1) is recorded and skipped; a time limit,
# abort or crash (any other status) stops the script
soft() { if [ "$1" -eq 1 ]; then echo "pass failed (status 1), skipped" >&2; return 0; fi; return "$1"; }
BENCH="$ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline $WL"
SHORT="$ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --stage-steps 1 $WL"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $SHORT > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $SHORT > $OUT/write.log 2>&1 && \
{ timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $SHORT > $OUT/sq.log 2>&1; soft $?; } && \
{ timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 $SHORT > $OUT/sq2.log 2>&1; soft $?; } && \
timeout -k 10 300 rocprofv3 --pmc TCC_REQ_sum TCC_BUSY_avr TCC_TAG_STALL_sum TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tcc -o run -- python3 $SHORT > $OUT/tcc.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta -o run -- python3 $SHORT > $OUT/ta.log 2>&1 && \
if [ -z "$WL" ]; then timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sample -o run -- python3 $ROOT/tools/bench_sample.py 10 > $OUT/sample.log 2>&1; fi
rc=$?
cd $ROOT
find $OUT -name "*.csv" | head -20
exit $rc
