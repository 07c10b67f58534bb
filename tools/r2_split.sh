# render_fwd time split by median-depth stage (GSR_OPT_BISECT_PASSES = -1 composite only, 1, 2; NO_REFINE)
set -o pipefail
mkdir -p gpurun_out
for v in -1 1 2; do
  timeout -k 10 120 python tools/ab_option.py 2 $v 10 > gpurun_out/split_$v.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/ab_option.py 5 1 10 > gpurun_out/split_norefine.log 2>&1 || exit 1
grep -h render_fwd gpurun_out/split_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['option'], d['value'], d['stage_ms_median'].get('render_fwd'))"
