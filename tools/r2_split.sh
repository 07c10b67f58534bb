# render_fwd time split (GSR_OPT_BISECT_PASSES = -1 composite only, 1 = probe walk only) + render stats at C3
set -o pipefail
mkdir -p gpurun_out
for v in -1 1; do
  timeout -k 10 120 python tools/ab_option.py 2 $v 10 > gpurun_out/split_$v.log 2>&1 || exit 1
done
grep -h render_fwd gpurun_out/split_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['option'], d['value'], d['stage_ms_median'].get('render_fwd'))"
timeout -k 10 120 python tools/render_stats.py
