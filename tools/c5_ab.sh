set -o pipefail
mkdir -p gpurun_out
for lib in default ${AB_LIB:-ab_libs/base.so} default ${AB_LIB:-ab_libs/base.so}; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  timeout -k 10 200 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/c5.log').read().strip().splitlines()[-1]); print('$lib', d['value'], {k:v for k,v in d['roofline']['stage_ms'].items() if v})"
done
