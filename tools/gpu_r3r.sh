#!/bin/bash
# round 3: the N > 1 path rehearsed with two ranks sharing the one GPU (gloo): the two-rank exchange test
# through the HIP backward, then bench.py under torchrun with each exchange form
set -o pipefail
OUT=gpurun_out/r3r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/dist.log 2>&1
rc=$?; tail -15 $OUT/dist.log; [ $rc -eq 0 ] || exit $rc
for ex in overlap factored allreduce; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --exchange $ex > $OUT/bench2_$ex.log 2>&1 || { tail -30 $OUT/bench2_$ex.log; exit 1; }
  grep '^{' $OUT/bench2_$ex.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ex', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['workload'], d['config']['parallelism'])"
done
# forward LPT tile order (global, and heaviest-first within each XCD's region) vs the XCD-contiguous default
for lib in default ab_libs/fwdlpt.so ab_libs/fwdlpt_xcd.so default ab_libs/fwdlpt.so ab_libs/fwdlpt_xcd.so; do
  if [ "$lib" = default ]; then unset GSR_LIB; else export GSR_LIB=$(pwd)/$lib; fi
  for wl in C3 C5; do
    timeout -k 10 200 python bench.py --config $wl --steps 30 --warmup 5 --no-cpu-baseline > $OUT/lpt.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/lpt.log').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$wl $lib', d['value'], 'render_fwd', s['render_fwd'], 'tile_lists', s['tile_lists'])"
  done
done
