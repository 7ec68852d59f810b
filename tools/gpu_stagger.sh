#!/bin/bash
# Whole-plane kernels: first-wave stagger sweep (RNT_PLANE_STAGGER, 100 MHz ticks), same box.
mkdir -p gpurun_out
export TMPDIR=/tmp RNT_PLANE=1
for i in 1 2; do
  for v in ${STAGGERS:-0 1000 2000 4000}; do
    RNT_PLANE_STAGGER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/st${v}_$i.json 2> gpurun_out/st${v}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/st${v}_$i.json').read().splitlines()[-1]);print('stagger=$v', round(d['value']), d['config']['parity_spot_check'], {k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()}, d['power'])"
  done
done
