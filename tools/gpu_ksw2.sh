#!/bin/bash
# Whole-plane tensor/key-switch vs four-step by batch: ct-mul at 2^14 x 8 and
# 2^12 x 4, default (whole where the picker takes it) vs RNT_PLANE=0.
set -o pipefail
mkdir -p gpurun_out/ksw2
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-power "$@" > gpurun_out/ksw2/$tag.json 2> gpurun_out/ksw2/$tag.err || { echo "$tag rc=$?"; tail -5 gpurun_out/ksw2/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ksw2/$tag.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('$tag', round(d['value']), d['config'].get('parity_spot_check'), r.get('kernel'), r.get('frac') and round(r['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
}
for b in 1 8 32 128 1024; do
  for plane in 1 0; do
    RNT_PLANE=$plane run ct14_b${b}_p$plane --workload ctmul --log-n 14 --limbs 8 --ct-batch $b --steps 10 --warmup 3
  done
done
for b in 1 32 256 1024; do
  for plane in 1 0; do
    RNT_PLANE=$plane run ct12_b${b}_p$plane --workload ctmul --log-n 12 --limbs 4 --ct-batch $b --steps 10 --warmup 3
  done
done
