#!/bin/bash
# Whole-plane tensor/key-switch vs four-step at 2^10, 2^11, 2^13 by batch.
set -o pipefail
mkdir -p gpurun_out/ksw3
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-power "$@" > gpurun_out/ksw3/$tag.json 2> gpurun_out/ksw3/$tag.err || { echo "$tag rc=$?"; tail -5 gpurun_out/ksw3/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ksw3/$tag.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('$tag', round(d['value']), d['config'].get('parity_spot_check'), r.get('kernel'), r.get('frac') and round(r['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
}
for cfg in "13 8" "13 4" "11 4" "10 2"; do
  set -- $cfg
  for b in 1 64 1024; do
    for plane in 1 0; do
      RNT_PLANE=$plane run ct$1x$2_b${b}_p$plane --workload ctmul --log-n $1 --limbs $2 --ct-batch $b --steps 10 --warmup 3
    done
  done
done
