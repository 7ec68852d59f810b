#!/bin/bash
# Whole-plane key-switch check: every GPU test, then same-box ct-mul and
# rotation bench lines at 2^14 x 8 (config 3) and 2^12 x 4, default vs
# RNT_PLANE=0 (the four-step key-switch), each step under its own limit.
set -o pipefail
mkdir -p gpurun_out/ksw
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ksw/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/ksw/pytest.log; exit 1; }
tail -2 gpurun_out/ksw/pytest.log
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-power "$@" > gpurun_out/ksw/$tag.json 2> gpurun_out/ksw/$tag.err || { echo "$tag rc=$?"; tail -5 gpurun_out/ksw/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ksw/$tag.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$tag', round(d['value']), d['unit'], d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
}
for plane in 1 0; do
  export RNT_PLANE=$plane
  run ct14_p$plane --workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 5 --warmup 2
  run ct12_p$plane --workload ctmul --log-n 12 --limbs 4 --ct-batch 1024 --steps 5 --warmup 2
  run ct14b1_p$plane --workload ctmul --log-n 14 --limbs 8 --ct-batch 1 --steps 40 --warmup 5
done
