#!/bin/bash
# Whole-plane row path (2^10 <= N <= 2^14): its GPU tests, then bench lines
# for the BASELINE configs' rings and the reference's u64 shapes (poly-mul
# and NTT workloads), each step under its own limit.
set -o pipefail
O=gpurun_out/whole; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_whole.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-power "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().splitlines()[-1])
print('$tag', round(d['value']), d['unit'], d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],4) for k,v in (d['roofline'].get('kernels') or {}).items()} if isinstance(d['roofline'].get('kernels'), dict) else '')
"
}
for plane in 1 0; do
  export RNT_PLANE=$plane
  run mul12_p$plane --log-n 12 --limbs 4 --batch 4096
  run ntt12_p$plane --workload ntt --log-n 12 --limbs 4 --batch 4096
  run mul14_p$plane --log-n 14 --limbs 8 --batch 1024
  run ntt14_p$plane --workload ntt --log-n 14 --limbs 8 --batch 1024
  run mul13u64_p$plane --log-n 13 --limbs 7 --prime-bits 61 --batch 1024
  run mul10u64_p$plane --log-n 10 --limbs 2 --prime-bits 62 --batch 16384
done
