#!/bin/bash
# NTT-path check: the 2^16 transform parity tests, then the NTT workload
# bench twice (with power), each step under its own limit.
set -o pipefail
O=gpurun_out/nttq; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_plane_ntt.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload ntt --no-cpu-baseline > $O/ntt_$i.json 2> $O/ntt_$i.err || { echo "ntt rc=$?"; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/ntt_$i.json').read().splitlines()[-1])
print('ntt', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],3) for k,v in d['roofline'].get('kernels',{}).items()}, (d.get('power') or {}).get('package_w_median'), (d.get('power') or {}).get('sclk_mhz_median'))
"
done
