#!/bin/bash
# Round-4 check after the plane/MFMA pruning: every GPU test, smoke(), the
# NTT workload and the poly-mul bench (each step under its own limit).
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --workload ntt --no-cpu-baseline > $O/ntt.json 2> $O/ntt.err || { echo "ntt rc=$?"; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/polymul.json 2> $O/polymul.err || { echo "polymul rc=$?"; exit 1; }
python3 -c "
import json
for f in ('ntt','polymul'):
    d=json.loads(open('$O/'+f+'.json').read().splitlines()[-1])
    print(f, round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],3) for k,v in d['roofline'].get('kernels',{}).items()}, d.get('power'))
"
