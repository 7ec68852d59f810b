#!/bin/bash
# W16 only in k_mf_tensor: tensor full-output stress, the 2^16 parity
# files, then ct-mul and NTT bench lines.
set -o pipefail
mkdir -p gpurun_out/mft3
timeout -k 10 400 python3 tools/tensor_stress2.py 4 64 > gpurun_out/mft3/stress2.log 2>&1 || { echo "stress rc=$?"; cut -c1-200 gpurun_out/mft3/stress2.log | tail; exit 1; }
grep -c equal gpurun_out/mft3/stress2.log
timeout -k 10 300 python3 tools/ntt_stress.py 4 128 > gpurun_out/mft3/ntt_stress.log 2>&1 || { echo "ntt stress rc=$?"; tail gpurun_out/mft3/ntt_stress.log; exit 1; }
grep -c " 0 words" gpurun_out/mft3/ntt_stress.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_plane_ntt.py tests/test_gpu_configs.py tests/test_sharded.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mft3/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/mft3/pytest.log; exit 1; }
tail -1 gpurun_out/mft3/pytest.log
for w in "ctmul --steps 6 --warmup 2" "ntt --steps 20 --warmup 3" "ctmul --steps 6 --warmup 2" "ntt --steps 20 --warmup 3"; do
  set -- $w; tag=$1$RANDOM
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-power --workload $w > gpurun_out/mft3/$tag.json 2> gpurun_out/mft3/$tag.err || { echo "$tag rc=$?"; tail -5 gpurun_out/mft3/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/mft3/$tag.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('$1', round(d['value']), d['config'].get('parity_spot_check'), r.get('frac') and round(r['frac'],3), {n:(v['launches'],round(v['avg_ms'],4)) for n,v in k.items()})
"
done
