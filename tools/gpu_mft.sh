#!/bin/bash
# The matrix-core tensor (k_mf_tensor): its parity tests and the ct-mul
# paths at 2^16 that run it, then same-box ct-mul A/B (config 4 shape) of
# this tree against the four-step tensor (the ks4 variant library).
set -o pipefail
mkdir -p gpurun_out/mft
timeout -k 10 600 python -u -m pytest tests/test_gpu_plane_ntt.py tests/test_gpu_configs.py tests/test_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mft/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/mft/pytest.log; exit 1; }
tail -1 gpurun_out/mft/pytest.log
for i in 1 2; do
  for v in base mft0; do
    lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = mft0 ] && lib=toy-heaan-ckks_amd/lib/variants/librnsntt_mft0.so
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --workload ctmul --steps 6 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/mft/$v$i.json 2> gpurun_out/mft/$v$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/mft/$v$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/mft/$v$i.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('$v$i', round(d['value']), d['config'].get('parity_spot_check'), {n:(v['launches'],round(v['avg_ms'],4)) for n,v in k.items()})
"
  done
done
