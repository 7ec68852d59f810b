#!/bin/bash
# k_ks_rows A/B against the `split` variant, plus the key-switch and 2^16
# transform parity tests (each GPU step under its own limit).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_plane_ntt.py -x -q -k "keyswitch or config5 or forward or inverse or cross or rescale" --timeout 300 --timeout-method thread > gpurun_out/ks2_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/ks2_pytest.log; exit 1; }
tail -2 gpurun_out/ks2_pytest.log
AB_TAG=r2rot1_ BENCH_ARGS="--workload rotate --rot-batch 1 --steps 10 --warmup 2" bash tools/ab.sh 2 base split || exit 1
AB_TAG=r2ct1_ BENCH_ARGS="--workload ctmul --ct-batch 1 --steps 40 --warmup 5" bash tools/ab.sh 1 base split || exit 1
timeout -k 10 200 python bench.py --workload ntt --no-cpu-baseline > gpurun_out/ntt_recomb.json 2>/dev/null || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/ntt_recomb.json').read().splitlines()[-1])
print('ntt', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()}, (d.get('power') or {}).get('package_w_median'))"
