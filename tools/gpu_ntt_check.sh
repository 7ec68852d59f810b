#!/bin/bash
# Whole-plane standalone transforms: every GPU test (the NTT at N = 2^16
# feeds most of them), then the NTT workload with the plane kernels (default)
# and the four-step ones (RNT_PLANE=0) alternately, and the default poly-mul.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out
for i in 1 2; do
  for v in 3 0; do
    RNT_PLANE=$v timeout -k 10 200 python bench.py --workload ntt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ntt_plane${v}_$i.json 2> gpurun_out/ntt_plane${v}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ntt_plane${v}_$i.json').read().splitlines()[-1]);print('RNT_PLANE=$v', round(d['value']), d['config'].get('parity_spot_check'), {k:round(v['avg_ms'],3) for k,v in d['roofline'].get('kernels',{}).items()}, d.get('power'))"
  done
done
