#!/bin/bash
# u64 whole-plane product at 2^14 (variant u64w14, 12 B of spills a lane) vs the
# four-step u64 product (this tree) at N = 2^14, 3 x 61-bit (test ring)
# : parity through the variant, then interleaved lines.
set -o pipefail
mkdir -p gpurun_out/u64w14
V=toy-heaan-ckks_amd/lib/variants/librnsntt_u64w14.so
RNSNTT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_whole.py -m gpu -x -q -k "13-61 or 14-61" --timeout 200 --timeout-method thread > gpurun_out/u64w14/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/u64w14/pytest.log; exit 1; }
tail -1 gpurun_out/u64w14/pytest.log
for i in 1 2 3; do
  for v in base u64w14; do
    lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = u64w14 ] && lib=$V
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --log-n 14 --limbs 3 --prime-bits 61 --batch 1024 --steps 20 --warmup 3 --no-cpu-baseline --no-power > gpurun_out/u64w14/$v$i.json 2> gpurun_out/u64w14/$v$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/u64w14/$v$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/u64w14/$v$i.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$v$i', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
  done
done
