#!/bin/bash
# u64 four-step row product kernels (k_tensor_rows<uint64_t>) at two waves per SIMD
# VGPRs (variant u64t; they take 131-132 and run three waves per SIMD) vs
# this tree: u64 parity through the variant, then interleaved poly-mul lines
# at N = 2^16, 16 x 62-bit (the reference's u64 width at the metric ring).
set -o pipefail
mkdir -p gpurun_out/u64t
V=toy-heaan-ckks_amd/lib/variants/librnsntt_u64t.so
RNSNTT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_replays.py tests/test_gpu_whole.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/u64t/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/u64t/pytest.log; exit 1; }
tail -1 gpurun_out/u64t/pytest.log
for i in 1 2 3; do
  for v in base u64t; do
    lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = u64t ] && lib=$V
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --workload ctmul --log-n 13 --limbs 7 --prime-bits 61 --ct-batch 128 --steps 6 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/u64t/$v$i.json 2> gpurun_out/u64t/$v$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/u64t/$v$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/u64t/$v$i.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$v$i', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
  done
done
