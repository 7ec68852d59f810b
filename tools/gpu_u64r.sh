#!/bin/bash
# u64 four-step row product kernels (k_row<uint64_t, 2, 7..9>) capped at 128
# VGPRs (variant u64r; they take 131-132 and run three waves per SIMD) vs
# this tree: u64 parity through the variant, then interleaved poly-mul lines
# at N = 2^16, 16 x 62-bit (the reference's u64 width at the metric ring).
set -o pipefail
mkdir -p gpurun_out/u64r
V=toy-heaan-ckks_amd/lib/variants/librnsntt_u64r.so
RNSNTT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_replays.py tests/test_gpu_whole.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/u64r/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/u64r/pytest.log; exit 1; }
tail -1 gpurun_out/u64r/pytest.log
for i in 1 2 3; do
  for v in base u64r; do
    lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = u64r ] && lib=$V
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --prime-bits 62 --batch 256 --steps 10 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/u64r/$v$i.json 2> gpurun_out/u64r/$v$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/u64r/$v$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/u64r/$v$i.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$v$i', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
  done
done
