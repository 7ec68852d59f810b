#!/bin/bash
# u64 whole-plane product rows at 2^10..2^12 capped at 128 VGPRs (variant
# u64s; uncapped 140-154, three waves per SIMD) vs this tree: u64 parity
# through the variant, then interleaved poly-mul lines at the reference's
# integration_mul.rs shape (2^10 x 2 x 62-bit) and 2^12 x 4 x 61-bit.
set -o pipefail
mkdir -p gpurun_out/u64s
V=toy-heaan-ckks_amd/lib/variants/librnsntt_u64s.so
RNSNTT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_whole.py tests/test_gpu_replays.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/u64s/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/u64s/pytest.log; exit 1; }
tail -1 gpurun_out/u64s/pytest.log
for cfg in "10 2 62" "12 4 61"; do
  set -- $cfg
  for i in 1 2; do
    for v in base u64s; do
      lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = u64s ] && lib=$V
      RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --log-n $1 --limbs $2 --prime-bits $3 --batch 4096 --steps 20 --warmup 3 --no-cpu-baseline --no-power > gpurun_out/u64s/$v$1_$i.json 2> gpurun_out/u64s/$v$1_$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/u64s/$v$1_$i.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('gpurun_out/u64s/$v$1_$i.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$v$1_$i', round(d['value']), d['config'].get('parity_spot_check'), round(d['roofline']['frac'],3), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
    done
  done
done
