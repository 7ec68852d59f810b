#!/bin/bash
# k_mf_tensor epilogue-operand prefetch (variant pf) vs the tree: full-output
# tensor stress with the variant, then interleaved ct-mul bench lines.
set -o pipefail
mkdir -p gpurun_out/pf
V=toy-heaan-ckks_amd/lib/variants/librnsntt_pf.so
RNSNTT_LIB=$V timeout -k 10 300 python3 tools/tensor_stress2.py 2 64 > gpurun_out/pf/stress.log 2>&1 || { echo "stress rc=$?"; cut -c1-200 gpurun_out/pf/stress.log | tail; exit 1; }
grep -c equal gpurun_out/pf/stress.log
for i in 1 2 3; do
  for v in base pf; do
    lib=toy-heaan-ckks_amd/lib/librnsntt.so; [ $v = pf ] && lib=$V
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --workload ctmul --steps 6 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/pf/$v$i.json 2> gpurun_out/pf/$v$i.err || { echo "$v rc=$?"; tail -5 gpurun_out/pf/$v$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/pf/$v$i.json').read().splitlines()[-1])
k=d['roofline'].get('kernels') or {}
print('$v$i', round(d['value']), d['config'].get('parity_spot_check'), {n:round(v['avg_ms'],4) for n,v in k.items()})
"
  done
done
