#!/bin/bash
# After the MFMA wait-state fix: the full-output tensor stress, the GPU
# suite, then same-box A/Bs: ct-mul (config 4 shape) with the matrix-core
# tensor vs the four-step tensor (variant mft0), and the NTT workload with
# the fix vs without it (variant nonop: HEAD's rnt_mfma).
set -o pipefail
mkdir -p gpurun_out/mft2
timeout -k 10 400 python3 tools/tensor_stress2.py 4 64 > gpurun_out/mft2/stress2.log 2>&1 || { echo "stress rc=$?"; cut -c1-200 gpurun_out/mft2/stress2.log | tail; exit 1; }
grep -c equal gpurun_out/mft2/stress2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mft2/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/mft2/pytest.log; exit 1; }
tail -1 gpurun_out/mft2/pytest.log
run() {  # run <tag> <lib> <bench args...>
  local tag=$1 lib=$2; shift 2
  RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-power "$@" > gpurun_out/mft2/$tag.json 2> gpurun_out/mft2/$tag.err || { echo "$tag rc=$?"; tail -5 gpurun_out/mft2/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/mft2/$tag.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('$tag', round(d['value']), d['config'].get('parity_spot_check'), r.get('frac') and round(r['frac'],3), {n:(v['launches'],round(v['avg_ms'],4)) for n,v in k.items()})
"
}
B=toy-heaan-ckks_amd/lib/librnsntt.so; V=toy-heaan-ckks_amd/lib/variants
for i in 1 2 3; do
  run ct_mf$i $B --workload ctmul --steps 6 --warmup 2
  run ct_4s$i $V/librnsntt_mft0.so --workload ctmul --steps 6 --warmup 2
done
for i in 1 2 3; do
  run ntt_nop$i $B --workload ntt --steps 20 --warmup 3
  run ntt_old$i $V/librnsntt_nonop.so --workload ntt --steps 20 --warmup 3
done
