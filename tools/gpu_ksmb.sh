#!/bin/bash
# Key-switch sub-chunk size vs the Infinity Cache at config 4 (N=2^16, L=16,
# ct-mul + relin + rescale, 128 cts): RNT_KS_WS_MB caps S per sub-chunk
# (64 MiB per ciphertext), so 128/192 MiB keeps one sub-chunk's S within the
# 256 MiB cache between k_colt_decompose and k_ks_rows.
set -o pipefail
mkdir -p gpurun_out/ksmb
for mb in 4096 256 192 128 64 4096 128; do
  RNT_KS_WS_MB=$mb timeout -k 10 200 python bench.py --workload ctmul --steps 6 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/ksmb/mb$mb.json 2> gpurun_out/ksmb/mb$mb.err || { echo "mb$mb rc=$?"; tail -5 gpurun_out/ksmb/mb$mb.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ksmb/mb$mb.json').read().splitlines()[-1])
r=d['roofline']; k=r.get('kernels') or {}
print('mb$mb', round(d['value']), d['config'].get('parity_spot_check'), r.get('frac') and round(r['frac'],3), {n:(v['launches'],round(v['avg_ms'],4)) for n,v in k.items()})
"
done
