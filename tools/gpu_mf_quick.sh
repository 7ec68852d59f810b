#!/usr/bin/env bash
# quick same-box poly-mul A/B: RNT_PLANE=3 (VALU plane kernel) vs 5 (MFMA)
set -euo pipefail
O=gpurun_out/r04; mkdir -p $O; tag=${1:-q}
for p in 5 3 5; do
  RNT_PLANE=$p timeout -k 10 240 python bench.py --no-cpu-baseline > $O/${tag}_p$p.json 2>/dev/null
  python -c "import json; d=json.load(open('$O/${tag}_p$p.json')); pw=d.get('power') or {}; print('plane $p', round(d['value']), round(d['ms_per_step'],3), d['config']['parity_spot_check'], pw.get('package_w_median'), pw.get('sclk_mhz_median'))"
done
