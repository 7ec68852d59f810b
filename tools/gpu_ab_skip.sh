#!/bin/bash
# Measurement builds (wrong words by design): k_mf_mul without the slot round
# trip of its first SKIP a^ tiles a wave (3, 5, 10 of 10).  If the slot's
# remaining footprint per XCD (32 CUs x (10 - SKIP) KiB a wave x 16 waves)
# then fits the 4 MiB L2, the traffic and the time drop by more than the
# skipped share: the case for more a^ tiles in the LDS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/ab.sh 2 base skip3 skip5 skip10 || exit 1
for v in base skip3 skip5 skip10; do
  if [ $v = base ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$v.so; fi
  RNSNTT_LIB=$lib timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-power > gpurun_out/skip_pmc_$v.json 2> gpurun_out/skip_pmc_$v.err || exit 1
  python3 - gpurun_out/skip_pmc_$v.json $v <<'PY' >&2
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], 'value', round(d['value']), 'traffic', r.get('traffic'), 'achieved', r.get('achieved'), {k: r.get(k) for k in ('traffic_read','traffic_write','pmc') if k in r})
PY
done
