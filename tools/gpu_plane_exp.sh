#!/bin/bash
# Whole-plane kernels: measurement builds (RNT_PLANE_EXP, wrong results by
# design) against the shipped build, same box: where the workgroup time goes.
mkdir -p gpurun_out
export TMPDIR=/tmp RNT_PLANE=${MODE:-1}
for i in 1 2; do
  for v in ship ${VARIANTS:-exp1 exp2 exp4 exp7}; do
    if [ $v = ship ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$v.so; fi
    RNSNTT_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pe_${v}_$i.json 2> gpurun_out/pe_${v}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/pe_${v}_$i.json').read().splitlines()[-1]);print('$v', round(d['value']), d['config']['parity_spot_check'], {k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()}, d['power']['package_w_median'], d['power']['sclk_mhz_median'])"
  done
done
