#!/bin/bash
# Whole-plane product check and A/B: its parity test, then the default bench
# with RNT_PLANE=0 / 1 / 2 alternately (same box), then the phase trace build.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread -k "plane or metric_path" > gpurun_out/plane_test.out 2>&1 || { tail -40 gpurun_out/plane_test.out; exit 1; }
tail -3 gpurun_out/plane_test.out
for i in 1 2; do
  for v in ${MODES:-0 1 2}; do
    RNT_PLANE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_plane${v}_$i.json 2> gpurun_out/ab_plane${v}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_plane${v}_$i.json').read().splitlines()[-1]);print('plane=$v', round(d['value']), d['config']['parity_spot_check'], {k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()}, d['power'])"
  done
done
RNSNTT_LIB=toy-heaan-ckks_amd/lib/variants/librnsntt_trace.so RNT_PLANE=${TRACE_MODE:-1} timeout -k 10 200 python tools/plane_trace.py 1024 > gpurun_out/trace3.json 2>&1 || exit 1
