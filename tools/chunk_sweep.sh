#!/bin/bash
# Infinity-Cache residency experiment: poly-mul throughput vs launch chunk.
mkdir -p gpurun_out
for mb in 0 256 128 64 32; do
  echo "== chunk ${mb} MiB" >&2
  RNT_MUL_CHUNK_MB=$mb timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/chunk_$mb.json 2> gpurun_out/chunk_$mb.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/chunk_$mb.json'));print($mb, round(d['value']), {k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()})" >&2
done
