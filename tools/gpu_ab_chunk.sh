#!/bin/bash
# Config 4 (1024 cts) with larger key-switch chunks: the pipeline chunk and
# the library's S cap (RNT_KS_WS_MB) together; interleaved, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abchunk; mkdir -p $O
for i in 1 2; do
  for v in ${CHUNKS:-"64:4096" "128:8192" "256:16384"}; do
    c=${v%%:*}; mb=${v#*:}
    RNT_KS_WS_MB=$mb timeout -k 10 400 python3 bench.py --workload ctmul --ct-batch 1024 --chunk $c --steps 4 --warmup 1 --no-cpu-baseline --no-power > $O/c${c}_$i.json 2> $O/c${c}_$i.err || { echo "chunk $c rc=$?"; tail -5 $O/c${c}_$i.err; exit 1; }
    echo "chunk $c run $i: $(python3 -c "import json;d=json.loads(open('$O/c${c}_$i.json').read().strip().splitlines()[-1]);print(round(d['value']),d['config']['parity_spot_check'],{k:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()})")"
  done
done
