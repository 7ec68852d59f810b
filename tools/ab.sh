#!/bin/bash
# ab.sh <reps> <variant...>: interleaved short bench runs of build variants
# (lib/variants/librnsntt_<v>.so; "base" = lib/librnsntt.so) on one box ->
# gpurun_out/ab_<v>_<i>.json, summarised per variant by tools/ab_summary.py.
set -o pipefail
mkdir -p gpurun_out
REPS=$1; shift
VARS=${@:-base}
for i in $(seq 1 $REPS); do
  for v in $VARS; do
    if [ "$v" = base ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$v.so; fi
    RNSNTT_LIB=$lib timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || exit $?
  done
done
for v in $VARS; do echo "== $v" >&2; python3 tools/ab_summary.py gpurun_out/ab_${v}_*.json >&2; done
