#!/bin/bash
# ab.sh <reps> <variant...>: interleaved short bench runs on one box.
# A variant is <lib>[+VAR=VAL...]: <lib> = "base" (lib/librnsntt.so) or a
# name from tools/build_variant.sh; the +VAR=VAL pairs are exported for that
# run (e.g. base+RNT_PLANE=0).  Results -> gpurun_out/ab_<variant>_<i>.json,
# summarised by tools/ab_summary.py.  BENCH_ARGS: the bench workload and
# shape (e.g. "--workload ctmul --ct-batch 1").  AB_PYTEST: a pytest -k
# expression; every variant first runs those GPU parity tests through its
# library (one process, its own time limit) and the A/B stops on a failure.
# (This replaces r03/r04's one-off tools/gpu_*.sh wrappers.)
set -o pipefail
mkdir -p gpurun_out
REPS=$1; shift
VARS=${@:-base}
# AB_POWER=1 keeps the bench's power probe (3 s more per run)
POWER_ARG=--no-power
[ "${AB_POWER:-0}" = "1" ] && POWER_ARG=
if [ -n "${AB_PYTEST:-}" ]; then
  for v in $VARS; do
    IFS='+' read -ra parts <<< "$v"
    libname=${parts[0]}
    if [ "$libname" = base ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$libname.so; fi
    tag=$(echo "${AB_TAG:-}$v" | tr '+=' '__')
    env RNSNTT_LIB=$lib "${parts[@]:1}" timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -k "$AB_PYTEST" --timeout 300 --timeout-method thread > gpurun_out/ab_${tag}_pytest.log 2>&1 || { echo "pytest ($v) rc=$?" >&2; tail -20 gpurun_out/ab_${tag}_pytest.log >&2; exit 1; }
    echo "== $v: $(tail -1 gpurun_out/ab_${tag}_pytest.log)" >&2
  done
fi
for i in $(seq 1 $REPS); do
  for v in $VARS; do
    IFS='+' read -ra parts <<< "$v"
    libname=${parts[0]}
    if [ "$libname" = base ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$libname.so; fi
    tag=$(echo "${AB_TAG:-}$v" | tr '+=' '__')
    env RNSNTT_LIB=$lib "${parts[@]:1}" timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-live-pmc $POWER_ARG $BENCH_ARGS > gpurun_out/ab_${tag}_$i.json 2> gpurun_out/ab_${tag}_$i.err || exit $?
  done
done
for v in $VARS; do tag=$(echo "${AB_TAG:-}$v" | tr '+=' '__'); echo "== $v" >&2; python3 tools/ab_summary.py gpurun_out/ab_${tag}_[0-9]*.json >&2; done
