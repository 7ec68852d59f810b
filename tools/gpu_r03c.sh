#!/bin/bash
# r03 re-entry check: GPU parity tests, smoke, the default bench line, a
# kernel-trace profile of it, and the phase timeline of the fused plane
# kernel (trace build).  Each GPU step has its own time limit; a failing step
# stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -2 "gpurun_out/$name.out" >&2
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)" >&2
    tail -20 "gpurun_out/$name.err" >&2
    exit $rc
  fi
  return 0
}
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_default 600 python bench.py
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-power
fi
if [ -f toy-heaan-ckks_amd/lib/variants/librnsntt_trace.so ] && [ "${TRACE:-1}" = "1" ]; then
  RNSNTT_LIB=toy-heaan-ckks_amd/lib/variants/librnsntt_trace.so step trace 200 python tools/plane_trace.py 1024
fi
for v in ${VARIANTS:-}; do
  RNSNTT_LIB=toy-heaan-ckks_amd/lib/variants/librnsntt_$v.so step "bench_$v" 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
