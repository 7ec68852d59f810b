#!/bin/bash
# r03 check after the whole-plane product became the default: GPU tests,
# the default bench line (with its CPU baseline), the 30-bit poly-mul, and
# the four-step path (RNT_PLANE=0) on the same box.  Each GPU step has its
# own time limit; a failing step stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
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
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
step bench_default 600 python bench.py
step bench_p30 300 python bench.py --prime-bits 30 --steps 20 --warmup 3 --no-cpu-baseline
RNT_PLANE=0 step bench_fourstep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
RNT_PLANE=0 step bench_fourstep_p30 300 python bench.py --prime-bits 30 --steps 20 --warmup 3 --no-cpu-baseline
