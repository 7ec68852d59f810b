#!/bin/bash
# One gpurun call: microbench, GPU parity tests, smoke, short bench.
# Every GPU step has its own time limit; a fault/abort/timeout stops the
# script (exit codes >= 124 or signals), plain test failures do not.
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.out" >&2
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)" >&2
    exit $rc
  fi
  return 0
}
#step mulrate 120 ./tools/bin/mulrate
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 10 --warmup 2
