#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the bench workloads, and
# (PROFILE=1) a rocprofv3 kernel trace.  Every GPU step has its own time
# limit; any failing step stops the script (a failed parity test may be a
# device fault: start nothing more).
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.out" >&2
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)" >&2
    tail -20 "gpurun_out/$name.err" >&2
    exit $rc
  fi
  return 0
}
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py --steps 20 --warmup 3
step bench_ctmul 900 python bench.py --workload ctmul --ct-batch ${CT_BATCH:-128} --steps 3 --warmup 1
step bench_rotate 900 python bench.py --workload rotate --rot-batch ${ROT_BATCH:-8} --steps 2 --warmup 1
if [ "${PROFILE:-0}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-power
fi
