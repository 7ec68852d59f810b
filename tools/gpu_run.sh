#!/bin/bash
# gpu_run.sh <script-steps...>: parity tests then the given extra scripts.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.out 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.out >&2
if [ $rc -ge 124 ]; then exit $rc; fi
for s in "$@"; do ./$s || exit $?; done
