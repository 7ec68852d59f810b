#!/bin/bash
# Parity tests, then A/B of key-switch row grids across batch sizes:
# tools/gpu_ab_ks_np.sh <reps> <variant...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${1:-2}; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out >&2
for ab in "ct4|--workload ctmul --ct-batch 4" "ct8|--workload ctmul --ct-batch 8" "ct12|--workload ctmul --ct-batch 12" \
          "ct128|--workload ctmul --ct-batch 128" "rot2|--workload rotate --rot-batch 2" "rot4|--workload rotate --rot-batch 4" \
          "rot8|--workload rotate --rot-batch 8"; do
  BENCH_ARGS="${ab#*|}" AB_TAG="${ab%%|*}" bash tools/ab.sh $REPS "$@" || exit $?
done
