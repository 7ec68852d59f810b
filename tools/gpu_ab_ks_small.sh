#!/bin/bash
# Parity tests, then A/B of key-switch row variants at the bench batches and
# at small batches (rotation of 1 ciphertext, ct-mul of 4 pairs):
# tools/gpu_ab_ks_small.sh <reps> <variant...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${1:-2}; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out >&2
BENCH_ARGS="--workload ctmul --ct-batch 128" AB_TAG=ct bash tools/ab.sh $REPS "$@" || exit $?
BENCH_ARGS="--workload rotate --rot-batch 8" AB_TAG=rot bash tools/ab.sh $REPS "$@" || exit $?
BENCH_ARGS="--workload rotate --rot-batch 1" AB_TAG=rot1 bash tools/ab.sh $REPS "$@" || exit $?
BENCH_ARGS="--workload ctmul --ct-batch 4" AB_TAG=ct4 bash tools/ab.sh $REPS "$@" || exit $?
