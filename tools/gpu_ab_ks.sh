#!/bin/bash
# A/B of key-switch kernel variants (tools/build_variant.sh) on the ct-mul
# and rotation workloads: tools/gpu_ab_ks.sh <reps> <variant...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${1:-2}; shift
BENCH_ARGS="--workload ctmul --ct-batch 128" AB_TAG=ct bash tools/ab.sh $REPS "$@" || exit $?
BENCH_ARGS="--workload rotate --rot-batch 8" AB_TAG=rot bash tools/ab.sh $REPS "$@" || exit $?
