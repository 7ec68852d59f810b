#!/bin/bash
# Pass-C twiddle chunk size (RNT_PLANE_CHC, base 8 vs 4): NTT and poly-mul
# workloads on one box (tools/ab.sh), after the plane-kernel GPU tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k plane > gpurun_out/pytest_plane.out 2>&1 || { tail -30 gpurun_out/pytest_plane.out; exit 1; }
tail -1 gpurun_out/pytest_plane.out
AB_POWER=1 BENCH_ARGS="--workload ntt" AB_TAG=ntt_ bash tools/ab.sh 3 base chc4 || exit $?
AB_POWER=1 AB_TAG=pm_ bash tools/ab.sh 2 base chc4 || exit $?
