#!/bin/bash
# Pass-C twiddle chunk pipelining (RNT_PLANE_TPIPE): every GPU test, then the
# NTT workload with and without it on the same box (tools/ab.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out
AB_POWER=1 BENCH_ARGS="--workload ntt" AB_TAG=ntt_ bash tools/ab.sh 3 base nopipe
