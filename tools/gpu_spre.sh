#!/bin/bash
# Key-switch rows with the next source limb's S rows prefetched global -> LDS
# (RNT_KS_SPRE): every GPU test, then the ct-mul workload (1024 and
# 128 pairs) against the RNT_KS_SPRE=0 build on the same box (tools/ab.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out
BENCH_ARGS="--workload ctmul --ct-batch 1024" AB_TAG=ct1024_ bash tools/ab.sh 2 base nospre || exit $?
BENCH_ARGS="--workload ctmul --ct-batch 128" AB_TAG=ct128_ bash tools/ab.sh 2 base nospre || exit $?
