#!/bin/bash
# The key-switch diagonal from the tensor's d2^ (default) against RNT_KS_DIAG=0
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_whole.py tests/test_gpu_replays.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/diag_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/diag_pytest.log; exit 1; }
tail -2 gpurun_out/diag_pytest.log
AB_TAG=dg4_ BENCH_ARGS="--workload ctmul --ct-batch 1024 --steps 4 --warmup 1" tools/ab.sh 3 base base+RNT_KS_DIAG=0 || exit 1
AB_TAG=dg3_ BENCH_ARGS="--workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 10 --warmup 2" tools/ab.sh 3 base base+RNT_KS_DIAG=0 || exit 1
AB_TAG=dg128_ BENCH_ARGS="--workload ctmul --ct-batch 128 --steps 10 --warmup 2" tools/ab.sh 2 base base+RNT_KS_DIAG=0 || exit 1
