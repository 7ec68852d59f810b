#!/bin/bash
# Key-switch rows A/B: the key-switch grid parity tests, then same-box
# interleaved bench runs of the one-ciphertext rotation (config 5) and
# one-pair / 128-pair ct-mul, this tree against the `oldks` variant
# (tools/build_variant.sh).  Each GPU step under its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_replays.py -x -q -k "keyswitch or config4 or config5 or rotation" --timeout 300 --timeout-method thread > gpurun_out/ks_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/ks_pytest.log; exit 1; }
tail -2 gpurun_out/ks_pytest.log
AB_TAG=rot1_ BENCH_ARGS="--workload rotate --rot-batch 1 --steps 10 --warmup 2" bash tools/ab.sh 2 base oldks || exit 1
AB_TAG=ct1_ BENCH_ARGS="--workload ctmul --ct-batch 1 --steps 40 --warmup 5" bash tools/ab.sh 2 base oldks || exit 1
AB_TAG=ct128_ BENCH_ARGS="--workload ctmul --steps 10 --warmup 2" bash tools/ab.sh 1 base oldks || exit 1
