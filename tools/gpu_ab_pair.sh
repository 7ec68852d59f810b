#!/bin/bash
# Key-switch rows two source limbs a step (RNT_KS_PAIR: NOPS = 2 transforms,
# one reduction for two products) against one a step: the whole GPU suite
# through the pair build first, the key-switch tests through the other, then
# ct-mul at config 4 (128 pairs), config 3 (1024 pairs) and the 8-ciphertext
# rotation at config 5, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pair_pytest.log 2>&1 || { echo "pytest rc=$?" >&2; tail -30 gpurun_out/pair_pytest.log >&2; exit 1; }
echo "== full suite (pair): $(tail -1 gpurun_out/pair_pytest.log)" >&2
AB_TAG=p4_ AB_PYTEST="keyswitch or config4 or diagonal" BENCH_ARGS="--workload ctmul --ct-batch 128" tools/ab.sh 3 base nopair || exit 1
AB_TAG=p3_ BENCH_ARGS="--workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 10 --warmup 2" tools/ab.sh 2 base nopair || exit 1
AB_TAG=p5_ BENCH_ARGS="--workload rotate --rot-batch 8 --steps 3" tools/ab.sh 2 base nopair || exit 1
