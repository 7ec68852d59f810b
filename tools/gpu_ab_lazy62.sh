#!/bin/bash
# The u64 Harvey-lazy product (lazy62) against the canonical u64 kernels
# (RNT_LAZY62=0), same box, interleaved: parity first, then the reference's
# wide-prime shapes.  Output: gpurun_out/ab_*lazy62*
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lazy62.py tests/test_gpu_replays.py tests/test_gpu_whole.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lazy62_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/lazy62_pytest.log; exit 1; }
tail -2 gpurun_out/lazy62_pytest.log
for shape in "horner:--log-n 13 --limbs 7 --prime-bits 61 --batch 1024" "n16:--log-n 16 --limbs 16 --prime-bits 62 --batch 256" "n10:--log-n 10 --limbs 2 --prime-bits 62 --batch 4096"; do
  name=${shape%%:*}; args=${shape#*:}
  AB_TAG=${name}_ BENCH_ARGS="$args" tools/ab.sh 3 base base+RNT_LAZY62=0 || exit 1
done
