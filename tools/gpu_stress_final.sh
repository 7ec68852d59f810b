#!/bin/bash
# Full-output stress of the shipped matrix-core kernels on the final tree:
# every word of the metric's poly-mul batch (k_mf_mul vs the four-step
# kernels, 3 rounds), of 128 polys' NTT round trips, and of the tensor at
# 1024 pairs, each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stress6; mkdir -p $O
timeout -k 10 500 python3 -u tools/mul_stress.py 3 1024 > $O/mul.log 2>&1 || { echo "mul rc=$?"; tail -20 $O/mul.log; exit 1; }
tail -5 $O/mul.log
timeout -k 10 400 python3 -u tools/ntt_stress.py 4 128 > $O/ntt.log 2>&1 || { echo "ntt rc=$?"; tail -20 $O/ntt.log; exit 1; }
tail -5 $O/ntt.log
timeout -k 10 500 python3 -u tools/tensor_stress2.py 3 64 > $O/tensor.log 2>&1 || { echo "tensor rc=$?"; tail -20 $O/tensor.log; exit 1; }
tail -5 $O/tensor.log
