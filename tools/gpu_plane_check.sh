#!/bin/bash
# Whole-plane product: its parity tests (every mode, edge operands, the
# metric's 1024-pair batch sampled), then a same-box A/B of the given
# variants (tools/ab.sh with the power probe).  A failing test stops it.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "plane or metric" > gpurun_out/plane_test.out 2>&1 || { tail -40 gpurun_out/plane_test.out; exit 1; }
tail -3 gpurun_out/plane_test.out
AB_POWER=1 bash tools/ab.sh ${REPS:-2} "$@" 2> >(tee gpurun_out/ab_summary.txt >&2)
