#!/bin/bash
# k_plane_fused A/B: the plane product's parity tests, then same-box
# interleaved default bench runs (with power) of this tree against the
# `oldplane` variant (tools/build_variant.sh PLANE_ONLY=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "plane or metric" --timeout 300 --timeout-method thread > gpurun_out/plane_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/plane_pytest.log; exit 1; }
tail -2 gpurun_out/plane_pytest.log
AB_POWER=1 AB_TAG=pl_ bash tools/ab.sh ${REPS:-3} base oldplane || exit 1
