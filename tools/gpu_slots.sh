#!/bin/bash
# CU-indexed a^ scratch (RNT_PLANE_SLOTS=1): full-batch word compare against
# the per-plane scratch kernel, the plane parity tests with it on, then a
# same-box interleaved bench A/B with power.
set -o pipefail
mkdir -p gpurun_out/slots
timeout -k 10 300 python3 tools/slots_check.py > gpurun_out/slots/check.log 2>&1 || { echo "check rc=$?"; tail -20 gpurun_out/slots/check.log; exit 1; }
cat gpurun_out/slots/check.log
RNT_PLANE_SLOTS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "plane or metric" --timeout 300 --timeout-method thread > gpurun_out/slots/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/slots/pytest.log; exit 1; }
tail -1 gpurun_out/slots/pytest.log
AB_POWER=1 AB_TAG=sl_ bash tools/ab.sh ${REPS:-3} base base+RNT_PLANE_SLOTS=1
