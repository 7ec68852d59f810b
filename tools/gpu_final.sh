#!/bin/bash
# Round-end evidence from one lease: every GPU test, smoke(), then the
# headline evidence (bench line with live PMC + power/sclk, rocprofv3
# kernel trace of the same command, SQ pass) -- tools/gpu_headline.sh
set -o pipefail
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
tools/gpu_headline.sh
