#!/bin/bash
# The shipped library as the driver will run it: every GPU test, smoke(),
# then the default bench line (N=1, live PMC, power probe).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
head -c 400 $O/bench.json; echo
