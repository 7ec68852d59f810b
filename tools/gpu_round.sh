#!/bin/bash
# Round-end check: every GPU test, smoke(), the default bench line and a
# rocprofv3 kernel-trace summary of it (each step under its own limit; any
# failure stops).  Output: gpurun_out/round/
set -o pipefail
O=gpurun_out/round; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/trace" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-power > $O/trace.out 2> $O/trace.err || { echo "trace rc=$?"; exit 1; }
echo done
