#!/bin/bash
# r06c: every GPU test, then the u64 lazy row occupancy A/B and the ct-mul /
# rotation lines after the uninitialised op outputs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AB_TAG=n16w_ BENCH_ARGS="--log-n 16 --limbs 16 --prime-bits 62 --batch 256" tools/ab.sh 3 base u64w3 || exit 1
timeout -k 10 300 python3 bench.py --workload ctmul --ct-batch 128 --steps 10 --warmup 2 --no-cpu-baseline > $O/ctmul.json 2> $O/ctmul.err || { echo "ctmul rc=$?"; tail -5 $O/ctmul.err; exit 1; }
head -c 250 $O/ctmul.json; echo
timeout -k 10 300 python3 bench.py --workload rotate --rot-batch 1 --steps 5 --warmup 1 --no-cpu-baseline > $O/rot1.json 2> $O/rot1.err || { echo "rot rc=$?"; tail -5 $O/rot1.err; exit 1; }
head -c 250 $O/rot1.json; echo
