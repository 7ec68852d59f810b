#!/bin/bash
# Round-6 closing evidence from ONE lease on the final tree: every GPU test,
# smoke(), the headline evidence (tools/gpu_headline.sh: bench line with live
# PMC + power/sclk, rocprofv3 kernel trace of the same command, SQ pass), the
# BASELINE config lines, the u64 and NTT lines, then the N-rank one-device
# rehearsal (tools/gpu_rehearse.sh).  Each step under its own limit; the
# first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
tools/gpu_headline.sh || exit 1
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -5 $O/$name.err; exit 1; }; echo "$name $(head -c 120 $O/$name.json)"; }
run ctmul128 --workload ctmul --ct-batch 128 --steps 10 --warmup 2 --no-cpu-baseline
run cfg4 --workload ctmul --ct-batch 1024 --steps 4 --warmup 1
run cfg3 --workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 10 --warmup 2
run rot1 --workload rotate --rot-batch 1 --steps 5 --warmup 1 --no-cpu-baseline
run rot8 --workload rotate --rot-batch 8 --steps 3 --warmup 1 --no-cpu-baseline
run u64n16 --log-n 16 --limbs 16 --prime-bits 62 --batch 256 --steps 10 --warmup 2 --no-cpu-baseline
run u64horner --log-n 13 --limbs 7 --prime-bits 61 --batch 1024 --steps 20 --warmup 3 --no-cpu-baseline
run ntt --workload ntt --steps 10 --warmup 2 --no-cpu-baseline
tools/gpu_rehearse.sh || exit 1
echo done
