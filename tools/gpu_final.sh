#!/bin/bash
# End-of-round check: GPU parity tests, smoke, the default bench line, a
# one-pair ct-mul line (the engine's call shape), then the kernel-trace and
# PMC profiles of the three workloads (tools/prof_all.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out >&2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >&2 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --workload ctmul --ct-batch 1 --steps 20 --warmup 3 > gpurun_out/bench_ctmul_b1.json 2> gpurun_out/bench_ctmul_b1.err || exit $?
bash tools/prof_all.sh ${1:-r02j} || exit $?
