#!/bin/bash
# r03d check of the shipped tree: every GPU test, smoke, the default bench
# line, the NTT workload line (whole-plane transforms), then the kernel-trace
# and PMC passes of the NTT workload (tools/profile_run.sh).  Each GPU step
# has its own time limit; a failing step stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out >&2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.out 2>&1 || { tail -20 gpurun_out/smoke.out; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -c 400 gpurun_out/bench_default.json >&2
timeout -k 10 600 python bench.py --workload ntt > gpurun_out/bench_ntt.json 2> gpurun_out/bench_ntt.err || { tail -20 gpurun_out/bench_ntt.err; exit 1; }
tail -c 400 gpurun_out/bench_ntt.json >&2
STEPS=5 bash tools/profile_run.sh r03d_ntt --workload ntt || exit $?
