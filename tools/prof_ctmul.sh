#!/bin/bash
# rocprofv3 kernel stats of the config-4 pipeline bench (ctmul workload).
set -o pipefail
mkdir -p gpurun_out/prof_ctmul
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_ctmul" -o run -- python3 bench.py --workload ctmul --ct-batch ${CT_BATCH:-64} --steps 3 --warmup 1 --no-cpu-baseline --no-power > gpurun_out/prof_ctmul/bench.out 2> gpurun_out/prof_ctmul/bench.err
