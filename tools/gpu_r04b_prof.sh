#!/bin/bash
# Round-4 closing profiles of the current tree: kernel-trace stats + PMC
# passes of the default poly-mul bench, the ct-mul (config 4 shape) and the
# NTT workload (tools/profile_run.sh; every step time-limited).
set -o pipefail
STEPS=5 bash tools/profile_run.sh r04b_polymul || exit $?
STEPS=3 bash tools/profile_run.sh r04b_ctmul --workload ctmul || exit $?
STEPS=5 bash tools/profile_run.sh r04b_ntt --workload ntt || exit $?
