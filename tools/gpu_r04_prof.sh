#!/bin/bash
# Round-4 profiles: kernel-trace stats + PMC passes of the NTT workload, the
# poly-mul and the ct-mul (tools/profile_run.sh; every step time-limited).
set -o pipefail
STEPS=5 bash tools/profile_run.sh r04_ntt --workload ntt || exit $?
STEPS=5 bash tools/profile_run.sh r04_polymul || exit $?
STEPS=3 bash tools/profile_run.sh r04_ctmul --workload ctmul || exit $?
