#!/bin/bash
# prof_all.sh <round>: tools/profile_run.sh (kernel trace + PMC passes) for
# the three bench workloads; summarise afterwards on the CPU with
# tools/pmc_summary.py (see profile_run.sh).
R=${1:-r02}
bash tools/profile_run.sh ${R}_polymul || exit $?
STEPS=3 bash tools/profile_run.sh ${R}_ctmul --workload ctmul --ct-batch 128 || exit $?
STEPS=1 bash tools/profile_run.sh ${R}_rotate --workload rotate --rot-batch 8 || exit $?
