#!/bin/bash
# Key-switch occupancy / staging A/Bs (profiles/r06/prediction_ks_occupancy.md):
# ct-mul at 128 pairs (config 4 ring) and the one-ciphertext rotation (config 5)
set -o pipefail
export TMPDIR=/tmp
AB_TAG=ks_ AB_PYTEST="config4_ct_mul or keyswitch_row_grids" BENCH_ARGS="--workload ctmul --ct-batch 128" tools/ab.sh 3 base ksw3 ksw5 base+RNT_DEC_JG=8 base+RNT_DEC_JG=4 || exit 1
AB_TAG=rot_ BENCH_ARGS="--workload rotate --rot-batch 1 --steps 5" tools/ab.sh 2 base ksw3 ksw5 || exit 1
