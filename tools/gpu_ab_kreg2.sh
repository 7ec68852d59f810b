#!/bin/bash
# The one-poly key-switch grid with register keys at two workgroups a CU
# (RNT_KS_KREG=1, RNT_KS_KREG_WAVES=2: 256 VGPRs, no spills), with and
# without the next S row in flight, against the shipped staging: parity
# first, then the one-ciphertext rotation interleaved.
set -o pipefail
export TMPDIR=/tmp
AB_TAG=kreg2_ AB_PYTEST="keyswitch_row_grids or config5_rotation or diagonal_from_tensor" BENCH_ARGS="--workload rotate --rot-batch 1 --steps 5" tools/ab.sh 3 base kreg2 kreg2ns || exit 1
