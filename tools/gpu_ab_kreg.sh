#!/bin/bash
# Key-switch rows on the one-poly grid (NP = 1): keys straight into
# registers (KREG) and the S row one source limb ahead (SPRE) against the
# r06 staging (nokreg: key_b by LDS-DMA, key_a into the exchange region after
# the transform).  Parity first (every row grid, the config-5 rotation, the
# diagonal), then the one-ciphertext rotation interleaved.
set -o pipefail
export TMPDIR=/tmp
AB_TAG=kreg_ AB_PYTEST="keyswitch_row_grids or config5_rotation or diagonal_from_tensor" BENCH_ARGS="--workload rotate --rot-batch 1 --steps 5" tools/ab.sh 3 base nospre nokreg || exit 1
