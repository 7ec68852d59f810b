#!/bin/bash
# The rotation's sigma(c0) gathered by the key-switch inverse (RNT_ROT_FUSE=1,
# default) against its own k_automorph_odd launch (RNT_ROT_FUSE=0): the
# rotation parity tests first, then config 5 (one and eight ciphertexts)
# interleaved on one box.
set -o pipefail
export TMPDIR=/tmp
AB_TAG=rf_ AB_PYTEST="rotation" BENCH_ARGS="--workload rotate --rot-batch 1 --steps 5" tools/ab.sh 3 base base+RNT_ROT_FUSE=0 || exit 1
AB_TAG=rf8_ BENCH_ARGS="--workload rotate --rot-batch 8 --steps 3" tools/ab.sh 2 base base+RNT_ROT_FUSE=0 || exit 1
