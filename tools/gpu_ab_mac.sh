#!/bin/bash
# Measurement build (wrong words by design): the key-switch rows' lazy
# Montgomery multiply-accumulate replaced by a one-op stand-in, to price it
# at config 4 (ct-mul at 128 pairs) before building a cheaper one.
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--workload ctmul --ct-batch 128" tools/ab.sh 3 base macmeas || exit 1
