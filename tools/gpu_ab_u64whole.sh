#!/bin/bash
# The u64 whole-plane product at the horner_chain.rs shape (2^13 x 7 x
# 61-bit): one 512-thread workgroup a CU at 256 VGPRs (no spills) against two
# at 128, canonical and Harvey-lazy; u64 parity tests first.
set -o pipefail
export TMPDIR=/tmp
AB_TAG=u64w_ AB_PYTEST="replay or lazy62 or wide or u64" BENCH_ARGS="--log-n 13 --limbs 7 --prime-bits 61 --batch 1024 --steps 20 --warmup 3" tools/ab.sh 3 base wc2 wlz2 wlz4 || exit 1
