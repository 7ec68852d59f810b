#!/bin/bash
# k_mf_mul2 (512 threads, two virtual waves a wave; RNT_MF_MUL2_REG a^ tiles a
# virtual wave in registers) against k_mf_mul: the metric-path parity tests
# through each library, then the poly-mul headline interleaved.
set -o pipefail
export TMPDIR=/tmp
AB_POWER=1 AB_TAG=mul2_ AB_PYTEST="plane_product or metric_path or metric_batch or metric_product" tools/ab.sh 3 base v2r0 v2r1 v2r2 || exit 1
