#!/bin/bash
# k_mf_mul's a^ slot stores with the nt (2) or sc1 (16) cache policy against
# the default: the metric-path parity tests, then the headline interleaved.
set -o pipefail
export TMPDIR=/tmp
AB_POWER=1 AB_TAG=slot_ AB_PYTEST="plane_product or metric_path or metric_batch or metric_product" tools/ab.sh 3 base st2 st16 || exit 1
