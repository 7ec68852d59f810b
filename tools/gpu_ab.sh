#!/bin/bash
# gpu_ab.sh <reps> <variant...>: same-box A/B of library variants with the
# power probe on (tools/ab.sh); the summary goes to stderr and
# gpurun_out/ab_summary.txt.
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_POWER=${AB_POWER:-1} bash tools/ab.sh "$@" 2> >(tee gpurun_out/ab_summary.txt >&2)
