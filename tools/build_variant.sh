#!/bin/bash
# build_variant.sh <name> [hipcc -D flags...]: a build variant of the kernels
# (rnt_kernels.hip with the given flags) linked with the normal API object
# -> toy-heaan-ckks_amd/lib/variants/librnsntt_<name>.so (for same-box A/B
# runs: tools/ab.sh).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/toy-heaan-ckks_amd/csrc; L=$ROOT/toy-heaan-ckks_amd/lib; V=$L/variants
mkdir -p $V
# KSRC=<file> compiles another version (e.g. from git show)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$C "$@" -c ${KSRC:-$C/rnt_kernels.hip} -o $V/k_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $V/k_$NAME.o $L/rnt_encode.o $L/rnt_sample.o $L/rnt_api.o -o $V/librnsntt_$NAME.so
echo $V/librnsntt_$NAME.so
