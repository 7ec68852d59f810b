#!/bin/bash
# build_variant.sh <name> [hipcc -D flags...]: a build variant of the kernels
# (rnt_kernels.hip, or with PLANE_ONLY=1 only rnt_plane.hip, with the given
# flags) linked with the normal objects of the rest ->
# toy-heaan-ckks_amd/lib/variants/librnsntt_<name>.so (for same-box A/B runs:
# tools/ab.sh).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/toy-heaan-ckks_amd/csrc; L=$ROOT/toy-heaan-ckks_amd/lib; V=$L/variants
mkdir -p $V
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$C"
OBJS_REST="$L/rnt_encode.o $L/rnt_sample.o $L/rnt_api.o"
if [ "${MF_ONLY:-0}" = "1" ]; then
  # only rnt_mfma.hip with the flags (KSRC=<file>: another version of it), the rest as built
  /opt/rocm/bin/hipcc $HF "$@" -c ${KSRC:-$C/rnt_mfma.hip} -o $V/m_$NAME.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $L/rnt_kernels.o $L/rnt_plane.o $V/m_$NAME.o $OBJS_REST -o $V/librnsntt_$NAME.so
  echo $V/librnsntt_$NAME.so
  exit 0
fi
if [ "${PLANE_ONLY:-0}" = "1" ]; then
  # KSRC=<file> compiles another version of rnt_plane.hip
  /opt/rocm/bin/hipcc $HF "$@" -c ${KSRC:-$C/rnt_plane.hip} -o $V/p_$NAME.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $L/rnt_kernels.o $V/p_$NAME.o $L/rnt_mfma.o $OBJS_REST -o $V/librnsntt_$NAME.so
else
  # KSRC=<file> compiles another version of rnt_kernels.hip
  /opt/rocm/bin/hipcc $HF "$@" -c ${KSRC:-$C/rnt_kernels.hip} -o $V/k_$NAME.o
  /opt/rocm/bin/hipcc $HF "$@" -c $C/rnt_plane.hip -o $V/p_$NAME.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $V/k_$NAME.o $V/p_$NAME.o $L/rnt_mfma.o $OBJS_REST -o $V/librnsntt_$NAME.so
fi
echo $V/librnsntt_$NAME.so
