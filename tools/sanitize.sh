#!/usr/bin/env bash
# Host sanitizer pass ("-fsanitize=address on host tests").
#
# Builds AddressSanitizer + UndefinedBehaviorSanitizer variants of
#   - oracle/oracle.c (the CPU checker), with clang,
#   - librnsntt.so, whose HOST code (rnt_api.cpp: validation, primes, psi,
#     tables, error detail, the refcounted contexts and the block cache's
#     host side) is instrumented; device code is not (each -fsanitize= sits
#     after -Xarch_host, and GPU sanitizers are not used on this pool),
# into build/asan/, then runs the CPU tests that exercise those host paths
# (tests/test_abi_cpu.py, tests/test_oracle.py, tests/test_sampler.py,
# tests/test_sharded.py's oracle-backend ranks) with the clang ASan runtime
# preloaded into python.  One runtime for both libraries (clang's), so the
# oracle is built with the ROCm clang rather than gcc here.
#
# Usage: tools/sanitize.sh [log]   (default log: profiles/r06_sanitizer_cpu.log)
set -euo pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r06_sanitizer_cpu.log}
LLVM=/opt/rocm/lib/llvm/bin
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
OUT=build/asan
mkdir -p "$OUT"
SAN="-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
HOSTSAN=""
for f in $SAN; do
  case $f in -fsanitize=*|-fno-sanitize-recover=*) HOSTSAN="$HOSTSAN -Xarch_host $f";; *) HOSTSAN="$HOSTSAN $f";; esac
done
CS=toy-heaan-ckks_amd/csrc
HIPFLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC"
{
  echo "# tools/sanitize.sh $(date -u +%Y-%m-%dT%H:%M:%SZ) at commit $(git rev-parse --short HEAD)$(git diff --quiet HEAD -- toy-heaan-ckks_amd oracle include || echo ' (+ uncommitted changes)')"
  echo "# oracle: $LLVM/clang $SAN"
  echo "# librnsntt host code: $HIPCC $HIPFLAGS$HOSTSAN"
} > "$LOG"
$LLVM/clang -O1 -g -fPIC -std=c11 -Wall -pthread $SAN -shared-libsan -shared oracle/oracle.c -o $OUT/liboracle.so
# the library's translation units, from the same list build() compiles
SRCS=$(python -c "import __graft_entry__ as g; print(' '.join(g.SOURCES))")
echo "# sources: $SRCS" >> "$LOG"
pids=()
objs=()
for src in $SRCS; do
  $HIPCC $HIPFLAGS $HOSTSAN -c $CS/$src -o $OUT/${src%.*}.o & pids+=($!)
  objs+=("$OUT/${src%.*}.o")
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -shared-libsan "${objs[@]}" -o $OUT/librnsntt.so
RT=$($LLVM/clang -print-file-name=libclang_rt.asan-x86_64.so)
echo "# runtime: $RT" >> "$LOG"
# leaks: python and torch keep allocations alive at exit by design, so leak
# detection is off; every other ASan/UBSan finding aborts the run
set +e
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  RNSNTT_LIB=$PWD/$OUT/librnsntt.so ORACLE_LIB=$PWD/$OUT/liboracle.so \
  python -m pytest tests/test_abi_cpu.py tests/test_oracle.py tests/test_sampler.py tests/test_sharded.py \
    -q -m "not gpu" -p no:cacheprovider >> "$LOG" 2>&1
rc=$?
set -e
reports=$(grep -c "ERROR: AddressSanitizer\|runtime error:" "$LOG" || true)
echo "# sanitizer reports: $reports" >> "$LOG"
if [ "$rc" -ne 0 ]; then
  echo "# FAILED: pytest exit status $rc" >> "$LOG"
else
  echo "# PASSED: pytest exit status 0" >> "$LOG"
fi
tail -5 "$LOG"
exit $rc
