#!/bin/bash
# profile_any.sh <tag> <bench args...>: kernel trace + separate PMC passes
# (FETCH, WRITE, SQ, GRBM) of one bench.py invocation -> gpurun_out/prof_<tag>.
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
step() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py $BARGS > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "== $name rc=$rc" >&2; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err" >&2; exit $rc; }
}
BARGS="$* --no-cpu-baseline --no-power"
step trace --kernel-trace --stats
step fetch --pmc FETCH_SIZE
step write --pmc WRITE_SIZE
step sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
step grbm --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU
if [ -n "$ICACHE" ]; then
  step ic --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_LDS SQ_INSTS_SMEM
fi
