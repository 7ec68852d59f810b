#!/bin/bash
# profile_run.sh <tag> [bench args...]: rocprofv3 kernel-trace stats of the
# bench (default workload unless args say otherwise), then separate PMC
# passes (no tracing domains combined with --pmc) of the same command.
# Every GPU step has its own time limit; any failure stops.  Summarise on
# the CPU afterwards: tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
# <workload> <batch> <log_n> <L>.
set -o pipefail
TAG=${1:-r02}
shift
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
BENCH="bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-power $*"
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH
step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$OUT/sq" -o run -- python3 $BENCH
step pmc_grbm 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d "$OUT/grbm" -o run -- python3 $BENCH
