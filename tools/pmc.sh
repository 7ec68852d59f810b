#!/bin/bash
# PMC counter passes over the bench (each pass its own rocprofv3 run, no
# tracing domains combined with --pmc).
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {  # run <tag> <counters...>
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/pmc/$tag" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-power --batch 64 > gpurun_out/pmc/$tag.out 2> gpurun_out/pmc/$tag.err
  local rc=$?; echo "pmc $tag rc=$rc" >&2; [ $rc -lt 124 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM
run tcc1 FETCH_SIZE
run tcc2 WRITE_SIZE
