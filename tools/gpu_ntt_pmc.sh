#!/usr/bin/env bash
# PMC passes of the NTT workload (the MFMA transforms k_mf_ntt at N = 2^16),
# one rocprofv3 run per pass.
set -uo pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/nttpmc; mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run() {
  local tag=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/$O/$tag" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-power --workload ntt --batch 256 > $O/$tag.out 2> $O/$tag.err
  local rc=$?; echo "pmc $tag rc=$rc"; [ $rc -lt 124 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM
run sq3 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_I8 GRBM_GUI_ACTIVE
run tcc1 FETCH_SIZE
run tcc2 WRITE_SIZE
