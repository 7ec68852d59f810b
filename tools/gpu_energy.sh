#!/bin/bash
# Energy-model data (tools/energy_model.py): for each workload
# one bench run with its power probe (rocm-smi package power and sclk while
# the step keeps running, read-only) and three rocprofv3 --pmc passes of the
# same shape (SQ instruction counts, FETCH_SIZE, WRITE_SIZE), each pass its
# own run.  Output: gpurun_out/energy/<tag>.{json,err} and .../<tag>_{sq,fetch,write}/
mkdir -p gpurun_out/energy
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/energy
run() {  # run <tag> <lib|-> <bench args...>
  local tag=$1 lib=$2; shift 2
  local env=()
  [ "$lib" != "-" ] && env=(RNSNTT_LIB=$ROOT/toy-heaan-ckks_amd/lib/variants/librnsntt_$lib.so)
  echo "== $tag" >&2
  env "${env[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  local rc=$?; echo "bench $tag rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc
  for pass in "sq:SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES" \
              "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
    local name=${pass%%:*} ctrs=${pass#*:}
    env "${env[@]}" timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/${tag}_$name -o run -- \
      python3 bench.py --no-cpu-baseline --no-power --steps 2 --warmup 1 "$@" > $OUT/${tag}_$name.out 2> $OUT/${tag}_$name.err
    rc=$?; echo "pmc $tag $name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc
  done
}
if [ -n "$ONLY" ]; then  # ONLY="tag lib args...;tag lib args..." runs just those
  IFS=';' read -ra items <<< "$ONLY"
  for it in "${items[@]}"; do run $it; done
  exit 0
fi
run polymul - --steps 20 --warmup 3
run polymul_meas1 meas1 --steps 20 --warmup 3
run polymul_meas2 meas2 --steps 20 --warmup 3
run polymul_b256 - --batch 256 --steps 40 --warmup 3
run polymul_p30 - --prime-bits 30 --steps 20 --warmup 3
run ntt - --workload ntt --steps 20 --warmup 3
run pointwise - --workload pointwise --steps 20 --warmup 3
run copy - --workload copy --steps 20 --warmup 3
run ctmul - --workload ctmul --ct-batch 128 --steps 5 --warmup 1
run rotate - --workload rotate --rot-batch 8 --rot-keys shared --steps 3 --warmup 1
