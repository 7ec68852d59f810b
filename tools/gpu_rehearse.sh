#!/bin/bash
# N-rank rehearsal of the driver's multi-GPU bench on ONE device
# (BENCH_ONE_DEVICE=1: every rank on device 0, the data-path joins over gloo
# because RCCL needs one GPU per rank).  Exercises the torchrun launch, the
# per-rank shards through the current kernels, the max-over-ranks timing and
# the N-rank parity spot check.  Output: gpurun_out/rehearse_*.json
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp BENCH_ONE_DEVICE=1
run() {  # run <name> <seconds> <bench args...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python bench.py --no-cpu-baseline --no-power "$@" > gpurun_out/rehearse_$name.json 2> gpurun_out/rehearse_$name.err || { echo "$name rc=$?" >&2; tail -20 gpurun_out/rehearse_$name.err >&2; exit 1; }
  echo "== $name $(head -c 200 gpurun_out/rehearse_$name.json)" >&2
}
run polymul_g8 400 --gpus 8 --steps 10 --warmup 2
run polymul_g2 300 --gpus 2 --steps 10 --warmup 2
run ctmul_g2_limb 400 --gpus 2 --workload ctmul --shard limb --steps 4 --warmup 1
run ctmul_g2_batch 400 --gpus 2 --workload ctmul --shard batch --steps 4 --warmup 1
run rotate_g8 500 --gpus 8 --workload rotate --steps 2 --warmup 1
