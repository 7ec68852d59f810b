#!/bin/bash
# The round's bench lines: default poly-mul, ct-mul (config 4), rotation
# (config 5: power-of-two offsets with per-offset keys, one ciphertext, and
# the every-offset sweep with one resident key).  Output: gpurun_out/bench_*.json
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <seconds> <bench args...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err || exit $?
  echo "== $name $(head -c 160 gpurun_out/bench_$name.json)" >&2
}
run polymul 300 --steps 20 --warmup 3
run ctmul 300 --workload ctmul --ct-batch 128 --steps 10 --warmup 2
run rotate 300 --workload rotate --rot-batch 8 --steps 3 --warmup 1
run rotate_b1 300 --workload rotate --rot-batch 1 --steps 5 --warmup 1
run rotate_all 400 --workload rotate --rot-offsets all --rot-batch 1 --steps 1 --warmup 0
