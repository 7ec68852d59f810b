#!/bin/bash
# Config-sized bench lines: config 4 at its 1024-ciphertext batch, config 5
# over every slot offset 1..N/2-1 with one resident key (SURVEY 8d sweep 2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload ctmul --ct-batch 1024 --steps 2 --warmup 1 > gpurun_out/bench_ctmul_1024.json 2> gpurun_out/bench_ctmul_1024.err || exit $?
timeout -k 10 500 python bench.py --workload rotate --rot-offsets all --rot-batch 1 --steps 1 --warmup 0 > gpurun_out/bench_rotate_all.json 2> gpurun_out/bench_rotate_all.err || exit $?
