#!/bin/bash
# Lists the PMC counters rocprofv3 offers on this GPU, then one --pmc pass
# of the default bench with the instruction-cache counters.
mkdir -p gpurun_out/icache
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 120 rocprofv3 -L > gpurun_out/icache/counters.txt 2>&1 || true
grep -o -E "SQC?_[A-Z0-9_]*(ICACHE|IFETCH|INST)[A-Z0-9_]*" gpurun_out/icache/counters.txt | sort -u > gpurun_out/icache/inst_counters.txt
cat gpurun_out/icache/inst_counters.txt
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES} --output-format csv -d "$ROOT/gpurun_out/icache/p1" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/icache/p1.out 2>&1 || { tail -20 gpurun_out/icache/p1.out; exit 1; }
if [ -n "${PMC2:-}" ]; then
timeout -s KILL 120 rocprofv3 --pmc $PMC2 --output-format csv -d "$ROOT/gpurun_out/icache/p2" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-power > gpurun_out/icache/p2.out 2>&1 || { tail -20 gpurun_out/icache/p2.out; exit 1; }
fi
