#!/bin/bash
# Headline evidence from ONE lease: the default bench
# line (with its live PMC passes and power/sclk probe), then a rocprofv3
# kernel-trace --stats pass of the same command (its own power/sclk probe),
# then an SQ counter pass -- all on the same box, each step under its own
# limit.  Summarise with tools/headline_summary.py gpurun_out/headline <tag>.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/headline; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-pmc ${BENCH_ARGS:-} > $O/trace.json 2> $O/trace.err || { echo "trace rc=$?"; tail -20 $O/trace.err; exit 1; }
head -c 300 $O/trace.json; echo
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-power --no-live-pmc ${BENCH_ARGS:-} > $O/sq.json 2> $O/sq.err || { echo "sq rc=$?"; tail -20 $O/sq.err; exit 1; }
echo done
