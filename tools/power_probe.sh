#!/bin/bash
# power_probe.sh [bench args...]: run a long bench in the background and
# sample board power, power cap and clocks (rocm-smi, read-only) while it
# runs -> gpurun_out/power_<tag>.log (is the poly-mul power-limited?).
mkdir -p gpurun_out
TAG=${TAG:-polymul}
LOG=gpurun_out/power_$TAG.log
rocm-smi --showpowercap --showmaxpower > $LOG 2>&1
echo "== idle" >> $LOG
rocm-smi --showpower --showclocks >> $LOG 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/power_$TAG.json 2> gpurun_out/power_$TAG.err &
PID=$!
sleep ${WAIT:-12}
for i in $(seq 1 ${SAMPLES:-8}); do
  echo "== sample $i $(date +%s.%N)" >> $LOG
  rocm-smi --showpower --showclocks >> $LOG 2>&1
  sleep 0.5
done
wait $PID
echo "bench rc=$?" >> $LOG
