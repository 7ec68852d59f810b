#!/usr/bin/env bash
# Power of back-to-back i8 MFMAs / v_mad_i64_i32 / add+xor on random operands
# (tools/openergy.hip), rocm-smi sampled while each mode runs.
set -uo pipefail
O=gpurun_out/r04
mkdir -p $O
for mode in idle mfma mad64 add32; do
  ( for k in $(seq 1 12); do rocm-smi -d 0 --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk clock level" ; sleep 0.25; done ) > $O/openergy_$mode.smi &
  sp=$!
  timeout -k 10 60 ./tools/bin/openergy $mode 6 > $O/openergy_$mode.txt 2>&1
  wait $sp
  echo "== $mode"; cat $O/openergy_$mode.txt
  grep "Package Power" $O/openergy_$mode.smi | awk '{print $NF}' | tail -8 | tr '\n' ' '; echo
  grep "sclk" $O/openergy_$mode.smi | tail -3 | tr '\n' ' '; echo
done
