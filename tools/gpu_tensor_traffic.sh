#!/bin/bash
# k_mf_tensor's traffic, temporary by temporary: PMC
# FETCH_SIZE / WRITE_SIZE passes of one 64-ct ct-mul chunk with the shipped
# library and with each measurement build (RNT_MF_TENSOR_MEAS=1..3, wrong
# results by design) that drops one temporary's round trip.  Summarise with
# tools/tensor_traffic.py.  Output: gpurun_out/ttraf/<variant>_{fetch,write}
set -o pipefail
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ttraf; mkdir -p $O
B="bench.py --workload ctmul --ct-batch 64 --steps 3 --warmup 1 --no-cpu-baseline --no-power --no-live-pmc"
for v in base tmeas1 tmeas2 tmeas3; do
  if [ $v = base ]; then lib=toy-heaan-ckks_amd/lib/librnsntt.so; else lib=toy-heaan-ckks_amd/lib/variants/librnsntt_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    RNSNTT_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${v}_$c -o run -- python3 $B > $O/${v}_$c.json 2> $O/${v}_$c.err || { echo "$v $c rc=$?"; tail -20 $O/${v}_$c.err; exit 1; }
  done
  echo "== $v done"
done
