#!/bin/bash
# BASELINE configs 3 and 4 as stated: ct x ct + relin +
# rescale at 2^14 x 8 and at 2^16 x 16, 1024 ciphertext pairs per step, each
# line with a rocprofv3 kernel-trace --stats pass of the same command, and
# the config-4 1024-ct oracle test.  Output: gpurun_out/cfg34/
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/cfg34; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "1024_ct" --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run <name> <bench args...>
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc=$?"; tail -20 $O/$name.err; exit 1; }
  head -c 240 $O/$name.json; echo
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$name -o run -- python3 bench.py --no-cpu-baseline --no-power "$@" > $O/trace_$name.json 2> $O/trace_$name.err || { echo "trace $name rc=$?"; tail -20 $O/trace_$name.err; exit 1; }
}
run cfg3 --workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 10 --warmup 2
run cfg4 --workload ctmul --ct-batch 1024 --steps 4 --warmup 1
echo done
