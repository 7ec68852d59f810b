#!/bin/bash
# r06d: the fused ct-mul + rescale: its parity tests and the ct-mul lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_replays.py tests/test_gpu_boundary.py tests/test_gpu_multiproc.py tests/test_gpu_sharded_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
timeout -k 10 300 python3 bench.py --workload ctmul --ct-batch 128 --steps 10 --warmup 2 --no-cpu-baseline --no-power > $O/ctmul128_$i.json 2> $O/ctmul128_$i.err || { echo "ctmul rc=$?"; tail -5 $O/ctmul128_$i.err; exit 1; }
head -c 200 $O/ctmul128_$i.json; echo
done
timeout -k 10 400 python3 bench.py --workload ctmul --ct-batch 1024 --steps 4 --warmup 1 > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 rc=$?"; tail -5 $O/cfg4.err; exit 1; }
head -c 200 $O/cfg4.json; echo
timeout -k 10 400 python3 bench.py --workload ctmul --log-n 14 --limbs 8 --ct-batch 1024 --steps 10 --warmup 2 > $O/cfg3.json 2> $O/cfg3.err || { echo "cfg3 rc=$?"; tail -5 $O/cfg3.err; exit 1; }
head -c 200 $O/cfg3.json; echo
