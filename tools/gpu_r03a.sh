#!/bin/bash
# r03 check: GPU tests, then the bench lines VERDICT r02 asked for (config-4
# ct-mul at the 1024-pair batch, the engine's one-ciphertext call shape from
# a replayed graph, the u64 poly-mul and ct-mul shapes).  Each GPU step has
# its own time limit; a failing step stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -2 "gpurun_out/$name.out" >&2
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)" >&2
    tail -20 "gpurun_out/$name.err" >&2
    exit $rc
  fi
  return 0
}
if [ "${TESTS:-1}" = "1" ]; then
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
step ctmul_b1024 600 python bench.py --workload ctmul --ct-batch 1024 --steps 3 --warmup 1 --no-cpu-baseline
step ctmul_b1023 600 python bench.py --workload ctmul --ct-batch 1023 --steps 3 --warmup 1 --no-cpu-baseline
step ctmul_b1_graph 300 python bench.py --workload ctmul --ct-batch 1 --graph --steps 200 --warmup 5
step ctmul_b1_eager 300 python bench.py --workload ctmul --ct-batch 1 --steps 200 --warmup 5 --no-cpu-baseline
step rotate_b1_graph 300 python bench.py --workload rotate --rot-batch 1 --graph --steps 10 --warmup 2 --no-cpu-baseline
step rotate_b1_eager 300 python bench.py --workload rotate --rot-batch 1 --steps 10 --warmup 2 --no-cpu-baseline
step polymul_u64_horner 300 python bench.py --log-n 13 --limbs 7 --prime-bits 61 --batch 1024 --steps 20 --warmup 3 --no-power
step polymul_u64_n16 300 python bench.py --log-n 16 --limbs 16 --prime-bits 62 --batch 256 --steps 10 --warmup 2 --no-power
step ctmul_u64_horner 300 python bench.py --workload ctmul --log-n 13 --limbs 7 --prime-bits 61 --ct-batch 128 --steps 5 --warmup 1
step ctmul_u64_n16 600 python bench.py --workload ctmul --log-n 16 --limbs 16 --prime-bits 62 --ct-batch 64 --steps 3 --warmup 1 --no-cpu-baseline
