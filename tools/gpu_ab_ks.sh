set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.out 2>&1 || { tail -30 gpurun_out/pytest_gpu.out; exit 1; }
tail -2 gpurun_out/pytest_gpu.out
BENCH_ARGS="--workload ctmul --ct-batch 128" AB_TAG=ct bash tools/ab.sh 3 base old || exit $?
BENCH_ARGS="--workload rotate --rot-batch 8" AB_TAG=rot bash tools/ab.sh 2 base old || exit $?
