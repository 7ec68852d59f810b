set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--workload ctmul --ct-batch 4" AB_TAG=ct4 bash tools/ab.sh 2 base wreg || exit $?
BENCH_ARGS="--workload ctmul --ct-batch 2 --log-n 14 --limbs 8" AB_TAG=c3 bash tools/ab.sh 2 base wreg || exit $?
BENCH_ARGS="--workload ctmul --ct-batch 1 --log-n 14 --limbs 8" AB_TAG=c3b1 bash tools/ab.sh 2 base wreg || exit $?
BENCH_ARGS="--workload rotate --rot-batch 1" AB_TAG=rot1 bash tools/ab.sh 2 base wreg || exit $?
