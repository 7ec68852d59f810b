set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r06a/pytest.log; exit 1; }
tail -2 gpurun_out/r06a/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r06a/smoke.log; exit 1; }
tail -1 gpurun_out/r06a/smoke.log
tools/gpu_headline.sh
