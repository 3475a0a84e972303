set -o pipefail
mkdir -p gpurun_out/r2m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2m/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2m/smoke.log 2>&1 || exit 12
