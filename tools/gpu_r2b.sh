set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2b/compact_tests.log 2>&1 || exit 11
timeout -k 10 400 python -u tools/sweep_select.py > gpurun_out/r2b/sweep_select.log 2>&1 || exit 12
