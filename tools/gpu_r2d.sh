set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d/sharded_tests.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d/gpu_tests.log 2>&1 || exit 12
