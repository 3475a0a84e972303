set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2e/native_tests.log 2>&1 || exit 11
timeout -k 10 200 python -u tools/query_overhead.py > gpurun_out/r2e/query_overhead.json 2> gpurun_out/r2e/query_overhead.err || exit 12
