set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 600 python -u -m pytest tests/test_c_harness.py tests/test_gpu_appender_c4.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2f/harness_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --config c4 > gpurun_out/r2f/bench_c4.json 2> gpurun_out/r2f/bench_c4.err || exit 12
