set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_arrow.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/probe/arrow_tests.log 2>&1 || exit 11
timeout -k 10 400 python3 -u bench.py --config c4 > gpurun_out/probe/c4_bench.log 2>&1 || exit 13
