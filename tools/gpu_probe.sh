set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_hotpath.py -x -q -m gpu -k "calibrate or filter_multi" --timeout 120 --timeout-method thread > gpurun_out/probe/cal_tests.log 2>&1 || exit 11
