set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_compact.py tests/test_gpu_sharded.py tests/test_gpu_arrow.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/probe/compact_tests.log 2>&1 || exit 12
NULLS_GRID=1,0 timeout -k 10 400 python3 -u tools/sel_null_probe.py 1000000000 > gpurun_out/probe/sel_null.log 2>&1 || exit 11
