set -o pipefail
mkdir -p gpurun_out/r2r
timeout -k 10 400 python -u -m pytest tests/test_gpu_hotpath.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2r/tests.log 2>&1 || exit 10
JIT_WAIT=3 SHAPES=c3,c3_where,c3_where2,filter_multi,multi_key timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/r2r/shapes.log 2>&1 || exit 11
