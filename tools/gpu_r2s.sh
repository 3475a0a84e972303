set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 400 python -u -m pytest tests/test_gpu_hotpath.py tests/test_gpu_nullable.py tests/test_gpu_sharded.py tests/test_gpu_fixtures.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s/tests.log 2>&1 || exit 10
NULLABLE=1 GRID='[{}, {"MBX_FM_VARIANT":"generic"}, {"MBX_FM_DEPTH":3}, {"MBX_FM_BLOCKS_PER_CU":2}, {"MBX_FM_BLOCKS_PER_CU":4}]' timeout -k 10 500 python -u tools/sweep_env.py 1000000000 filter_multi filter_multi3 filter_mm c2n c5n c5n_sumv > gpurun_out/r2s/fm.log 2>&1 || exit 11
