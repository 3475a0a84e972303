set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hotpath.py tests/test_gpu_nullable.py tests/test_gpu_sharded.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/probe/fm_tests.log 2>&1 || exit 11
GRID='[{}, {"MBX_FM_BLOCKS_PER_CU": 3}, {"MBX_FM_BLOCKS_PER_CU": 1}, {"MBX_FM_VARIANT": "generic"}]' timeout -k 10 400 python3 -u tools/sweep_env.py 1000000000 filter_multi filter_multi3 filter_mm filter_cnt2 filter_wide > gpurun_out/probe/fm_sweep.log 2>&1 || exit 12
NULLABLE=1 GRID='[{}, {"MBX_FM_BLOCKS_PER_CU": 3}, {"MBX_FM_BLOCKS_PER_CU": 1}, {"MBX_FM_VARIANT": "generic"}]' timeout -k 10 300 python3 -u tools/sweep_env.py 1000000000 c2n c5n c5n_sumv > gpurun_out/probe/fm_sweep_nullable.log 2>&1 || exit 13
