set -o pipefail
mkdir -p gpurun_out/r2q
JIT_WAIT=3 GRID='[{}, {"MBX_FM_BLOCKS_PER_CU":1}, {"MBX_FM_BLOCKS_PER_CU":2}, {"MBX_FM_BLOCKS_PER_CU":3}, {"MBX_FM_BLOCKS_PER_CU":4}, {"MBX_FM_DEPTH":3}, {"MBX_FM_DEPTH":4}, {"MBX_FM_BLOCKS_PER_CU":1,"MBX_FM_DEPTH":4}, {"MBX_FM_BLOCKS_PER_CU":2,"MBX_FM_DEPTH":3}]' timeout -k 10 400 python -u tools/sweep_env.py 1000000000 filter_multi filter_multi3 > gpurun_out/r2q/fm.log 2>&1 || exit 11
JIT_WAIT=3 GRID='[{}, {"MBX_JIT":"0"}, {"MBX_JIT":"0","MBX_GD_VARIANT":"d2_g3"}, {"MBX_JIT":"0","MBX_GD_VARIANT":"d3_g1"}, {"MBX_JIT":"0","MBX_GD_VARIANT":"d4_g1"}]' timeout -k 10 400 python -u tools/sweep_env.py 1000000000 c3_where c3_where2 > gpurun_out/r2q/gw.log 2>&1 || exit 12
