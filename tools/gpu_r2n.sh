set -o pipefail
mkdir -p gpurun_out/r2n
SWEEP_SQLS=c3 SWEEP_ROUNDS=5 SWEEP_VARIANTS=d2_g1,d2_g3,d2_g1+h2,d2_g2+h2,d2_g3+h2 timeout -k 10 400 python -u tools/sweep_group.py 1000000000 > gpurun_out/r2n/sweep.log 2>&1 || exit 11
MBX_GD_H=2 MBX_GD_VARIANT=d2_g1 timeout -k 10 300 python -u -m pytest tests/test_gpu_hotpath.py -x -q --timeout 120 --timeout-method thread -k "group or c3" > gpurun_out/r2n/tests_h2.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest tests/test_gpu_arrow.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2n/tests_arrow.log 2>&1 || exit 13
timeout -k 10 300 python bench.py --config c4 > gpurun_out/r2n/bench_c4.json 2> gpurun_out/r2n/bench_c4.err || exit 14
MBX_PREFAULT=0 timeout -k 10 300 python bench.py --config c4 > gpurun_out/r2n/bench_c4_noprefault.json 2>> gpurun_out/r2n/bench_c4.err || exit 15
