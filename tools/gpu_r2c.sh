set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c/compact_tests.log 2>&1 || exit 11
MBX_FK_CHUNK=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 120 --timeout-method thread -k "parity and 30000017 or parity and 4097" > gpurun_out/r2c/compact_tests_k8.log 2>&1 || exit 12
SWEEP_SQLS=sel,sel4 SWEEP_VARIANTS=count_first,bits,k8,k8_g1,fk_g1,fk_g2,fk_g1d4,cr_g1,cr_g1d6 timeout -k 10 400 python -u tools/sweep_select.py > gpurun_out/r2c/sweep_select.log 2>&1 || exit 13
