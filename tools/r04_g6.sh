# storer zone map compiled for 4-loader kernels only (8-loader NULL-able
# instances 128 VGPRs + spills -> 109, none) + round counts in one LDS read:
# selection tests, shapes, rocprof trace of the NULL-able output shape, the
# 8 MB read-back with warm-up-free adaptive trials.
set -o pipefail
mkdir -p gpurun_out/g6
R=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_nullable.py tests/test_gpu_ctas_adopt.py tests/test_gpu_sharded.py tests/test_gpu_arrow.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g6/tests.log 2>&1 || exit 81
NULLABLE=1 REPS=7 SHAPES=sel,selv,sel2,sel3,seln_pred,seln_out,seln_both,compact,compact2 timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/g6/shapes.log 2> gpurun_out/g6/shapes.err || exit 82
( cd /tmp && export TMPDIR=/tmp NULLABLE=1 SHAPES=seln_out,sel REPS=6 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g6/trace -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g6/trace.log 2>&1 ) || exit 83
for mode in "" 0 1 2; do
  if [ -n "$mode" ]; then export MBX_EXPERIMENTS=1 MBX_LINK_MID_MODE=$mode; fi
  timeout -k 10 120 python -u tools/c4_mid_probe.py >> gpurun_out/g6/c4mid.jsonl 2>> gpurun_out/g6/c4mid.err || exit 85
done
echo G6_OK
