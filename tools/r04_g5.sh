# storer partial passes: selection / NULL-able / sharded tests, selection
# shapes (kernel medians), rocprof trace + WRITE_SIZE of seln_out, and the
# 8 MB read-back per method.
set -o pipefail
mkdir -p gpurun_out/g5
R=${GRAFT_REPO_ROOT:-$PWD}
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_nullable.py tests/test_gpu_ctas_adopt.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g5/tests.log 2>&1 || exit 71
NULLABLE=1 REPS=7 SHAPES=sel,selv,sel2,sel3,seln_pred,seln_out,seln_both,compact,compact2 timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/g5/shapes.log 2> gpurun_out/g5/shapes.err || exit 72
( cd /tmp && export TMPDIR=/tmp NULLABLE=1 SHAPES=seln_out REPS=6 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g5/trace -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g5/trace.log 2>&1 ) || exit 73
( cd /tmp && export TMPDIR=/tmp NULLABLE=1 SHAPES=seln_out REPS=4 && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/g5/w -o w -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g5/pmc.log 2>&1 ) || exit 74
for mode in "" 0 1 2; do
  if [ -n "$mode" ]; then export MBX_EXPERIMENTS=1 MBX_LINK_MID_MODE=$mode; fi
  timeout -k 10 120 python -u tools/c4_mid_probe.py >> gpurun_out/g5/c4mid.jsonl 2>> gpurun_out/g5/c4mid.err || exit 75
done
echo G5_OK
