# per-role cycle split (MBX_SR_DEBUG=1) of the NULL-able output shape vs its
# NULL-free twin and sel on one box; selection tests; 8 MB read-back with
# block-wise adaptive trials.
set -o pipefail
mkdir -p gpurun_out/g7
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_nullable.py tests/test_gpu_ctas_adopt.py tests/test_gpu_extremes.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g7/tests.log 2>&1 || exit 91
for s in seln_out seln_pred sel selv; do
  echo "== $s" >> gpurun_out/g7/dbg.log
  MBX_EXPERIMENTS=1 MBX_SR_DEBUG=1 NULLABLE=1 REPS=3 SHAPES=$s timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g7/dbg.log 2>&1 || exit 92
done
NULLABLE=1 REPS=7 SHAPES=sel,selv,seln_pred,seln_out timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/g7/shapes.log 2> gpurun_out/g7/shapes.err || exit 93
for mode in "" 0 1 2; do
  if [ -n "$mode" ]; then export MBX_EXPERIMENTS=1 MBX_LINK_MID_MODE=$mode; fi
  timeout -k 10 120 python -u tools/c4_mid_probe.py >> gpurun_out/g7/c4mid.jsonl 2>> gpurun_out/g7/c4mid.err || exit 95
done
echo G7_OK
