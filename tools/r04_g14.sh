# merged two-range copy for sentinel-staged outputs only: selection /
# NULL-able / CTAS / extremes / hot-path tests, shapes COPY1=0 vs 2, the full
# -m gpu suite, smoke and the headline line with a rocprof trace.
set -o pipefail
mkdir -p gpurun_out/g14
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_nullable.py tests/test_gpu_ctas_adopt.py tests/test_gpu_extremes.py tests/test_gpu_hotpath.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g14/tests_sel.log 2>&1 || exit 161
for c in 0 2 0 2; do
  echo "== COPY1=$c" >> gpurun_out/g14/ab.log
  MBX_EXPERIMENTS=1 MBX_SR_COPY1=$c NULLABLE=1 REPS=7 SHAPES=sel,selv,seln_pred,seln_out timeout -k 10 300 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g14/ab.log 2>&1 || exit 162
done
STEPS=tests,smoke,bench,prof bash tools/gpu.sh > gpurun_out/g14/gpu_sh.log 2>&1 || exit 163
echo G14_OK
