# merged two-range storer copy (8 loaders, one output): selection / NULL-able
# / CTAS / extremes / sharded / fixture tests first (a failure stops the run),
# then shapes merged (COPY1=0) vs per-range (COPY1=2) alternated, the full
# -m gpu suite and the headline line.
set -o pipefail
mkdir -p gpurun_out/g13
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_nullable.py tests/test_gpu_ctas_adopt.py tests/test_gpu_extremes.py tests/test_gpu_hotpath.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g13/tests_sel.log 2>&1 || exit 151
for c in 0 2 0 2; do
  echo "== COPY1=$c" >> gpurun_out/g13/ab.log
  MBX_EXPERIMENTS=1 MBX_SR_COPY1=$c NULLABLE=1 REPS=7 SHAPES=sel,selv,seln_pred,seln_out,compact timeout -k 10 300 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g13/ab.log 2>&1 || exit 152
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g13/gpu_tests.log 2>&1 || exit 153
timeout -k 10 300 python bench.py > gpurun_out/g13/bench_c2.json 2> gpurun_out/g13/bench_c2.err || exit 154
echo G13_OK
