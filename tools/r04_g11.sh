# round-4 head: -m gpu, smoke, the headline line, its rocprof kernel trace,
# and the selection shapes.
set -o pipefail
mkdir -p gpurun_out/g11
STEPS=tests,smoke,bench,prof bash tools/gpu.sh > gpurun_out/g11/gpu_sh.log 2>&1 || exit 131
NULLABLE=1 REPS=7 SHAPES=sel,selv,seln_pred,seln_out,compact timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/g11/shapes.log 2> gpurun_out/g11/shapes.err || exit 132
echo G11_OK
