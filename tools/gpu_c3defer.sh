# Round-5 check of the deferred GROUP BY count: the -m gpu suite, then the C3
# line and the per-query overhead tool twice.  Results: gpurun_out/c3d/.
set -o pipefail
mkdir -p gpurun_out/c3d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c3d/gpu_tests.log 2>&1 || exit 11
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 5 --no-cpu --extra "" > gpurun_out/c3d/c3_$rep.json 2> gpurun_out/c3d/c3_$rep.err || exit 12
  timeout -k 10 100 python tools/query_overhead.py 1000000 > gpurun_out/c3d/qo_$rep.json 2> gpurun_out/c3d/qo_$rep.err || exit 14
done
echo C3D_OK
