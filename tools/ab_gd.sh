# A/B of the C3 GROUP BY flush: per-workgroup records + group_partials_compact
# (default) against the global-atomic flush (MBX_EXPERIMENTS=1
# MBX_GD_ATOMIC_FLUSH=1); GROUP BY GPU tests first.  Results: gpurun_out/gd/.
set -o pipefail
mkdir -p gpurun_out/gd
timeout -k 10 700 python -u -m pytest ${GD_TESTS:-tests/test_gpu_hotpath.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gd/tests.log 2>&1 || exit 11
for rep in 1 2 3; do
  for m in parts atomic; do
    if [ $m = atomic ]; then X="MBX_EXPERIMENTS=1 MBX_GD_ATOMIC_FLUSH=1"; else X=""; fi
    env $X timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 5 --no-cpu --extra "" > gpurun_out/gd/c3_${m}_$rep.json 2> gpurun_out/gd/c3_${m}_$rep.err || exit 12
    env $X timeout -k 10 100 python tools/query_overhead.py 1000000 > gpurun_out/gd/qo_${m}_$rep.json 2> gpurun_out/gd/qo_${m}_$rep.err || exit 14
  done
done
echo AB_OK
