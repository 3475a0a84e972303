# Round-5 A/B of the C2 emit folded into filter_agg_lds (HISTORY.md, Round 5): the
# build under test had MBX_FA_NOFUSE (experiments only) to switch the fold off; the fold
# was reverted after this A/B, so on the current tree both modes run the same code.
set -o pipefail
mkdir -p gpurun_out/fuse
timeout -k 10 600 python -u -m pytest tests/test_gpu_hotpath.py tests/test_gpu_fixtures.py tests/test_gpu_sharded.py tests/test_gpu_rccl_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fuse/tests.log 2>&1 || exit 11
for rep in 1 2 3; do
  for m in fuse nofuse; do
    if [ $m = nofuse ]; then X="MBX_EXPERIMENTS=1 MBX_FA_NOFUSE=1"; else X=""; fi
    env $X timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --extra "" > gpurun_out/fuse/c2_${m}_$rep.json 2> gpurun_out/fuse/c2_${m}_$rep.err || exit 12
    env $X timeout -k 10 200 python bench.py --config c5 --steps 100 --warmup 10 --no-cpu --extra "" > gpurun_out/fuse/c5_${m}_$rep.json 2> gpurun_out/fuse/c5_${m}_$rep.err || exit 13
    env $X timeout -k 10 100 python tools/query_overhead.py 1000000 > gpurun_out/fuse/qo_${m}_$rep.json 2> gpurun_out/fuse/qo_${m}_$rep.err || exit 14
  done
done
echo AB_OK
