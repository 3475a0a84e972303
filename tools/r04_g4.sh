# sharded tests (merge fast path) + shard overhead, C4 with the adaptive
# mid-size read-back, then the storer store-flavour A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_arrow.py tests/test_gpu_appender_c4.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_g4_tests.log 2>&1 || exit 61
timeout -k 10 240 python tools/shard_overhead.py --iters 1000 > gpurun_out/r04_shard_overhead2.json 2> gpurun_out/r04_shard_overhead2.err || exit 62
timeout -k 10 400 python bench.py --config c4 > gpurun_out/r04_bench_c4.json 2> gpurun_out/r04_bench_c4.err || exit 63
bash tools/r04_nt.sh > gpurun_out/r04_nt.log 2>&1 || exit 64
echo G4_OK
