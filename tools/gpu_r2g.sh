set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 200 python -u tools/text_getter_bench.py > gpurun_out/r2g/text_getter.json 2> gpurun_out/r2g/text_getter.err || exit 11
timeout -k 10 200 python bench.py --config c1 > gpurun_out/r2g/bench_c1.json 2> gpurun_out/r2g/bench_c1.err || exit 12
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2g/gpu_tests.log 2>&1 || exit 13
