set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2h/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2h/smoke.log 2>&1 || exit 12
timeout -k 10 200 python bench.py > gpurun_out/r2h/bench_c2.json 2> gpurun_out/r2h/bench_c2.err || exit 13
timeout -k 10 200 python bench.py --config c3 > gpurun_out/r2h/bench_c3.json 2> gpurun_out/r2h/bench_c3.err || exit 14
