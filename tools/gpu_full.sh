set -o pipefail
mkdir -p gpurun_out/prof
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 12
timeout -k 10 200 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 13
timeout -k 10 200 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 14
timeout -k 10 200 python bench.py --config c5 --rows 1250000000 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 15
timeout -k 10 300 python bench.py --config c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 16
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof/c2 -o c2 -- python3 /root/repo/bench.py --steps 10 --no-cpu > /root/repo/gpurun_out/prof_c2.log 2>&1 || exit 17
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof/c3 -o c3 -- python3 /root/repo/bench.py --config c3 --steps 10 --no-cpu > /root/repo/gpurun_out/prof_c3.log 2>&1 || exit 18
# the NULL-able shapes (filter_multi with validity, compact_validity), kernel trace
NULLABLE=1 SHAPES=c2n,c5n,seln_out timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof/nullable -o nullable -- python3 /root/repo/tools/shape_bench.py 1000000000 > /root/repo/gpurun_out/prof_nullable.log 2>&1 || exit 19
