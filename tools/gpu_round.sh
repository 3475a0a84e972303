# Round evidence at head: -m gpu suite, smoke, the C2 / C3 / sel bench lines and
# their rocprofv3 kernel-trace summaries (gpurun_out/round/).
set -o pipefail
mkdir -p gpurun_out/round/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/round/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || exit 12
timeout -k 10 240 python bench.py > gpurun_out/round/bench_c2.json 2> gpurun_out/round/bench_c2.err || exit 13
timeout -k 10 240 python bench.py --config c3 > gpurun_out/round/bench_c3.json 2> gpurun_out/round/bench_c3.err || exit 14
timeout -k 10 300 python bench.py --config sel > gpurun_out/round/bench_sel.json 2> gpurun_out/round/bench_sel.err || exit 15
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/round/prof/c2 -o c2 -- python3 /root/repo/bench.py --steps 10 --no-cpu > /root/repo/gpurun_out/round/prof_c2.log 2>&1 || exit 16
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/round/prof/c3 -o c3 -- python3 /root/repo/bench.py --config c3 --steps 10 --no-cpu > /root/repo/gpurun_out/round/prof_c3.log 2>&1 || exit 17
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/round/prof/sel -o sel -- python3 /root/repo/bench.py --config sel --steps 10 --no-cpu > /root/repo/gpurun_out/round/prof_sel.log 2>&1 || exit 18
cd /root/repo
timeout -k 10 400 python bench.py --config c4 > gpurun_out/round/bench_c4.json 2> gpurun_out/round/bench_c4.err || exit 19
