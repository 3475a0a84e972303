set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1 || exit 12
timeout -k 10 200 python bench.py > gpurun_out/r2a/bench_c2.json 2> gpurun_out/r2a/bench_c2.err || exit 13
timeout -k 10 200 python bench.py --config c3 > gpurun_out/r2a/bench_c3.json 2> gpurun_out/r2a/bench_c3.err || exit 14
nproc > gpurun_out/r2a/host.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/r2a/host.txt; lscpu >> gpurun_out/r2a/host.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r2a/host.txt 2>&1 || true
timeout -k 10 300 python bench.py --gpus 2 --config c5 --dist-backend gloo --rows 500000000 --steps 10 > gpurun_out/r2a/bench_c5_n2_gloo.json 2> gpurun_out/r2a/bench_c5_n2_gloo.err || exit 15
