set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu > gpurun_out/probe/bench_c3.log 2>&1 || exit 11
GRID='[{}]' timeout -k 10 400 python3 -u tools/sweep_env.py 1000000000 c3 c3_where > gpurun_out/probe/c3_sweep.log 2>&1 || exit 12
