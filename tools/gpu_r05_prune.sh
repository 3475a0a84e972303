# Round 5, after pruning the measured-slower variants: the whole -m gpu suite,
# smoke, and the headline bench (C2 + C3/sel extras) with its rocprof summary.
set -o pipefail
mkdir -p gpurun_out/r05p
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p/gpu_tests.log 2>&1 || exit 41
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05p/smoke.log 2>&1 || exit 42
timeout -k 10 300 python bench.py > gpurun_out/r05p/bench_c2.json 2> gpurun_out/r05p/bench_c2.err || exit 43
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05p/prof -o c2 -- python3 $R/bench.py --steps 10 --no-cpu > $R/gpurun_out/r05p/prof_c2.log 2>&1 ) || exit 44
echo DONE
