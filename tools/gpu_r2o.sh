set -o pipefail
mkdir -p gpurun_out/r2o

MBX_SR_MIN_ROWS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 120 --timeout-method thread -k "not runs_the_hip" > gpurun_out/r2o/tests_min0.log 2>&1 || exit 11
MBX_SR_MIN_ROWS=0 GRID='[{}, {"MBX_SR_DEPTH":3}, {"MBX_SR_DEPTH":6}, {"MBX_SR_S":1}, {"MBX_SR_S":4}, {"MBX_SR_DEPTH":3,"MBX_SR_S":1}, {"MBX_SR_H":2,"MBX_SR_DEPTH":2}, {"MBX_SR_NL":4}, {"MBX_SR_NL":4,"MBX_SR_NARROW":0}]' timeout -k 10 400 python -u tools/sweep_rounds.py 1000000000 sel > gpurun_out/r2o/sweep.log 2>gpurun_out/r2o/sweep.err || exit 12
timeout -k 10 300 python bench.py --config sel > gpurun_out/r2o/bench_sel.json 2> gpurun_out/r2o/bench_sel.err || exit 13
