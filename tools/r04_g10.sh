# ballot-mode validity for the 8-loader NULL-able output (MBX_SR_VBALL=1):
# the NULL-able / selection / CTAS / extremes tests with it on (any failure
# stops the run), the shapes on vs off, the role split, rocprof trace and
# WRITE_SIZE / FETCH_SIZE of seln_out with it on, then the full -m gpu suite
# and the headline bench line with the defaults.
set -o pipefail
mkdir -p gpurun_out/g10
R=${GRAFT_REPO_ROOT:-$PWD}
MBX_SR_VBALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_nullable.py tests/test_gpu_compact.py tests/test_gpu_ctas_adopt.py tests/test_gpu_extremes.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g10/tests_vball.log 2>&1 || exit 121
for vb in 1 0 1 0; do
  echo "== VBALL=$vb" >> gpurun_out/g10/ab.log
  MBX_EXPERIMENTS=1 MBX_SR_VBALL=$vb NULLABLE=1 REPS=6 SHAPES=seln_out,seln_pred,seln_both timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g10/ab.log 2>&1 || exit 122
done
MBX_EXPERIMENTS=1 MBX_SR_VBALL=1 MBX_SR_DEBUG=1 NULLABLE=1 REPS=2 SHAPES=seln_out timeout -k 10 200 python -u tools/shape_bench.py 1000000000 > gpurun_out/g10/dbg.log 2>&1 || exit 123
( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 MBX_SR_VBALL=1 NULLABLE=1 SHAPES=seln_out REPS=6 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g10/trace -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g10/trace.log 2>&1 ) || exit 124
( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 MBX_SR_VBALL=1 NULLABLE=1 SHAPES=seln_out REPS=4 && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/g10/w -o w -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g10/pmc.log 2>&1 ) || exit 125
( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 MBX_SR_VBALL=1 NULLABLE=1 SHAPES=seln_out REPS=4 && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/g10/f -o f -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g10/pmcf.log 2>&1 ) || exit 126
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g10/gpu_tests.log 2>&1 || exit 127
timeout -k 10 300 python bench.py > gpurun_out/g10/bench_c2.json 2> gpurun_out/g10/bench_c2.err || exit 128
echo G10_OK
