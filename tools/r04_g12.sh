# ballot pack v2 (word map + compress): NULL-able / selection tests with
# MBX_SR_VBALL=1 (a failure stops the run), then seln_out / seln_pred with it
# on vs off alternated, and a rocprof kernel trace with it on.
set -o pipefail
mkdir -p gpurun_out/g12
R=${GRAFT_REPO_ROOT:-$PWD}
MBX_SR_VBALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_nullable.py tests/test_gpu_compact.py tests/test_gpu_ctas_adopt.py tests/test_gpu_extremes.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g12/tests_vball.log 2>&1 || exit 141
for vb in 1 0 1 0; do
  echo "== VBALL=$vb" >> gpurun_out/g12/ab.log
  MBX_EXPERIMENTS=1 MBX_SR_VBALL=$vb NULLABLE=1 REPS=7 SHAPES=seln_out,seln_pred timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g12/ab.log 2>&1 || exit 142
done
( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 MBX_SR_VBALL=1 NULLABLE=1 SHAPES=seln_out REPS=6 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g12/trace -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/g12/trace.log 2>&1 ) || exit 143
echo G12_OK
