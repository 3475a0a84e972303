# whole-pass storer loops restored + no-wait control stores + per-instance
# zone-map role: full -m gpu suite, smoke, selection shapes with the role
# split, the headline bench line, C4.
set -o pipefail
mkdir -p gpurun_out/g9
STEPS=tests,smoke bash tools/gpu.sh > gpurun_out/g9/gpu_sh.log 2>&1 || exit 111
NULLABLE=1 REPS=7 SHAPES=sel,selv,sel2,sel3,seln_pred,seln_out,seln_both,compact,compact2 timeout -k 10 300 python -u tools/shape_bench.py 1000000000 > gpurun_out/g9/shapes.log 2> gpurun_out/g9/shapes.err || exit 112
for s in seln_out seln_pred sel; do
  echo "== $s" >> gpurun_out/g9/dbg.log
  MBX_EXPERIMENTS=1 MBX_SR_DEBUG=1 NULLABLE=1 REPS=2 SHAPES=$s timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g9/dbg.log 2>&1 || exit 113
done
timeout -k 10 300 python bench.py > gpurun_out/g9/bench_c2.json 2> gpurun_out/g9/bench_c2.err || exit 114
timeout -k 10 400 python bench.py --config c4 > gpurun_out/g9/bench_c4.json 2> gpurun_out/g9/bench_c4.err || exit 115
echo G9_OK
