# round-3 GPU pass: the -m gpu suite, the headline bench (C2 + C3/sel extras),
# the in-library multi-device rehearsal (2 shards on the one GPU) and the
# fixed per-query cost of the shard path.  Each GPU step has its own limit and
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-tests,bench,shards,overhead}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || exit 11
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 13
fi
if [[ $STEPS == *shards* ]]; then
  timeout -k 10 240 python bench.py --shards-per-gpu 2 --no-cpu > gpurun_out/bench_c2_s2.json 2> gpurun_out/bench_c2_s2.err || exit 14
  timeout -k 10 240 python bench.py --shards-per-gpu 2 --config c5 --no-cpu > gpurun_out/bench_c5_s2.json 2> gpurun_out/bench_c5_s2.err || exit 15
  timeout -k 10 240 python bench.py --shards-per-gpu 2 --config c3 --no-cpu > gpurun_out/bench_c3_s2.json 2> gpurun_out/bench_c3_s2.err || exit 16
fi
if [[ $STEPS == *overhead* ]]; then
  timeout -k 10 240 python tools/shard_overhead.py > gpurun_out/shard_overhead.json 2> gpurun_out/shard_overhead.err || exit 17
fi
if [[ $STEPS == *shapes* ]]; then
  NULLABLE=1 SHAPES=${SHAPES:-seln_out,seln_pred,seln_both,sel,compact,compact2} timeout -k 10 300 python tools/shape_bench.py ${SHAPE_ROWS:-1000000000} > gpurun_out/shapes.json 2> gpurun_out/shapes.err || exit 18
fi
if [[ $STEPS == *prof* ]]; then
  mkdir -p gpurun_out/prof
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_c2.log 2>&1 ) || exit 19
fi
if [[ $STEPS == *c4* ]]; then
  timeout -k 10 300 python bench.py --config c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 20
  MBX_EXPERIMENTS=1 MBX_LINK_MIN=${LINK_MIN:-2097152} timeout -k 10 300 python bench.py --config c4 > gpurun_out/bench_c4_link.json 2> gpurun_out/bench_c4_link.err || exit 21
fi
echo ALL_OK
