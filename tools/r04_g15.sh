# round-4 head, multi-shard and C4 evidence: 2- and 8-shard in-library lines,
# the per-query shard overhead split, and C4 (adaptive 8 MB read-back).
set -o pipefail
mkdir -p gpurun_out/g15
for c in c2 c5 c3; do
  timeout -k 10 240 python bench.py --shards-per-gpu 2 --config $c --no-cpu > gpurun_out/g15/bench_${c}_s2.json 2> gpurun_out/g15/bench_${c}_s2.err || exit 171
done
timeout -k 10 240 python bench.py --shards-per-gpu 8 --config c2 --no-cpu > gpurun_out/g15/bench_c2_s8.json 2> gpurun_out/g15/bench_c2_s8.err || exit 172
timeout -k 10 240 python tools/shard_overhead.py --iters 1000 > gpurun_out/g15/shard_overhead.json 2> gpurun_out/g15/shard_overhead.err || exit 173
timeout -k 10 400 python bench.py --config c4 > gpurun_out/g15/bench_c4.json 2> gpurun_out/g15/bench_c4.err || exit 174
echo G15_OK
