# Round-4 probes: C3 step trace, C3 placement counters, 8 MB read-back
# variants, shard overhead split, in-library 2-shard / gloo-vote / sel lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/c3_step_trace.py > gpurun_out/r04_c3_trace.json 2> gpurun_out/r04_c3_trace.err || exit 40
timeout -k 10 200 python tools/c3_step_trace.py alone > gpurun_out/r04_c3_trace_alone.json 2>> gpurun_out/r04_c3_trace.err || exit 40
timeout -k 10 200 ./tools/link8_probe 8 100 > gpurun_out/r04_link8.log 2>&1 || exit 42
timeout -k 10 240 python tools/shard_overhead.py --iters 1000 > gpurun_out/r04_shard_overhead.json 2> gpurun_out/r04_shard_overhead.err || exit 43
bash tools/r04_tlb.sh > gpurun_out/r04_tlb.log 2>&1 || exit 41
bash tools/r04_g2.sh || exit 44
echo G3_OK
