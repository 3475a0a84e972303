set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u bench.py --gpus 1 --shards-per-gpu 2 --steps 5 --warmup 2 --extra "" --no-cpu --config c5 > gpurun_out/r04_b_inlib2.json 2> gpurun_out/r04_b_inlib2.err &&
timeout -k 10 240 python -u bench.py --gpus 1 --shards-per-gpu 2 --steps 5 --warmup 2 --extra "" --no-cpu --config c3 > gpurun_out/r04_b_inlib2_c3.json 2> gpurun_out/r04_b_inlib2_c3.err &&
timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --config c5 --no-cpu > gpurun_out/r04_b_vote2.json 2> gpurun_out/r04_b_vote2.err &&
timeout -k 10 240 python -u bench.py --config sel --steps 5 --warmup 2 --no-cpu > gpurun_out/r04_b_sel.json 2> gpurun_out/r04_b_sel.err
echo rc=$?
