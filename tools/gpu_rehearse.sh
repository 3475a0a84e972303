set -o pipefail
cd /root/repo
for c in c2 c5 c3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951${#c} bench.py --gpus 2 --config $c --dist-backend gloo --no-cpu --steps 10 > gpurun_out/rehearse_n2_$c.json 2> gpurun_out/rehearse_n2_$c.err || exit 31
done
