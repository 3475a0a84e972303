set -o pipefail
mkdir -p /root/repo/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/c3 -o c3 -- python3 /root/repo/bench.py --config c3 --steps 5 --warmup 1 --no-cpu > /root/repo/gpurun_out/pmc_c3.log 2>&1 || exit 21
SHAPES=sel,sel3 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/self -o self -- python3 /root/repo/tools/shape_bench.py 1000000000 > /root/repo/gpurun_out/pmc_self.log 2>&1 || exit 22
SHAPES=sel,sel3 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/selw -o selw -- python3 /root/repo/tools/shape_bench.py 1000000000 > /root/repo/gpurun_out/pmc_selw.log 2>&1 || exit 23
