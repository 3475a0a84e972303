# C3 HBM read traffic per group_direct launch (FETCH_SIZE pass of its own).
set -o pipefail
mkdir -p /root/repo/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/c3 -o c3 -- python3 /root/repo/bench.py --config c3 --steps 5 --warmup 1 --no-cpu > /root/repo/gpurun_out/pmc_c3.log 2>&1 || exit 21
