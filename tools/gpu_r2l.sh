set -o pipefail
mkdir -p gpurun_out/r2l/prof
timeout -k 10 300 python bench.py --config sel > gpurun_out/r2l/bench_sel.json 2> gpurun_out/r2l/bench_sel.err || exit 11
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r2l/prof/sel -o sel -- python3 /root/repo/bench.py --config sel --steps 10 --no-cpu > /root/repo/gpurun_out/r2l/prof_sel.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /root/repo/gpurun_out/r2l/pmc/self -o self -- python3 /root/repo/bench.py --config sel --steps 5 --warmup 1 --no-cpu > /root/repo/gpurun_out/r2l/pmc_self.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /root/repo/gpurun_out/r2l/pmc/selw -o selw -- python3 /root/repo/bench.py --config sel --steps 5 --warmup 1 --no-cpu > /root/repo/gpurun_out/r2l/pmc_selw.log 2>&1 || exit 14
