# HBM traffic of the NULL-able-column kernels (filter_multi_lds with validity,
# compact_validity): one FETCH_SIZE and one WRITE_SIZE pass, 1e9 rows.
set -o pipefail
mkdir -p /root/repo/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
export NULLABLE=1 SHAPES=c2n,seln_out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/nf -o nf -- python3 /root/repo/tools/shape_bench.py 1000000000 > /root/repo/gpurun_out/pmc_nf.log 2>&1 || exit 31
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /root/repo/gpurun_out/pmc/nw -o nw -- python3 /root/repo/tools/shape_bench.py 1000000000 > /root/repo/gpurun_out/pmc_nw.log 2>&1 || exit 32
