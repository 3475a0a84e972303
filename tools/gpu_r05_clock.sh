set -o pipefail
mkdir -p gpurun_out/r05
R=$PWD
DUCKDB_MB_AMD_LIB=$R/duckdb.mbt_amd/libduckdb_mb_amd_clk.so timeout -k 10 300 python -u tools/c3_clock.py 15 > gpurun_out/r05/c3_clock.jsonl 2> gpurun_out/r05/c3_clock.err || exit 31
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r05/grbm -o grbm -- python3 $R/tools/c3_clock.py pmc 15 > $R/gpurun_out/r05/grbm.log 2>&1 ) || exit 32
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests.log 2>&1 || exit 33
echo DONE
