set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmcsq
for c in c3h:100000 c3s:1000000; do
  cfg=${c%%:*}; g=${c##*:}
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/pmcsq/$cfg -o sq -- python3 $R/bench.py --config $cfg --groups $g --extra "" --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/pmcsq/$cfg.log 2>&1 ) || exit 5
done
echo ok
