# SQ / LDS counters (PMC_SQ_SETS) or HBM bytes (PMC_HBM=1) of the partitioned GROUP BY lines,
# one rocprofv3 --pmc pass per counter set (PMC_CONFIGS = config:groups ...)
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmcsq
SETS=${PMC_SQ_SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
if [ -n "$PMC_HBM" ]; then SETS="FETCH_SIZE;WRITE_SIZE"; fi
for c in ${PMC_CONFIGS:-c3h:100000 c3s:1000000}; do
  cfg=${c%%:*}; g=${c##*:}
  IFS=';' read -ra SS <<< "$SETS"
  k=0
  for set in "${SS[@]}"; do
    k=$((k + 1))
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmcsq/${cfg}_$g/$k -o p -- python3 $R/bench.py --config $cfg --groups $g --extra "" --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/pmcsq/${cfg}_${g}_$k.log 2>&1 ) || exit 5
  done
done
echo ok
