# C3 placement, one more pass: L2 hit / miss counts of the group_direct
# launches with the C3 table alone vs after the C2 table, and the round-3
# layout probe on this box.
set -o pipefail
mkdir -p gpurun_out/g16
R=${GRAFT_REPO_ROOT:-$PWD}
for mode in alone after_c2; do
  timeout -k 10 200 python -u tools/c3_tlb_probe.py $mode 10 >> gpurun_out/g16/times.jsonl 2>> gpurun_out/g16/err.log || exit 181
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/g16/tcc_$mode -o p -- python3 $R/tools/c3_tlb_probe.py $mode 6 >> $R/gpurun_out/g16/pmc.log 2>&1 ) || exit 182
done
timeout -k 10 300 python tools/c3_layout_probe.py > gpurun_out/g16/c3_layout.json 2> gpurun_out/g16/c3_layout.err || exit 183
echo G16_OK
