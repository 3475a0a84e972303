# C3 placement: kernel time and translation counters of the group_direct
# launches with the C3 table alone vs allocated after the 8 GB C2 table
# (tools/c3_tlb_probe.py).  One counter set per rocprofv3 run.
set -o pipefail
mkdir -p gpurun_out/tlb
R=${GRAFT_REPO_ROOT:-$PWD}
for mode in alone after_c2; do
  timeout -k 10 200 python -u tools/c3_tlb_probe.py $mode 10 >> gpurun_out/tlb/times.jsonl 2>> gpurun_out/tlb/err.log || exit 31
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/gpurun_out/tlb/utcl1_$mode -o p -- python3 $R/tools/c3_tlb_probe.py $mode 6 >> $R/gpurun_out/tlb/pmc.log 2>&1 ) || exit 32
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/tlb/utcl2_$mode -o p -- python3 $R/tools/c3_tlb_probe.py $mode 6 >> $R/gpurun_out/tlb/pmc.log 2>&1 ) || exit 33
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_SERIALIZATION_STALL TCP_UTCL1_THRASHING_STALL --output-format csv -d $R/gpurun_out/tlb/stall_$mode -o p -- python3 $R/tools/c3_tlb_probe.py $mode 6 >> $R/gpurun_out/tlb/pmc.log 2>&1 ) || exit 34
done
echo TLB_OK
